"""The rescue launch of segment-shared windows (csrc/rescue.hip
rescue_seg_kernel, round 5): flagged windows compacted per
512-window chunk, then pass 0 by shared segment states over dense runs of R
windows (R chosen per launch from H = hop / 64 and K, not necessarily a
divisor of the chunk), pass 0 per window for sparse runs and for fold plans
(by the fold), and the exact chain for what pass 0 leaves.

The data here mixes runs of near-tie windows (two plan tones at equal power:
every window flagged) with runs of clean FSK (nothing flagged), with random
run lengths, so every chunk sees dense runs, sparse runs, runs cut by the
chunk's end and partial last chunks; over every H from 1 to 15 and tone
plans from K = 2 to 16 (plain SLIDE and fold-slide). Every symbol must be the
oracle's (oracle/fsk_oracle.c through oracle.goertzel) and no flag bit may be
left. A round-5 run length of 61 (hop 256, K = 2) once read past the list's
end here (profiles/round5/r5n/bounds_probe_before_fix.log).
"""
import numpy as np
import pytest

import error_model as EM

pytestmark = pytest.mark.gpu

N = 1024
K16 = tuple(46.875 * (20 + 7 * i) for i in range(16))
FOLD3 = (8 * EM.BIN, 16 * EM.BIN, 504 * EM.BIN)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def mixed_stream(freqs, blocks, seed):
    """Runs of 1..40 n-sample blocks alternating between two tones at equal
    power (near ties) and clean FSK at sigma 400."""
    rng = np.random.default_rng(seed)
    tie = EM.family("two_tone_equal", freqs, N, blocks, seed)
    fsk = EM.family("fsk_s400", freqs, N, blocks, seed + 1)
    out = np.empty(blocks * N, np.int16)
    b, use_tie = 0, bool(rng.integers(0, 2))
    while b < blocks:
        r = int(rng.integers(1, 41))
        e = min(blocks, b + r)
        src = tie if use_tie else fsk
        out[b * N:e * N] = src[b * N:e * N]
        b, use_tie = e, not use_tie
    return out


def run(A, O, freqs, hop, W, seed, expect_slide=True):
    blocks = -(-((W - 1) * hop + N) // N)
    x = mixed_stream(freqs, blocks, seed)[:(W - 1) * hop + N]
    with A.Demodulator(A.make_cfg(n=N, hop=hop, freqs=freqs)) as d:
        if expect_slide:
            assert d.slide_windows > 0
        assert d.rescue_tau64 > 0
        sym = d.batch(x, n_windows=W)
    rs, _ = O.goertzel(x, freqs, N, hop=hop, fs=EM.FS, threads=16)
    assert not (sym & 0x80).any()
    bad = np.flatnonzero(sym != rs[:W])
    assert bad.size == 0, bad[:8].tolist()


@pytest.mark.parametrize("H", list(range(1, 16)))
def test_every_hop_k2(A, O, torch, H):
    """2-FSK at hop 64 H: every run length R the launch can pick for K = 2;
    W leaves a partial last chunk."""
    run(A, O, A.FSK2_FREQS, 64 * H, 3 * 512 + 77, seed=H)


@pytest.mark.parametrize("plan", ["FSK8_FREQS", "K16", "FOLD3"])
@pytest.mark.parametrize("H", [1, 3, 4, 7, 15])
def test_plans(A, O, torch, plan, H):
    """8-FSK (fold-slide: pass 0 by the fold, no runs), K = 16 on the plain
    bank (few windows per run: ((R - 1) H + 16) K <= 512), K = 3 fold at the
    band edges."""
    freqs = getattr(A, plan) if hasattr(A, plan) else globals()[plan]
    # (K = 16 on integer bins above hop 384: AUTO takes the residue detector,
    # windows one by one, pass 0 by the residue fold in this launch)
    run(A, O, freqs, 64 * H, 2 * 512 + 301, seed=100 + H,
        expect_slide=not (plan == "K16" and 64 * H > 384))


FOLD16 = tuple(EM.BIN * 8 * (2 + i) for i in range(16))      # 16 tones on multiples of 8 bins
FOLD13 = FOLD16[:13]
FOLD12 = FOLD16[:12]
FFT_ODD = tuple(EM.BIN * (33 + 7 * i) for i in range(4))      # FFT bins not multiples of 8
ODD8 = tuple(EM.BIN * (32 + 9 * i) for i in range(8))         # residues 0 .. 7
EDGES4 = (1 * EM.BIN, 2 * EM.BIN, 511 * EM.BIN, 510 * EM.BIN)  # residues 1, 2, 7, 6


@pytest.mark.parametrize("plan,method,fold64", [
    ("FOLD12", 3, 1),    # fold kernel, pass 0 by the fold (K <= kFold64MaxK)
    ("FOLD13", 3, 0),    # above it: the fold kernels' pass 0 by segments
    ("FOLD16", 3, 0),
    ("FOLD16", 2, 0),    # FFT, bins on multiples of 8 but K > 12: by segments
    ("FOLD12", 2, 1),    # FFT by the fold
    ("FFT_ODD", 2, 0),   # FFT, odd bins: by segments
    ("ODD8", 4, 2),      # residue detector: by the residue fold, every residue class
    ("EDGES4", 4, 2),    # the band edges, complex classes only
    ("FOLD16", 4, 2),    # K = 16, residue 0 only (real chains)
])
@pytest.mark.parametrize("hop", [1024, 256])
def test_pass0_forms(A, O, torch, plan, method, fold64, hop):
    """Each form of the first pass the plan selects (plan.h fold64: by the
    fold at K <= 12 on multiples of 8 bins, by the residue fold on the residue
    detector, else by 64-sample segments; in the
    detector kernel at hop = n, in the rescue launch of segment-shared windows
    at hop 256, in the FFT kernel) on runs of near ties: every symbol the
    oracle's, no flag left."""
    freqs = globals()[plan]
    cfg = A.make_cfg(n=N, hop=hop, freqs=freqs, method=method)
    assert A.plan_info(cfg)["fold64"] == fold64
    W = 1536 + 77
    blocks = -(-((W - 1) * hop + N) // N)
    x = mixed_stream(freqs, blocks, seed=7 + len(freqs) + hop)[:(W - 1) * hop + N]
    with A.Demodulator(cfg) as d:
        assert d.rescue_tau64 > 0
        sym = d.batch(x, n_windows=W)
    rs, _ = (O.fft_demod(x, freqs, N, hop=hop, fs=EM.FS, threads=16) if method == 2 else
             O.goertzel(x, freqs, N, hop=hop, fs=EM.FS, threads=16))
    assert not (sym & 0x80).any()
    bad = np.flatnonzero(sym != rs[:W])
    assert bad.size == 0, bad[:8].tolist()


@pytest.mark.parametrize("hop", [1024, 512, 256])
def test_plain_fsk2_pass0_forms(A, O, torch, hop):
    """The survey's 2-FSK on the plain bank: pass 0 by the fold where its
    windows are evaluated one by one (hop = n and hop 512 ... any hop without
    segment sharing is direct), by shared segment states in the rescue launch
    at hop 256 (SLIDE)."""
    freqs = A.FSK2_FREQS
    cfg = A.make_cfg(n=N, hop=hop, freqs=freqs)
    slide = hop < N and hop % 64 == 0
    assert A.plan_info(cfg)["fold64"] == int(not slide)
    W = 1536 + 77
    blocks = -(-((W - 1) * hop + N) // N)
    x = mixed_stream(freqs, blocks, seed=3 + hop)[:(W - 1) * hop + N]
    with A.Demodulator(cfg) as d:
        assert (d.slide_windows > 0) == slide
        sym = d.batch(x, n_windows=W)
    rs, _ = O.goertzel(x, freqs, N, hop=hop, fs=EM.FS, threads=16)
    assert not (sym & 0x80).any()
    assert np.array_equal(sym, rs[:W])
