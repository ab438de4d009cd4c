"""Overlapping windows through the fold detector's segment-shared form
(fold.hip fold_slide_kernel): n = 1024, hop = 64 H < n, tone
plans on multiples of 8 bins. A lane's folded sums (even or odd segments of
the window at 8 positions) run forward from window to window — minus the H
segments that leave, plus the H that enter, E/O swapped between partner lanes
for odd H — so every window's sums are the integers direct folding forms and
its result must be BIT-identical to fold_tile_kernel evaluating it alone
(FSKD_NO_SLIDE=1 selects that kernel on the same handle configuration). The
oracle bar is the same as every detector's: |P| within 1e-5 of the window's
max P and the exact-argmax decision rule (tests/decision.py).
"""
import os

import numpy as np
import pytest

from decision import check_decisions

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _exact_rescue_everywhere(monkeypatch):
    """The segment-shared kernels rescue their flagged windows with the exact
    double chain (rescue launch); the direct kernels' in-kernel rescue first
    tries a double pass by segments, whose powers are within
    its model of the exact ones but not the same bits. These tests compare
    the two kernels' arithmetic bit for bit, so the direct runs take the
    exact path too (FSKD_RESCUE_SEG=0, read at demod_create)."""
    monkeypatch.setenv("FSKD_RESCUE_SEG", "0")

MAG_TOL = 1e-5
FOLDED = 3
K3 = tuple(46.875 * b for b in (40, 64, 120))                 # generic fold, odd K
K5 = tuple(46.875 * b for b in (16, 48, 56, 96, 200))
K16 = tuple(46.875 * (24 + 8 * i) for i in range(16))        # the LDS-free K = 16 fold
FSK8_SHUFFLED = tuple(1500.0 + 375.0 * i for i in (5, 2, 7, 0, 3, 6, 1, 4))  # F16, permuted slots


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def wt(hop):
    """Windows per fold tile: 4 R, the largest R whose 16 + (4R - 1) H
    segments fit the 80-segment tile (demod_api.cpp, kFoldSlideSegs)."""
    return 4 * max(1, ((80 - 16) // (hop // 64) + 1) // 4)


def plan(A, name):
    return getattr(A, name) if hasattr(A, name) else globals()[name]


def demod(A, freqs, hop, flat, W, direct=False, method=FOLDED):
    """(symbols, magnitudes) of W windows; direct: the per-window kernel."""
    old = os.environ.get("FSKD_NO_SLIDE")
    if direct:
        os.environ["FSKD_NO_SLIDE"] = "1"
    try:
        with A.Demodulator(n=1024, hop=hop, freqs=freqs, method=method) as d:
            assert d.method == FOLDED
            # the two runs really take different kernels
            assert d.slide_windows == (0 if (direct or hop % 64) else wt(hop))
            return d.batch(flat, n_windows=W, mags=True)
    finally:
        if direct:
            if old is None:
                del os.environ["FSKD_NO_SLIDE"]
            else:
                os.environ["FSKD_NO_SLIDE"] = old


def run(A, O, freqs, hop, W, seed, amplitude=8000, sigma=400, method=FOLDED):
    """Oracle parity and bit-identity with the direct fold kernel."""
    n = 1024
    src = (W - 1) * hop // n + 2
    pcm, _ = O.synth_fsk(freqs, n, src, seed, amplitude, sigma)
    flat = pcm.reshape(-1)
    Wh = min(W, (flat.size - n) // hop + 1)
    sym, mag = demod(A, freqs, hop, flat, Wh, method=method)
    ref_sym, ref_P = O.goertzel(flat, freqs, n, hop, Wh)
    denom = np.maximum(ref_P.max(axis=1), 1e-30)
    err = float((np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max())
    assert err <= MAG_TOL, f"magnitude rel err {err:.3e}"
    check_decisions(sym, mag, ref_sym, ref_P)
    sym_d, mag_d = demod(A, freqs, hop, flat, Wh, direct=True, method=method)
    assert np.array_equal(sym, sym_d)
    assert np.array_equal(mag.view(np.uint32), mag_d.view(np.uint32))
    return Wh


@pytest.mark.parametrize("hop", [64 * h for h in range(1, 16)])
@pytest.mark.parametrize("freqs", ["FSK8_FREQS", "K3"])
def test_every_hop(A, O, torch, freqs, hop):
    """Every H (odd H swaps the E / O sums between partner lanes), F16 and the
    generic fold, with a partial last tile (2 full tiles + 3 windows)."""
    run(A, O, plan(A, freqs), hop, 2 * wt(hop) + 3, seed=hop + 7)


@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 15, 16, 17, 31, 33, 1000])
def test_window_counts_hop256(A, O, torch, W):
    """hop 256 (16 windows per 76-segment tile, 4 per 16-lane group): tile
    edges, groups with no live window, short batches."""
    assert run(A, O, A.FSK8_FREQS, 256, W, seed=W) == W


@pytest.mark.parametrize("freqs", ["FSK2_FREQS", "K5", "K16", "FSK8_SHUFFLED"])
@pytest.mark.parametrize("hop", [64, 128, 256, 512, 960])
def test_tone_plans(A, O, torch, freqs, hop):
    run(A, O, plan(A, freqs), hop, 3 * wt(hop) + 2, seed=hop + 3)


@pytest.mark.parametrize("amplitude,sigma", [(32767, 2000), (300, 400), (8000, 0)])
@pytest.mark.parametrize("hop", [64, 192, 256])
def test_levels(A, O, torch, amplitude, sigma, hop):
    """Full scale (16-segment sums near 2^19), small signals, no noise."""
    run(A, O, A.FSK8_FREQS, hop, 300, seed=amplitude + hop, amplitude=amplitude, sigma=sigma)


def test_extreme_samples(A, torch):
    """Rails, alternating rails and random full-range samples: the sums stay
    exact (|sum| <= 16 x 32768), the result equals the direct kernel bit for
    bit at every window."""
    n, hop = 1024, 128
    rng = np.random.default_rng(5)
    x = np.concatenate([np.full(3 * n, 32767), np.full(2 * n, -32768),
                        np.tile([32767, -32768], 2 * n), rng.integers(-32768, 32768, 9 * n)])
    flat = x.astype(np.int16)
    W = (flat.size - n) // hop + 1
    for f in (A.FSK8_FREQS, K3):
        sym, mag = demod(A, f, hop, flat, W)
        sym_d, mag_d = demod(A, f, hop, flat, W, direct=True)
        assert np.array_equal(sym, sym_d)
        assert np.array_equal(mag.view(np.uint32), mag_d.view(np.uint32))


def test_auto_takes_fold_slide(A, torch):
    """AUTO: fold-eligible plans with K >= 3 take the fold detector at every
    hop (its segment-shared form at hop = 64 H); other integer-bin plans keep
    the plain SLIDE up to hop 384."""
    for hop in (64, 128, 256, 512, 1024, 200):
        with A.Demodulator(freqs=A.FSK8_FREQS, hop=hop) as d:
            assert d.method == FOLDED, hop
    with A.Demodulator(freqs=tuple(46.875 * (32 + 9 * i) for i in range(8)), hop=128) as d:
        assert d.method == 1


def test_streaming_overlap(A, O, torch):
    """Streaming demodulate() at hop 256 with ragged packets (the carry buffer
    feeds the segment-shared fold batches) against the oracle's stream."""
    n, hop = 1024, 256
    pcm, _ = O.synth_fsk(A.FSK8_FREQS, n, 40, 99, 8000, 400)
    flat = pcm.reshape(-1)
    ref = O.Stream(n=n, hop=hop, freqs=A.FSK8_FREQS)
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=hop) as d:
        assert d.method == FOLDED
        pos, got, want = 0, [], []
        rng = np.random.default_rng(3)
        while pos < flat.size:
            step = int(rng.integers(1, 5000))
            chunk = flat[pos:pos + step]
            pos += step
            got.append(d.demodulate(chunk))
            want.append(ref.push(chunk)[0])
    assert np.array_equal(np.concatenate(got), np.concatenate(want))


def test_large_stream_hop256(A, torch):
    """4M windows at hop 256 over the 2^30-sample synthetic 8-FSK stream:
    every window equals the direct fold kernel's (bits), and the windows
    aligned to n decode to the transmitted symbols."""
    n, hop, K = 1024, 256, 8
    src = 1 << 20
    cfg = A.make_cfg(freqs=A.FSK8_FREQS, n=n, hop=n)
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    d_true = torch.empty(src, dtype=torch.uint8, device="cuda")
    A.synth_fsk(cfg, 4321, src, 8000, 400, d_pcm, d_true)
    W = (src * n - n) // hop + 1
    out = []
    for direct in (False, True):
        old = os.environ.get("FSKD_NO_SLIDE")
        if direct:
            os.environ["FSKD_NO_SLIDE"] = "1"
        try:
            sym = torch.empty(W, dtype=torch.uint8, device="cuda")
            mag = torch.empty(W * K, dtype=torch.float32, device="cuda")
            with A.Demodulator(freqs=A.FSK8_FREQS, hop=hop) as d:
                assert d.method == FOLDED
                assert (d.slide_windows == 0) == direct
                d.batch_device(d_pcm, W, sym, mag)
            torch.cuda.synchronize()
            out.append((sym, mag))
        finally:
            if direct:
                if old is None:
                    del os.environ["FSKD_NO_SLIDE"]
                else:
                    os.environ["FSKD_NO_SLIDE"] = old
    (sym, mag), (sym_d, mag_d) = out
    assert int((sym[::4] != d_true).sum().item()) == 0
    assert bool((sym == sym_d).all().item())
    assert bool((mag.view(torch.int32) == mag_d.view(torch.int32)).all().item())
