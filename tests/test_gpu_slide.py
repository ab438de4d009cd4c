"""Overlapping windows through the segment-shared plain bank (goertzel.hip
SLIDE): n = 1024, hop = 64 H < n. Each 64-sample segment's
Goertzel state is computed once per tile and shared by the windows that
contain it, so the tests sweep what that sharing depends on — H (windows per
tile Wt = (64 - 16) / H + 1), the last tile's partial window count, K up to
16 (the LDS partial slab), the Reinsch plan and non-integer tones — against
the double-precision oracle (oracle/fsk_oracle.c goertzel_window_d via
oracle.py), with the same bar as every detector: |P| within 1e-5 of the
window's max P and the exact-argmax decision rule (tests/decision.py).
"""
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
GOERTZEL = 1
FSK8_ODD = tuple(46.875 * (32 + 9 * i) for i in range(8))
NONINT3 = (1234.5, 2345.6, 4321.0)
REINSCH2 = (30.0, 23950.0)          # |sin w| < 0.1: the Reinsch-form recurrence
K16 = tuple(46.875 * (20 + 7 * i) for i in range(16))


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def wt(hop):
    return (64 - 16) // (hop // 64) + 1


def run(A, O, freqs, hop, W, seed, amplitude=8000, sigma=400, method=GOERTZEL):
    n = 1024
    src = (W - 1) * hop // n + 2
    pcm, _ = O.synth_fsk(freqs, n, src, seed, amplitude, sigma)
    flat = pcm.reshape(-1)
    Wh = min(W, (flat.size - n) // hop + 1)
    with A.Demodulator(n=n, hop=hop, freqs=freqs, method=method) as d:
        assert d.method == GOERTZEL
        assert d.slide_windows == (wt(hop) if hop % 64 == 0 and hop < n else 0)
        sym, mag = d.batch(flat, n_windows=Wh, mags=True)
    ref_sym, ref_P = O.goertzel(flat, freqs, n, hop, Wh)
    denom = np.maximum(ref_P.max(axis=1), 1e-30)
    err = float((np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max())
    assert err <= MAG_TOL, f"magnitude rel err {err:.3e}"
    check_decisions(sym, mag, ref_sym, ref_P)
    return Wh


@pytest.mark.parametrize("hop", [64 * h for h in range(1, 16)])
def test_every_hop(A, O, torch, hop):
    """Every H, with a partial last tile (2 full tiles + 3 windows)."""
    run(A, O, A.FSK2_FREQS, hop, 2 * wt(hop) + 3, seed=hop)


@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 12, 13, 14, 27, 1000])
def test_window_counts_hop256(A, O, torch, W):
    """hop 256 (Wt = 13): tile edges and the 4-window passes (13 = 3 x 4 + 1)."""
    assert run(A, O, A.FSK2_FREQS, 256, W, seed=W) == W


@pytest.mark.parametrize("freqs", ["FSK8_FREQS", "FSK8_ODD", "NONINT3", "REINSCH2", "K16"])
@pytest.mark.parametrize("hop", [128, 256, 512, 960])
def test_tone_plans(A, O, torch, freqs, hop):
    f = getattr(A, freqs) if freqs == "FSK8_FREQS" else globals()[freqs]
    run(A, O, f, hop, 3 * wt(hop) + 2, seed=hop + len(f))


@pytest.mark.parametrize("amplitude,sigma", [(32767, 2000), (300, 400), (8000, 0)])
def test_levels(A, O, torch, amplitude, sigma):
    run(A, O, A.FSK8_FREQS, 256, 500, seed=amplitude, amplitude=amplitude, sigma=sigma)
    run(A, O, FSK8_ODD, 128, 500, seed=amplitude + 1, amplitude=amplitude, sigma=sigma)


def test_auto_takes_slide_for_overlap(A, torch):
    """AUTO picks the segment-shared plain bank for overlapping windows at
    hop 64 H unless the plan folds (K >= 3 on multiples of 8 bins: the fold
    detector's own segment-shared form, tests/test_gpu_fold_slide.py);
    folded / residue stay available explicitly, hop = n keeps the fold."""
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=128) as d:
        assert d.method == 3
    for hop in (128, 256, 384):     # residue plans: SLIDE up to hop 384
        with A.Demodulator(freqs=FSK8_ODD, hop=hop) as d:
            assert d.method == GOERTZEL, hop
    with A.Demodulator(freqs=FSK8_ODD, hop=512) as d:
        assert d.method == 4
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=256) as d:
        assert d.method == 3
    with A.Demodulator(freqs=A.FSK2_FREQS, hop=512) as d:
        assert d.method == GOERTZEL
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=1024) as d:
        assert d.method == 3
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=256, method=3) as d:
        assert d.method == 3
    with A.Demodulator(freqs=A.FSK8_FREQS, hop=200) as d:   # not a multiple of 64
        assert d.method == 3


@pytest.mark.parametrize("freqs", ["FSK2_FREQS", "FSK8_FREQS", "NONINT3", "REINSCH2", "K16"])
@pytest.mark.parametrize("hop", [64, 128, 256, 512])
def test_bit_identical_to_direct_windows(A, O, torch, freqs, hop):
    """Every window hop = 64 H apart whose start is a multiple of n is also a
    window of the hop = n stream, which the direct plain bank evaluates alone:
    the SLIDE result must be the same bits (same segment chains, rotations and
    reduction order)."""
    f = getattr(A, freqs) if hasattr(A, freqs) else globals()[freqs]
    n, src = 1024, 96
    pcm, _ = O.synth_fsk(f, n, src, hop + len(f), 8000, 400)
    flat = pcm.reshape(-1)
    with A.Demodulator(freqs=f, hop=n, method=GOERTZEL) as d:
        sym_d, mag_d = d.batch(flat, mags=True)
    W = (flat.size - n) // hop + 1
    with A.Demodulator(freqs=f, hop=hop, method=GOERTZEL) as d:
        sym_s, mag_s = d.batch(flat, n_windows=W, mags=True)
    step = n // hop
    assert np.array_equal(sym_s[::step], sym_d)
    assert np.array_equal(mag_s[::step].view(np.uint32), mag_d.view(np.uint32))


def test_large_stream_hop256(A, O, torch):
    """4M windows of the synthetic 2-FSK stream (2^30 samples, the configs[3]
    stream): every window aligned to n is bit-identical to the hop = n direct
    evaluation and decodes to the transmitted symbol; an 8192-window sample at
    the end of the stream (last, partial tile included) against the oracle.
    Windows straddling a symbol boundary can put both tone powers ~1e-4 below
    the window's energy N sum x^2 / 2; fp32 evaluation error scales with that
    energy (the direct path reads 3e-5 of max P there too, e.g. at hop 264), so
    the sample's bar normalises by max(max P, energy / 100)."""
    n, hop = 1024, 256
    src = 1 << 20
    cfg = A.make_cfg(freqs=A.FSK2_FREQS, n=n, hop=n)
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    d_true = torch.empty(src, dtype=torch.uint8, device="cuda")
    A.synth_fsk(cfg, 12345, src, 8000, 400, d_pcm, d_true)
    W = (src * n - n) // hop + 1
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    mag = torch.empty(W * 2, dtype=torch.float32, device="cuda")
    with A.Demodulator(freqs=A.FSK2_FREQS, hop=hop) as d:
        d.batch_device(d_pcm, W, sym, mag)
    sym_d = torch.empty(src, dtype=torch.uint8, device="cuda")
    mag_d = torch.empty(src * 2, dtype=torch.float32, device="cuda")
    with A.Demodulator(freqs=A.FSK2_FREQS, hop=n) as d:
        d.batch_device(d_pcm, src, sym_d, mag_d)
    torch.cuda.synchronize()
    assert int((sym[::4] != d_true).sum().item()) == 0
    assert bool((sym[::4] == sym_d).all().item())
    assert bool((mag.view(W, 2)[::4].contiguous().view(torch.int32) ==
                 mag_d.view(src, 2).view(torch.int32)).all().item())
    S = 8192
    x = d_pcm[-(S * hop // n + 4):].cpu().numpy().reshape(-1)
    off = W - ((x.size - n) // hop + 1)                  # first window of the sample
    ref_sym, ref_P = O.goertzel(x, A.FSK2_FREQS, n, hop)
    g_sym = sym[off:].cpu().numpy()
    g_mag = mag.view(W, 2)[off:].cpu().numpy()
    xw = np.lib.stride_tricks.sliding_window_view(x.astype(np.float64), n)[::hop]
    energy = n * (xw * xw).sum(axis=1) / 2
    denom = np.maximum(ref_P.max(axis=1), energy / 100)
    assert (np.abs(g_mag.astype(np.float64) - ref_P).max(axis=1) / denom).max() <= MAG_TOL
    check_decisions(g_sym, g_mag, ref_sym, ref_P, denom)


def draw(i):
    rng = np.random.default_rng(0x51DE + i)
    H = int(rng.integers(1, 16))
    k = int(rng.integers(1, 17))
    if rng.random() < 0.5:
        bins = np.sort(rng.choice(np.arange(2, 510), k, replace=False)).astype(np.float64)
    else:
        for _ in range(1000):
            bins = np.sort(rng.uniform(2.0, 510.0, k))
            if k == 1 or np.diff(bins).min() >= 2.0:
                break
    freqs = tuple(float(b) * 48000.0 / 1024 for b in rng.permutation(bins))
    W = int(rng.integers(1, 300))
    amplitude = int(rng.choice([300, 2000, 8000, 20000]))
    sigma = int(rng.choice([0, 100, 400, 1500]))
    return H, freqs, W, amplitude, sigma


@pytest.mark.parametrize("i", range(40))
def test_random_sweep(A, O, torch, i):
    """Seeded random H, K (1..16), integer / off-bin plans, window count and
    level; windows whose tone powers sit far below their energy (a symbol
    boundary cancelling every tone) are normalised by energy / 100, as in
    test_large_stream_hop256."""
    H, freqs, W, amplitude, sigma = draw(i)
    n, hop = 1024, 64 * H
    src = (W - 1) * hop // n + 2
    pcm, _ = O.synth_fsk(freqs, n, src, 77 + i, amplitude, sigma)
    flat = pcm.reshape(-1)
    Wh = min(W, (flat.size - n) // hop + 1)
    with A.Demodulator(n=n, hop=hop, freqs=freqs, method=GOERTZEL) as d:
        sym, mag = d.batch(flat, n_windows=Wh, mags=True)
    ref_sym, ref_P = O.goertzel(flat, freqs, n, hop, Wh)
    xw = np.lib.stride_tricks.sliding_window_view(flat.astype(np.float64), n)[::hop][:Wh]
    energy = n * (xw * xw).sum(axis=1) / 2
    denom = np.maximum(np.maximum(ref_P.max(axis=1), energy / 100), 1e-30)
    assert (np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max() <= MAG_TOL
    check_decisions(sym, mag, ref_sym, ref_P, denom)


@pytest.mark.parametrize("hop,channels", [(256, 1), (128, 2), (64, 1), (960, 2)])
def test_streaming_demodulate(A, O, torch, hop, channels):
    """demodulate() over ragged packets (carry buffer across calls) with the
    segment-shared bank: the same symbols as the oracle's stream."""
    n = 1024
    L, _ = O.synth_fsk(A.FSK2_FREQS, n, 40, 900 + hop)
    R, _ = O.synth_fsk(A.FSK2_FREQS, n, 40, 901 + hop)
    mono = L.reshape(-1)
    stream = mono if channels == 1 else np.stack([mono, R.reshape(-1)], axis=1).reshape(-1)
    ref = O.Stream(A.FSK2_FREQS, n=n, hop=hop, channels=channels)
    sizes = [2880, 100, 1, 4097, 2880, 64, 7000]
    got, want = [], []
    with A.Demodulator(A.make_cfg(freqs=A.FSK2_FREQS, hop=hop, channels=channels,
                                  method=GOERTZEL)) as d:
        pos, i = 0, 0
        while pos < mono.size:
            fr = sizes[i % len(sizes)]
            i += 1
            chunk = stream[pos * channels:(pos + fr) * channels]
            pos += fr
            got.append(d.demodulate(chunk))
            want.append(ref.push(chunk)[0])
            assert d.pending() == ref.pending()
    got, want = np.concatenate(got), np.concatenate(want)
    assert got.size == want.size == (40 * n - n) // hop + 1
    assert (got == want).all()
