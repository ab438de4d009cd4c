"""Seeded random sweep of the GPU path against the oracle: detector, window
length, hop, tone count and plan, batch size and signal level drawn together,
so combinations the hand-picked cases of test_gpu_parity.py do not list are
still covered (every detector behind the same C ABI, demod_batch).

Bar as in test_gpu_parity.py: |X_k|^2 within 1e-5 of the window's max_k P_ref
(double oracle; of its spectral energy where that is larger, mag_denom),
symbols bit-exact on every window (tests/decision.py): hop < n windows
straddle two symbols and two tones can then carry near-equal power; the
decision rescue decides those in double.
"""
import numpy as np
import pytest

from decision import check_decisions

pytestmark = pytest.mark.gpu

MAG_TOL = 1e-5
FS = 48000.0
N_CASES = 120
# FSKD_SWEEP_SEED=s draws a different set of cases (default 0: the committed
# set); a deeper ad-hoc run: FSKD_SWEEP_SEED=1 ... -m gpu tests/test_gpu_sweep.py
SEED_OFFSET = 1000003 * int(__import__("os").environ.get("FSKD_SWEEP_SEED", "0"))


def mag_denom(P, mono, n, hop):
    """Per-window normaliser of |P_gpu - P_ref|: max_k P_ref, or the window's
    spectral energy n * sum(x^2) / 2 when that is larger (equal to max_k P for
    a clean tone). The fp32 error scales with the window's energy, not with the
    tone powers: where hop < n splices two symbols with unrelated phases, a
    single tone (K = 1) can cancel to far below the energy, and 1e-5 of that P
    is below fp32 resolution (as for the degenerate windows of
    test_gpu_parity.py::test_zero_and_extreme_input)."""
    x = mono.astype(np.float64)
    c2 = np.concatenate([[0.0], np.cumsum(x * x)])
    starts = np.arange(P.shape[0]) * hop
    energy = n * (c2[starts + n] - c2[starts]) / 2
    return np.maximum(np.maximum(P.max(axis=1), energy), 1e-30)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def draw_case(i, fft_nonint=False):
    """fft_nonint: the FFT detector may get off-bin tones (it picks the nearest
    bin, as oracle.fft_demod does); the streaming oracle is the Goertzel bank,
    so streaming cases keep FFT tones on integer bins."""
    rng = np.random.default_rng(0x5EED + i + SEED_OFFSET)
    method = ["auto", "goertzel", "folded", "residue", "fft"][i % 5]
    n = 1024 if method == "fft" else int(2 ** rng.integers(6, 13))  # 64 .. 4096
    half = n // 2
    if method == "folded":
        slots = np.arange(8, half - 1, 8)                  # multiples of 8 bins
    elif method == "residue" or (method == "fft" and not fft_nonint) or rng.random() < 0.5:
        slots = np.arange(2, half - 1)                     # integer bins
    else:
        slots = None                                       # arbitrary frequencies
    kmax = 16 if slots is None else min(16, len(slots))
    k = int(rng.integers(1, kmax + 1))
    if slots is None:
        for _ in range(1000):
            b = np.sort(rng.uniform(2.0, half - 2.0, k))
            if k == 1 or np.diff(b).min() >= 2.0:
                break
        else:
            # no draw kept the tones 2 bins apart (many tones in a short
            # window): spread them evenly instead, with a random sub-bin offset,
            # so the plan stays resolvable (tones a fraction of a bin apart
            # make most decisions ties, which the case is not testing)
            step = (half - 4.0) / k
            b = 2.0 + step * (np.arange(k) + 0.5) + rng.uniform(-0.25, 0.25) * min(step - 2.0, 1.0)
    else:
        b = np.sort(rng.choice(slots, k, replace=False)).astype(np.float64)
    freqs = tuple(float(x) * FS / n for x in rng.permutation(b))
    # the ABI takes hops that are multiples of 8 in [8, n] (demod_api.cpp validate)
    hop = n if rng.random() < 0.4 else 8 * int(rng.integers(1, n // 8 + 1))
    W = int(rng.integers(1, 400))
    amplitude = int(rng.choice([300, 2000, 8000, 20000]))
    sigma = int(rng.choice([0, 100, 400, 1500]))
    return dict(method=method, n=n, freqs=freqs, hop=hop, W=W, amplitude=amplitude,
                sigma=sigma, seed=1000 + i)


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_case(A, O, torch, i):
    c = draw_case(i, fft_nonint=True)
    m = {"auto": A.METHOD_AUTO, "goertzel": A.METHOD_GOERTZEL, "folded": A.METHOD_FOLDED,
         "residue": A.METHOD_RESIDUE, "fft": A.METHOD_FFT}[c["method"]]
    n, hop, freqs = c["n"], c["hop"], c["freqs"]
    pcm, _ = O.synth_fsk(freqs, n, c["W"], c["seed"], c["amplitude"], c["sigma"])
    flat = pcm.reshape(-1)
    # bound the oracle's work (small hops over long windows): at most 3000 windows
    Wh = min((flat.size - n) // hop + 1, 3000)
    flat = flat[:(Wh - 1) * hop + n]
    with A.Demodulator(n=n, hop=hop, freqs=freqs, method=m) as d:
        if m != A.METHOD_AUTO:
            assert d.method == m, c
        sym, mag = d.batch(flat, n_windows=Wh, mags=True)
    if c["method"] == "fft":
        ref_sym, ref_P = O.fft_demod(flat, freqs, n, hop)
    else:
        ref_sym, ref_P = O.goertzel(flat, freqs, n, hop, Wh)
    assert sym.shape == ref_sym.shape and mag.shape == ref_P.shape
    denom = mag_denom(ref_P, flat, n, hop)
    err = (np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max()
    assert err <= MAG_TOL, (err, c)
    # every window, straddling and structurally tied ones included (hop not a
    # multiple of n splits a window's power between two symbols' tones)
    check_decisions(sym, mag, ref_sym, ref_P, denom)


N_STREAM_CASES = 40


@pytest.mark.parametrize("i", range(N_STREAM_CASES))
def test_random_stream(A, O, torch, i):
    """Streaming demodulate(pcm, n) with random ragged packets: mono or
    stereo (left, right or (L+R)>>1), any detector, hop <= n, against the
    oracle's streaming restatement (oracle.Stream): same symbols, same pending
    count after every call, magnitudes within the bar."""
    c = draw_case(100 + i)
    rng = np.random.default_rng(0xABC + i + SEED_OFFSET)
    m = {"auto": A.METHOD_AUTO, "goertzel": A.METHOD_GOERTZEL, "folded": A.METHOD_FOLDED,
         "residue": A.METHOD_RESIDUE, "fft": A.METHOD_FFT}[c["method"]]
    n, hop, freqs = c["n"], c["hop"], c["freqs"]
    W = min(c["W"], 120)
    channels = int(rng.integers(1, 3))
    mode = int(rng.integers(0, 3)) if channels == 2 else 0
    Lc, _ = O.synth_fsk(freqs, n, W, c["seed"], c["amplitude"], c["sigma"])
    if channels == 1:
        stream = Lc.reshape(-1)
    else:
        Rc, _ = O.synth_fsk(freqs, n, W, c["seed"] + 1, c["amplitude"], c["sigma"])
        stream = np.stack([Lc.reshape(-1), Rc.reshape(-1)], axis=1).reshape(-1)
    ref = O.Stream(freqs, n=n, hop=hop, channels=channels, channel_mode=mode)
    got_s, got_m, want_s, want_P = [], [], [], []
    total = stream.size // channels
    with A.Demodulator(n=n, hop=hop, freqs=freqs, method=m, channels=channels,
                       channel_mode=mode) as d:
        pos = 0
        while pos < total:
            fr = int(rng.choice([0, 1, 7, 2880, int(rng.integers(1, 3 * n))]))
            chunk = stream[pos * channels:(pos + fr) * channels]
            pos += fr
            s, mg = d.demodulate(chunk, mags=True)
            rs, rP = ref.push(chunk)
            got_s.append(s), got_m.append(mg), want_s.append(rs), want_P.append(rP)
            assert d.pending() == ref.pending(), c
    gs, ws = np.concatenate(got_s), np.concatenate(want_s)
    gm, wP = np.concatenate(got_m), np.concatenate(want_P)
    assert gs.size == ws.size == (total - n) // hop + 1, c
    # oracle.Stream evaluates the Goertzel bank; for the FFT detector that is
    # the same |X_k|^2, since FFT draws put every tone on an integer bin
    if channels == 1:
        mono = stream
    else:
        lr = stream.reshape(-1, 2).astype(np.int32)
        mono = (lr[:, 0], lr[:, 1], (lr[:, 0] + lr[:, 1]) >> 1)[mode]
    denom = mag_denom(wP, mono, n, hop)
    err = (np.abs(gm.astype(np.float64) - wP).max(axis=1) / denom).max()
    assert err <= MAG_TOL, (err, c)
    check_decisions(gs, gm, ws, wP, denom)


N_STRUCT_CASES = 40


@pytest.mark.parametrize("i", range(N_STRUCT_CASES))
def test_random_permuted_plans(A, O, torch, i):
    """Plans that take the permuted-slot kernels at n = 1024 (DESIGN.md §4.2,
    §4.3): fold by 16 (K = 8, four tones on multiples of 16 bins and four on
    odd multiples of 8) and the residue kernel's compile-time classes (K = 8
    or 16 with K / 4 tones per class; cases 24+: even-bin plans, K / 2 tones
    in each of classes 0 and 3 or all K in one of them), in random tone
    order, hop and level; magnitudes and symbols in the caller's tone order."""
    rng = np.random.default_rng(0xC1A55 + i + SEED_OFFSET)
    kind = (("fold16", "residue8", "residue16")[i % 3] if i < 24 else
            ("even_split8", "even_one8", "even_split16", "even_one16")[i % 4])
    if kind.startswith("even"):
        K = 8 if kind.endswith("8") else 16
        c0 = [b for b in range(4, 505) if b % 4 == 0]          # residues 0, 4: class 0
        c3 = [b for b in range(2, 505) if b % 4 == 2]          # residues 2, 6: class 3
        if kind.startswith("even_split"):
            bins = np.concatenate([rng.choice(c0, K // 2, replace=False),
                                   rng.choice(c3, K // 2, replace=False)])
        else:
            bins = rng.choice(c0 if rng.random() < 0.5 else c3, K, replace=False)
        method = A.METHOD_RESIDUE
    elif kind == "fold16":
        z0 = rng.choice(np.arange(1, 31) * 16, 4, replace=False)
        z8 = rng.choice(np.arange(0, 31) * 16 + 8, 4, replace=False)
        bins = np.concatenate([z0, z8])
        method = A.METHOD_FOLDED
    else:
        K = 8 if kind == "residue8" else 16
        cls_of = {0: 0, 4: 0, 1: 1, 7: 1, 3: 2, 5: 2, 2: 3, 6: 3}
        bins = []
        for c in range(4):
            rhos = [r for r, cc in cls_of.items() if cc == c]
            pool = [b for b in range(8, 505) if b % 8 in rhos and b not in bins]
            bins += list(rng.choice(pool, K // 4, replace=False))
        bins = np.array(bins)
        method = A.METHOD_RESIDUE
    bins = rng.permutation(bins)
    freqs = tuple(float(b) * 46.875 for b in bins)
    hop = 1024 if rng.random() < 0.5 else 8 * int(rng.integers(1, 129))
    W = int(rng.integers(1, 500))
    pcm, _ = O.synth_fsk(freqs, 1024, W, 7000 + i, int(rng.choice([300, 8000, 30000])),
                         int(rng.choice([0, 400, 1500])))
    flat = pcm.reshape(-1)
    Wh = min((flat.size - 1024) // hop + 1, 3000)
    flat = flat[:(Wh - 1) * hop + 1024]
    with A.Demodulator(hop=hop, freqs=freqs, method=method) as d:
        assert d.method == method
        sym, mag = d.batch(flat, n_windows=Wh, mags=True)
    ref_sym, ref_P = O.goertzel(flat, freqs, 1024, hop, Wh)
    denom = mag_denom(ref_P, flat, 1024, hop)
    err = (np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max()
    assert err <= MAG_TOL, (err, kind, list(bins))
    check_decisions(sym, mag, ref_sym, ref_P, denom)


N_SLIDE_CASES = 40


@pytest.mark.parametrize("i", range(N_SLIDE_CASES))
def test_random_segment_shared(A, O, torch, i, monkeypatch):
    """The segment-shared paths at n = 1024, hop = 64 H < n:
    the plain SLIDE (any plan) and the fold detector's running sums (plans on
    multiples of 8 bins, incl. fold-by-16 plans), drawn with random H, K,
    tone order, batch size and level; against the oracle with the same bar,
    and bit-identical to the direct kernels (FSKD_NO_SLIDE=1). Both rescue
    their flagged windows with the exact double chain (FSKD_RESCUE_SEG=0: the
    direct kernels' first pass by segments is within its model of the exact
    powers, not the same bits)."""
    import os
    monkeypatch.setenv("FSKD_RESCUE_SEG", "0")
    rng = np.random.default_rng(0x511DE + i + SEED_OFFSET)
    n = 1024
    kind = ("fold", "fold16", "plain")[i % 3]
    if kind == "fold16":
        z0 = rng.choice(np.arange(1, 31) * 16, 4, replace=False)
        z8 = rng.choice(np.arange(0, 31) * 16 + 8, 4, replace=False)
        bins = rng.permutation(np.concatenate([z0, z8])).astype(np.float64)
        method = A.METHOD_FOLDED
    elif kind == "fold":
        k = int(rng.integers(1, 17))
        bins = rng.choice(np.arange(8, 505, 8), k, replace=False).astype(np.float64)
        method = A.METHOD_FOLDED
    else:
        k = int(rng.integers(1, 17))
        if rng.random() < 0.5:
            bins = rng.choice(np.arange(2, 510), k, replace=False).astype(np.float64)
        else:
            bins = rng.uniform(2.0, 510.0, k)
        method = A.METHOD_GOERTZEL
    freqs = tuple(float(b) * FS / n for b in bins)
    hop = 64 * int(rng.integers(1, 16))
    W = int(rng.integers(1, 700))
    amplitude = int(rng.choice([300, 2000, 8000, 32767]))
    sigma = int(rng.choice([0, 100, 400, 1500]))
    src = (W - 1) * hop // n + 2
    pcm, _ = O.synth_fsk(freqs, n, src, 77 + i, amplitude, sigma)
    flat = pcm.reshape(-1)
    Wh = min(W, (flat.size - n) // hop + 1)
    out = []
    for direct in (False, True):
        old = os.environ.get("FSKD_NO_SLIDE")
        if direct:
            os.environ["FSKD_NO_SLIDE"] = "1"
        try:
            with A.Demodulator(n=n, hop=hop, freqs=freqs, method=method) as d:
                assert d.method == method
                assert (d.slide_windows == 0) == direct
                out.append(d.batch(flat, n_windows=Wh, mags=True))
        finally:
            if direct:
                if old is None:
                    del os.environ["FSKD_NO_SLIDE"]
                else:
                    os.environ["FSKD_NO_SLIDE"] = old
    (sym, mag), (sym_d, mag_d) = out
    assert np.array_equal(sym, sym_d), (kind, hop, W)
    assert np.array_equal(mag.view(np.uint32), mag_d.view(np.uint32)), (kind, hop, W)
    ref_sym, ref_P = O.goertzel(flat, freqs, n, hop, Wh)
    denom = mag_denom(ref_P, flat, n, hop)
    err = (np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max()
    assert err <= MAG_TOL, (err, kind, hop, W)
    check_decisions(sym, mag, ref_sym, ref_P, denom)
