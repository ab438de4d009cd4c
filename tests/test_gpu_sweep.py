"""Seeded random sweep of the GPU path against the oracle: detector, window
length, hop, tone count and plan, batch size and signal level drawn together,
so combinations the hand-picked cases of test_gpu_parity.py do not list are
still covered (every detector behind the same C ABI, demod_batch).

Bar as in test_gpu_parity.py: |X_k|^2 within 1e-5 of the window's max_k P_ref
(double oracle), symbols bit-exact wherever the oracle's decision is not a tie
inside that tolerance (hop < n windows straddle two symbols, and two tones can
then carry near-equal power); such ties must stay rare.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MAG_TOL = 1e-5
FS = 48000.0
N_CASES = 48


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def draw_case(i):
    rng = np.random.default_rng(0x5EED + i)
    method = ["auto", "goertzel", "folded", "residue", "fft"][i % 5]
    n = 1024 if method == "fft" else int(2 ** rng.integers(6, 13))  # 64 .. 4096
    half = n // 2
    if method == "folded":
        slots = np.arange(8, half - 1, 8)                  # multiples of 8 bins
    elif method in ("residue", "fft") or rng.random() < 0.5:
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
    c = draw_case(i)
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
    denom = np.maximum(ref_P.max(axis=1), 1e-30)
    err = (np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom).max()
    assert err <= MAG_TOL, (err, c)
    Ps = np.sort(ref_P, axis=1)
    posed = (Ps[:, -1] - Ps[:, -2]) / denom > 4 * MAG_TOL if ref_P.shape[1] > 1 \
        else np.ones(Wh, bool)
    # windows inside one symbol have one clear winner; windows straddling two
    # symbols (hop not a multiple of n) can split the power evenly
    assert posed.mean() >= (0.99 if hop % n == 0 else 0.9), c
    bad = np.flatnonzero(posed & (sym != ref_sym))
    assert bad.size == 0, (bad[:8], c)
