"""Near-tie decisions on every detector.

Windows carry two tones whose powers differ by a designed ratio 1 + eps,
eps in {0, 1e-7 .. 1e-4}, in both orders (so the higher-index tone is
sometimes the larger one), with random phases. int16 rounding then spreads
the realised power ratios over a few 1e-6 around eps: many windows fall
inside 2^-19 (the band the round-1 packed-key argmax resolved to the lower
tone whatever the powers said), far inside the fp32 error of the powers.
Every decision must equal the double oracle's (tests/decision.py): the
detectors flag these windows and the decision rescue decides them with the
oracle's own double arithmetic (rescue.hip). With the rescue
switched off (FSKD_NO_RESCUE=1, a measurement switch) the fp32 decisions
differ from the oracle on some of them: the rescue is what makes them exact.
"""
import contextlib
import os
import zlib

import numpy as np
import pytest

from decision import check_decisions

pytestmark = pytest.mark.gpu

AUTO, GOERTZEL, FFT, FOLDED, RESIDUE = 0, 1, 2, 3, 4
FSK8_ODD = tuple(46.875 * (32 + 9 * i) for i in range(8))
NONINT8 = tuple(1234.5 + 1111.1 * i for i in range(8))


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def near_tie_windows(freqs, W, seed, n=1024, amp=9000.0):
    """W windows, each two random tones a, b of the plan with random phases;
    b's amplitude is solved (bisection, double precision, before rounding to
    int16) so that the two tones' DFT powers at their own frequencies are in
    ratio P_b / P_a = 1 + eps exactly — including the leakage between them,
    which matters for off-bin plans."""
    rng = np.random.default_rng(seed)
    K = len(freqs)
    t = np.arange(n)
    eps_set = np.array([0.0, 1e-7, 3e-7, 1e-6, 2e-6, 5e-6, 1e-5, 1e-4])
    ab = np.array([rng.choice(K, 2, replace=False) for _ in range(W)])
    eps = eps_set[np.arange(W) % eps_set.size]
    ph = rng.uniform(0, 2 * np.pi, (W, 2))
    w = 2 * np.pi * np.asarray(freqs, np.float64)[ab] / 48000.0          # (W, 2)
    tones = np.cos(w[:, :, None] * t + ph[:, :, None])                  # (W, 2, n)
    E = np.exp(-1j * w[:, :, None] * t)                                  # (W, 2, n)
    c = np.einsum("wjn,wkn->wjk", tones, E)   # c[w, j, k]: tone j's DFT at tone k's frequency

    def ratio(a2):
        Xa = amp * c[:, 0, 0] + a2 * c[:, 1, 0]
        Xb = amp * c[:, 0, 1] + a2 * c[:, 1, 1]
        return np.abs(Xb) ** 2 / np.abs(Xa) ** 2

    lo, hi = np.full(W, 0.5 * amp), np.full(W, 2.0 * amp)
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        up = ratio(mid) < 1.0 + eps
        lo, hi = np.where(up, mid, lo), np.where(up, hi, mid)
    a2 = 0.5 * (lo + hi)
    v = amp * tones[:, 0] + a2[:, None] * tones[:, 1]
    x = np.clip(np.round(v), -32768, 32767).astype(np.int16)
    return x, ab


@pytest.mark.parametrize("plan,method", [
    ("FSK8_FREQS", FOLDED),      # fold by 16 (F16), window_sum_decide_split8
    ("FSK8_FREQS", GOERTZEL),    # plain bank, K = 8, window_sum_decide
    ("FSK8_ODD", RESIDUE),       # residue kernel, compile-time classes (DCLS)
    ("ODD5", RESIDUE),           # residue kernel, LDS class file (unbalanced plan)
    ("ODD16", RESIDUE),          # K = 16: two candidates per lane (V = 32)
    ("NONINT8", GOERTZEL),       # off-bin tones
    ("FSK2_FREQS", GOERTZEL),    # K = 2 all-reduce path
    ("FSK8_FREQS", FFT),         # FFT detector's row pick
])
def test_near_ties_follow_exact_argmax(A, O, torch, plan, method):
    freqs = {"FSK8_FREQS": A.FSK8_FREQS, "FSK8_ODD": FSK8_ODD, "NONINT8": NONINT8,
             "FSK2_FREQS": A.FSK2_FREQS, "ODD5": FSK8_ODD[:5],
             "ODD16": tuple(46.875 * (32 + 9 * i) for i in range(16))}[plan]
    W = 4000
    x, pairs = near_tie_windows(freqs, W, seed=zlib.crc32(f"{plan}/{method}".encode()))
    with A.Demodulator(freqs=freqs, method=method) as d:
        assert d.method == method
        sym, mag = d.batch(x, mags=True)
        tau = d.rescue_tau
        tau64 = d.rescue_tau64
    assert tau64 > 0
    oracle = O.fft_demod if method == FFT else O.goertzel
    ref_sym, ref_P = oracle(x, freqs, 1024)
    in_band = check_decisions(sym, mag, ref_sym, ref_P)
    # the test must reach the band it is about: realised fp32 power ratios
    # within 2^-19 of each other, with the larger power on the higher index
    m = mag.astype(np.float64)
    top2 = np.sort(m, axis=1)[:, -2:]
    rel = (top2[:, 1] - top2[:, 0]) / np.maximum(top2[:, 1], 1e-30)
    hi_wins = pairs.max(axis=1) == sym
    tight = (rel < 2.0 ** -19) & (rel > 0)
    assert tight.sum() >= 20, tight.sum()
    assert (tight & hi_wins).sum() >= 5, (tight & hi_wins).sum()
    assert in_band > 0
    # windows whose oracle margin is well inside the rescue threshold tau
    # sqrt(NE P_max) (NE the window's energy scale, the folded window's for
    # the fold detector) were rescued: their powers are double
    # powers rounded to fp32 (the first pass's, or the oracle's own exactly)
    xw = x.reshape(W, 1024).astype(np.float64)
    if method == FOLDED:
        xf = xw.reshape(W, 8, 128).sum(axis=1)
        NE = 128.0 * (xf * xf).sum(axis=1)
    else:
        NE = 1024.0 * (xw * xw).sum(axis=1)
    Ps = np.sort(ref_P, axis=1)
    sure = (Ps[:, -1] - Ps[:, -2]) < 0.5 * tau * np.sqrt(NE * Ps[:, -1])
    assert sure.sum() >= 20
    ref32 = ref_P[sure].astype(np.float32).view(np.int32)
    # the in-kernel rescue's first pass decides most of them from its own
    # double powers: each within its derived bound of the oracle's,
    # |sqrt P_0 - sigma P_oracle| <= rho_first sqrt(sum x^2) (tests/
    # test_rescue_model64.py), then rounded to fp32 (half an ulp: 2^-24
    # relative in P, 2^-25 in sqrt P)
    m = A.error_model(A.make_cfg(freqs=freqs, method=method))
    assert m["tau64"] == pytest.approx(tau64, rel=1e-12)
    e_raw = (xw[sure] * xw[sure]).sum(axis=1)[:, None]   # the raw window's (fold too)
    g = mag[sure].astype(np.float64)
    sig = np.sign(ref_P[sure]) * np.sqrt(np.abs(ref_P[sure]))
    bound = m["rho_first"] * np.sqrt(e_raw) + 2.0 ** -24 * np.sqrt(g)
    assert (np.abs(np.sqrt(g) - sig) <= bound).all()
    # with that pass off every rescued window takes the exact chain (the
    # double FFT for the FFT detector): the oracle's powers rounded to fp32,
    # bit for bit, and the same symbols
    with env(FSKD_RESCUE_SEG="0"):
        with A.Demodulator(freqs=freqs, method=method) as d:
            assert d.rescue_tau64 == 0.0
            sym_x, mag_x = d.batch(x, mags=True)
    assert np.array_equal(sym_x, sym)
    assert np.array_equal(mag_x[sure].view(np.int32), ref32)
    # the same windows decided in fp32 alone: some differ from the oracle
    with env(FSKD_NO_RESCUE="1"):
        with A.Demodulator(freqs=freqs, method=method) as d:
            sym32 = d.batch(x)
    assert (sym32 & 0x80).sum() == 0
    assert (sym32 != ref_sym).sum() > 0
    assert (sym32 == sym).mean() > 0.9


@contextlib.contextmanager
def env(**kv):
    """Measurement switches read at demod_create."""
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("plan,method", [("FSK2_FREQS", GOERTZEL), ("FSK8_FREQS", FOLDED),
                                         ("FSK8_ODD", RESIDUE), ("NONINT8", GOERTZEL),
                                         ("FSK8_FREQS", FFT)])
def test_rescue_double_ties_take_the_exact_chain(A, O, torch, plan, method):
    """Windows whose tone powers tie in exact arithmetic (a single impulse:
    |X_k| = its amplitude at every frequency; two impulses symmetric about the
    window's middle for pairs of tones) are inside the first pass's double
    band, so they reach the exact chain: symbols and every magnitude are the
    oracle's, bit for bit."""
    freqs = {"FSK2_FREQS": A.FSK2_FREQS, "FSK8_FREQS": A.FSK8_FREQS, "FSK8_ODD": FSK8_ODD,
             "NONINT8": NONINT8}[plan]
    rng = np.random.default_rng(zlib.crc32(plan.encode()))
    W = 512
    x = np.zeros((W, 1024), np.int16)
    pos = rng.integers(0, 1024, W)
    x[np.arange(W), pos] = rng.integers(1000, 30000, W) * rng.choice([-1, 1], W)
    with A.Demodulator(freqs=freqs, method=method) as d:
        tau64 = d.rescue_tau64
        sym, mag = d.batch(x, mags=True)
    assert tau64 > 0
    ref_sym, ref_P = (O.fft_demod if method == FFT else O.goertzel)(x, freqs, 1024)
    assert np.array_equal(sym, ref_sym)
    assert np.array_equal(mag.view(np.int32), ref_P.astype(np.float32).view(np.int32))


@pytest.mark.parametrize("freqs,method,n,hop,expect", [
    ((1500.0, 3000.0), GOERTZEL, 1024, 1024, True),
    (tuple(1500.0 + 375.0 * i for i in range(8)), FOLDED, 1024, 1024, True),
    (FSK8_ODD, RESIDUE, 1024, 1024, True),
    ((46.875 * 1, 46.875 * 2), GOERTZEL, 1024, 1024, True),      # bin 1
    ((46.875 * 0.3, 1500.0), GOERTZEL, 1024, 1024, True),        # below bin 1
    ((1500.0, 3000.0), GOERTZEL, 1024, 256, True),               # SLIDE: the rescue launch's pass 0
    (tuple(1500.0 + 375.0 * i for i in range(8)), AUTO, 1024, 256, True),  # fold-slide, by the fold
    ((1500.0, 3000.0), GOERTZEL, 4096, 4096, False),             # n != 1024
    ((1500.0, 3000.0), FFT, 1024, 1024, True),                   # FFT: at its bins
    ((1500.0, 3000.0), FFT, 1024, 256, True),
    ((0.0, 3000.0), FFT, 1024, 1024, True),                      # a bin at DC: finite now
])
def test_rescue_tau64_is_the_stated_model(A, torch, freqs, method, n, hop, expect):
    """The handle's tau64 is the derived bound's (demod_error_model: 4
    rho_first / sqrt(n), rho_first checked by tests/test_rescue_model64.py),
    and 0 where no first pass runs (n != 1024)."""
    cfg = A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)
    with A.Demodulator(cfg) as d:
        t = d.rescue_tau64
    if expect:
        m = A.error_model(cfg)
        assert t > 0 and t == pytest.approx(m["tau64"], rel=1e-12)
        assert t == pytest.approx(4.0 * m["rho_first"] / 32.0, rel=1e-12)
    else:
        assert t == 0.0


@pytest.mark.parametrize("plan,method", [("FSK8_FREQS", FOLDED), ("FSK8_ODD", RESIDUE),
                                         ("FSK8_FREQS", GOERTZEL)])
def test_exact_fp32_ties_go_to_lowest_tone(A, torch, plan, method):
    """Windows with every tone at exactly 0 power (silence) — exact ties in
    fp32 and in double — decide the lowest tone, without a rescue."""
    freqs = A.FSK8_FREQS if plan == "FSK8_FREQS" else FSK8_ODD
    x = np.zeros((4, 1024), np.int16)
    with A.Demodulator(freqs=freqs, method=method) as d:
        sym, mag = d.batch(x, mags=True)
    assert (sym == 0).all() and (mag == 0).all()


@pytest.mark.parametrize("sigma", [400, 2000])
@pytest.mark.parametrize("plan", ["FSK2_FREQS", "FSK8_FREQS"])
def test_decision_margins_at_bench_levels(A, O, torch, sigma, plan):
    """The bench signal at sigma 400 (parity level) and 2000 (stress): count
    the windows whose oracle top-2 margin falls inside the fp32 band, and
    check every decision (the full-size bench stream uses the same generator)."""
    freqs = getattr(A, plan)
    W = 32768
    cfg = A.make_cfg(freqs=freqs)
    d_pcm = torch.empty((W, 1024), dtype=torch.int16, device="cuda")
    d_true = torch.empty(W, dtype=torch.uint8, device="cuda")
    d_sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    d_mag = torch.empty((W, len(freqs)), dtype=torch.float32, device="cuda")
    A.synth_fsk(cfg, A.BENCH_SEED ^ sigma, W, 8000, sigma, d_pcm, d_true)
    with A.Demodulator(cfg) as d:
        d.batch_device(d_pcm, W, d_sym, d_mag)
    ref_sym, ref_P = O.goertzel(d_pcm.cpu().numpy(), freqs, 1024, threads=8)
    sym, mag = d_sym.cpu().numpy(), d_mag.cpu().numpy()
    in_band = check_decisions(sym, mag, ref_sym, ref_P)
    print(f"\n{plan} sigma {sigma}: {in_band} of {W} windows inside the fp32 band, "
          f"{int((sym != d_true.cpu().numpy()).sum())} transmitted-symbol errors")
    if sigma == 400:
        assert in_band == 0 and (sym == d_true.cpu().numpy()).all()


@pytest.mark.parametrize("hop", [1024, 256, 200])
def test_fft_rescue_spectrum_is_the_oracles(A, O, torch, hop):
    """The FFT rescue (rescue_fft_kernel: the ten radix-2 stages in three
    register passes) re-runs the definition's butterflies on the same
    operands, so a rescued window's whole stored spectrum is the oracle's
    double spectrum rounded to fp32, bit for bit — on aligned near-tie
    windows and on the straddling windows of a sliding stream over them."""
    freqs = A.FSK8_FREQS
    x, _ = near_tie_windows(freqs, 800, seed=4242 + hop)
    flat = x.reshape(-1)
    W = (flat.size - 1024) // hop + 1
    with A.Demodulator(freqs=freqs, hop=hop, method=FFT) as d:
        tau = d.rescue_tau
        d_pcm = torch.from_numpy(flat.copy()).cuda()
        d_sym = torch.empty(W, dtype=torch.uint8, device="cuda")
        d_mag = torch.empty((W, len(freqs)), dtype=torch.float32, device="cuda")
        d_spec = torch.empty((W, 513), dtype=torch.float32, device="cuda")
        d.batch_spectrum_async(d_pcm, W, d_sym, d_mag, d_spec)
        torch.cuda.synchronize()
    sym, mag, spec = d_sym.cpu().numpy(), d_mag.cpu().numpy(), d_spec.cpu().numpy()
    ref_sym, ref_P = O.fft_demod(flat, freqs, 1024, hop)
    check_decisions(sym, mag, ref_sym, ref_P)
    Ps = np.sort(ref_P, axis=1)
    # well inside the threshold tau sqrt(NE P_max) (NE = n sum x^2 <= the
    # kernel's Parseval energy): flagged, hence rescued
    idx = np.arange(W)[:, None] * hop + np.arange(1024)[None, :]
    xw = flat[idx].astype(np.float64)
    NE = 1024.0 * (xw * xw).sum(axis=1)
    sure = np.flatnonzero((Ps[:, -1] - Ps[:, -2]) < 0.5 * tau * np.sqrt(NE * Ps[:, -1]))
    assert sure.size >= (20 if hop == 1024 else 5), sure.size
    full = np.stack([O.fft_power(flat[i * hop:i * hop + 1024]) for i in sure]).astype(np.float32)
    assert np.array_equal(spec[sure].view(np.uint32), full.view(np.uint32))
    assert np.array_equal(mag[sure].view(np.uint32), ref_P[sure].astype(np.float32).view(np.uint32))
