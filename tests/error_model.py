"""The fp32 error model behind the decision rescue, measured window by window.

DESIGN.md §2a: a detector's fp32 tone power carries an error
    |P_gpu - P_ref| <= r sqrt(P_max NE) + r^2 NE              (*)
with NE the energy scale of the window the detector transforms (n sum x^2;
the fold detector: (n/8) sum xf^2 of the N/8-folded window) and r the
detector's bound for the tone plan; the kernels flag a window when its fp32
top-2 margin is below tau sqrt(NE P_max), tau = 12 r (a margin carries two
powers' errors, x 6 safety), or P_max < tau^2 NE / 16, and the rescue
re-decides flagged windows in double. r = tau / 12 comes from the handle
(demod_rescue_tau), so what is checked is the constant the shipped kernels
use, for the plan they run.

evaluate() runs one detector configuration on one signal family with the
rescue's flags kept but the rescue itself off (FSKD_NO_RESCUE=flags: every
magnitude is the kernel's fp32 value) and checks, on every window:
  1. the model (*) with the handle's r (reports the worst ratio, and the
     worst error as a fraction of tau);
  2. the kernel flags exactly the windows the stated threshold selects
     (within 1e-3 of it, the fp32 rounding of the test itself; the FFT's
     stage-2 energy is Parseval's 2 sum_{b<=512} P_b, between NE and 2 NE),
     and every window whose fp32 tone powers are all exactly 0 unless it is
     digital silence;
  3. every window it leaves unflagged carries the oracle's symbol.
Test infrastructure: only tests/ and bench.py's checker legs import this.
"""
import os

import numpy as np

FS = 48000.0
BIN = FS / 1024

# (name, freqs, n, hop, method, notes): detector paths x tone plans. method:
# 1 plain bank, 2 FFT, 3 fold, 4 residue (demod.h DEMOD_METHOD_*)
CASES = [
    ("plain_k2", (1500.0, 3000.0), 1024, 1024, 1),
    ("plain_k8_nonint", tuple(1500.0 + 377.3 * i for i in range(8)), 1024, 1024, 1),
    # one bin outside the Reinsch switch (|sin w| = 0.104 > 0.1): the plan factor
    ("plain_edge_lo", (17 * BIN, 34 * BIN), 1024, 1024, 1),
    # a near-Nyquist pair, both outside the switch
    ("plain_nyquist_pair", (495 * BIN, 490 * BIN), 1024, 1024, 1),
    ("plain_reinsch", (3 * BIN, 509 * BIN), 1024, 1024, 1),
    ("plain_n4096", (1500.0, 3000.0), 4096, 4096, 1),
    ("plain_n256", (1500.0, 3000.0), 256, 256, 1),
    ("plain_slide_h256", (1500.0, 3000.0), 1024, 256, 1),
    ("plain_k8_slide_h256", tuple(1500.0 + 377.3 * i for i in range(8)), 1024, 256, 1),
    ("fold_f16_k8", tuple(1500.0 + 375.0 * i for i in range(8)), 1024, 1024, 3),
    ("fold_k2", (1500.0, 3000.0), 1024, 1024, 3),
    ("fold_edge", (24 * BIN, 488 * BIN, 32 * BIN), 1024, 1024, 3),
    ("fold_n4096", tuple(1500.0 + 375.0 * i for i in range(8)), 4096, 4096, 3),
    ("fold_n256", (1500.0, 3000.0), 256, 256, 3),
    ("fold_slide_k8_h256", tuple(1500.0 + 375.0 * i for i in range(8)), 1024, 256, 3),
    ("residue_dcls_k8", tuple(BIN * (32 + 9 * i) for i in range(8)), 1024, 1024, 4),
    ("residue_lds_k5", tuple(BIN * (32 + 9 * i) for i in range(5)), 1024, 1024, 4),
    ("residue_n4096", tuple(FS / 4096 * (128 + 9 * i) for i in range(8)), 4096, 4096, 4),
    ("residue_n256", tuple(FS / 256 * (8 + 3 * i) for i in range(5)), 256, 256, 4),
    ("fft_h1024", (1500.0, 3000.0), 1024, 1024, 2),
    ("fft_h256_k8", tuple(1500.0 + 375.0 * i for i in range(8)), 1024, 256, 2),
]

FAMILIES = ["fsk_s400", "fsk_s0", "fsk_full_s2000", "clipped_square", "dc_tone", "random_full",
            "quiet_s3", "two_tone_equal", "phase_flip", "near_nyquist_tone"]


def family(name, freqs, n, blocks, seed):
    """`blocks` consecutive n-sample symbols of one signal family as one int16
    stream (windows at hop < n straddle them)."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    K = len(freqs)
    t = np.arange(n)
    f = np.asarray(freqs, np.float64)
    if name.startswith("fsk"):
        amp, sig = {"fsk_s400": (8000, 400), "fsk_s0": (8000, 0), "fsk_full_s2000": (32767, 2000)}[name]
        pcm, _ = O.synth_fsk(freqs, n, blocks, seed, amplitude=amp, sigma=sig, fs=FS)
        return pcm.reshape(-1)
    sym = rng.integers(0, K, blocks)
    ph = rng.uniform(0, 2 * np.pi, (blocks, 1))
    w = 2 * np.pi * f[sym][:, None] / FS
    if name == "clipped_square":       # full-scale square waves at a plan tone
        v = np.where(np.sin(w * t + ph) >= 0, 32767.0, -32768.0)
    elif name == "dc_tone":            # a DC offset under a tone
        v = rng.uniform(-16000, 16000, (blocks, 1)) + 8000 * np.sin(w * t + ph)
    elif name == "random_full":        # uniform full-scale int16
        return rng.integers(-32768, 32768, blocks * n).astype(np.int16)
    elif name == "quiet_s3":           # dithered silence / idle-channel noise
        v = rng.normal(0, 3, (blocks, n))
    elif name == "two_tone_equal":     # two plan tones at equal amplitude: near ties
        s2 = (sym + 1 + rng.integers(0, max(K - 1, 1), blocks)) % K
        w2 = 2 * np.pi * f[s2][:, None] / FS
        v = 12000 * (np.sin(w * t + ph) + np.sin(w2 * t + rng.uniform(0, 2 * np.pi, (blocks, 1))))
    elif name == "phase_flip":         # a tone cancelling itself across the window
        v = 8000 * np.sin(w * t + ph + np.where(t >= n // 2, np.pi, 0.0)) + rng.normal(0, 50, (blocks, n))
    elif name == "near_nyquist_tone":  # a strong tone at 23.9 kHz beside a plan tone
        v = 20000 * np.sin(2 * np.pi * 23900.0 / FS * t + ph) + 6000 * np.sin(w * t)
    else:
        raise ValueError(name)
    return np.clip(np.round(v), -32768, 32767).astype(np.int16).reshape(-1)


def window_energy(x, n, hop, W, fold):
    """NE per window: n sum x^2, or (n/8) sum xf^2 of the N/8-folded window."""
    idx = np.arange(W)[:, None] * hop + np.arange(n)[None, :]
    xw = x[idx].astype(np.float64)
    if fold:
        xf = xw.reshape(W, 8, n // 8).sum(axis=1)
        return (n / 8) * (xf * xf).sum(axis=1)
    return n * (xw * xw).sum(axis=1)


def evaluate(A, O, case, fam, W=4096, threads=16, seed=1):
    name, freqs, n, hop, method = case
    blocks = -(-((W - 1) * hop + n) // n)
    x = family(fam, freqs, n, blocks, seed)[:(W - 1) * hop + n]
    old = os.environ.get("FSKD_NO_RESCUE")
    os.environ["FSKD_NO_RESCUE"] = "flags"
    try:
        d = A.Demodulator(A.make_cfg(n=n, hop=hop, freqs=freqs, method=method))
    finally:
        if old is None:
            del os.environ["FSKD_NO_RESCUE"]
        else:
            os.environ["FSKD_NO_RESCUE"] = old
    with d:
        got = int(d.method)
        tau = d.rescue_tau
        sym, mag = d.batch(x, n_windows=W, mags=True)
    fft = got == 2
    rs, rP = (O.fft_demod if fft else O.goertzel)(x, freqs, n, hop=hop, fs=FS, threads=threads)
    rs, rP = rs[:W], rP[:W]
    fold = got == 3
    NE = window_energy(x, n, hop, W, fold)
    r = tau / 12.0
    g = mag.astype(np.float64)
    dP = np.abs(g - rP).max(axis=1)
    Pm = rP.max(axis=1)
    bound = r * np.sqrt(Pm * NE) + r * r * NE
    ok = bound > 0
    ratio = np.zeros(W)
    ratio[ok] = dP[ok] / bound[ok]
    # the error as a fraction of tau's model (tau = 12 r): what fraction of
    # the margin threshold tau sqrt(P_max NE) (+ its second-order term) one
    # power's error uses
    frac_tau = ratio / 12.0
    zero_ne = ~ok
    # 2. the flags against the stated threshold, from the kernel's own powers
    flag = (sym & 0x80) != 0
    gs = np.sort(g, axis=1)
    p1 = gs[:, -1]
    p2 = gs[:, -2] if g.shape[1] > 1 else np.zeros(W)
    m = p1 - p2
    lo_ne, hi_ne = (NE, 2 * NE) if fft else (NE, NE)

    def sel(ne, s):
        c = tau * tau * ne * s
        return (p1 > 0) & ((m * m < c * p1) | (16 * p1 < c))
    must = sel(lo_ne, 0.999)     # below the threshold: flagged
    may = sel(hi_ne, 1.001)      # above it: not flagged
    # every fp32 tone power exactly 0: flagged unless the window is digital
    # silence (the oracle's powers are then its own rounding noise)
    raw = window_energy(x, n, hop, W, False)
    zero = (p1 == 0) & (raw > 0)
    must |= zero
    may |= zero
    if g.shape[1] < 2:
        must = may = np.zeros(W, bool)
    missed = np.flatnonzero(must & ~flag)
    extra = np.flatnonzero(flag & ~may)
    # 3. unflagged decisions equal the oracle's (digital silence: all powers 0
    # in fp32 and in double -> tone 0)
    silent = (g == 0).all(axis=1) & (raw == 0)
    wrong = np.flatnonzero(~flag & ~silent & ((sym & 0x7F) != rs))
    return {"case": name, "family": fam, "method": got, "windows": W, "tau": tau,
            "r": r, "worst_ratio_to_model": float(ratio.max()),
            "worst_err_frac_of_tau": float(frac_tau.max()),
            "windows_zero_energy": int(zero_ne.sum()),
            "flagged": int(flag.sum()), "flag_missed": int(missed.size), "flag_extra": int(extra.size),
            "unflagged_wrong": int(wrong.size),
            "_detail": (missed[:4].tolist(), extra[:4].tolist(), wrong[:4].tolist())}
