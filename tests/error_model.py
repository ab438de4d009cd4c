"""The decision rescue's derived error bounds, checked window by window on
the GPU.

DESIGN.md §2a (round 5): for each tone plan, audio-network_amd/csrc/
error_model.cpp derives from the kernels' operation sequences and fp32
constants (no measured constant; demod_error_model)
    |sqrt(P_gpu,k) - |X_k||      <= rho_det sqrt(E_det)
    |sigma(P_oracle,k) - |X_k||  <= rho_ref sqrt(sum x^2)
so on every window and tone
    |sqrt(P_gpu,k) - sigma(P_oracle,k)| <= rho_det sqrt(E_det) + rho_ref sqrt(sum x^2)   (*)
with E_det the energy the kernel sums (raw sum x^2; fold detector: sum xf^2
of the n/8 fold; FFT: raw, the kernel's own Parseval sum covering it). The
kernels flag a window when (P_1 - P_2)^2 < t2e E_eff P_1 (E_eff: raw sum x^2,
(sqrt(sum xf^2) + amb_d)^2 for the fold detector, Parseval's 2 sum_b P_b for
the FFT), or P_1 == 0 with E_eff > 0; the rescue re-decides flagged windows
in double.

evaluate() runs one detector configuration on one signal family with the
rescue's flags kept but the rescue itself off (FSKD_NO_RESCUE=flags: every
magnitude is the kernel's fp32 value) and checks, on every window:
  1. (*) (reports the worst ratio, and the worst sqrt-power error as a fraction
     of the flag threshold's sqrt margin);
  2. the kernel flags exactly the windows the stated threshold selects
     (within 1e-3 of it, the fp32 rounding of the test itself; the FFT's
     stage-2 energy lies between n sum x^2 and 2 n sum x^2);
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


def window_energies(x, n, hop, W):
    """(raw sum x^2, folded sum xf^2) per window, exact."""
    idx = np.arange(W)[:, None] * hop + np.arange(n)[None, :]
    xw = x[idx].astype(np.int64)
    xf = xw.reshape(W, 8, n // 8).sum(axis=1)
    return (xw * xw).sum(axis=1).astype(np.float64), (xf * xf).sum(axis=1).astype(np.float64)


def sigma(P):
    return np.sign(P) * np.sqrt(np.abs(P))


def evaluate(A, O, case, fam, W=4096, threads=16, seed=1):
    name, freqs, n, hop, method = case
    blocks = -(-((W - 1) * hop + n) // n)
    x = family(fam, freqs, n, blocks, seed)[:(W - 1) * hop + n]
    old = os.environ.get("FSKD_NO_RESCUE")
    os.environ["FSKD_NO_RESCUE"] = "flags"
    try:
        cfg = A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)
        d = A.Demodulator(cfg)
    finally:
        if old is None:
            del os.environ["FSKD_NO_RESCUE"]
        else:
            os.environ["FSKD_NO_RESCUE"] = old
    with d:
        got = int(d.method)
        tau = d.rescue_tau
        sym, mag = d.batch(x, n_windows=W, mags=True)
    m = A.error_model(cfg)
    fft = got == 2
    fold = got == 3
    rs, rP = (O.fft_demod if fft else O.goertzel)(x, freqs, n, hop=hop, fs=FS, threads=threads)
    rs, rP = rs[:W], rP[:W]
    e_raw, e_fold = window_energies(x, n, hop, W)
    e_det = e_fold if fold else e_raw
    g = mag.astype(np.float64)
    bound = m["rho_det"] * np.sqrt(e_det) + m["rho_ref"] * np.sqrt(e_raw)
    err = np.abs(np.sqrt(g) - sigma(rP)).max(axis=1)
    ok = bound > 0
    ratio = np.zeros(W)
    ratio[ok] = err[ok] / bound[ok]
    zero_e = ~ok
    assert (err[zero_e] == 0).all() if zero_e.any() else True
    # the flag test's sqrt margin is sqrt(t2e E_eff) / 2 = 2 bound (x safety):
    # one power's error as a fraction of it
    frac_tau = ratio / 2.0
    flag = (sym & 0x80) != 0
    gs = np.sort(g, axis=1)
    p1 = gs[:, -1]
    p2 = gs[:, -2] if g.shape[1] > 1 else np.zeros(W)
    mm = p1 - p2
    if fft:
        lo_e, hi_e = n * e_raw, 2 * n * e_raw
    elif fold:
        d_ = m["amb_d"]
        eff = np.where(e_fold > 0, (np.sqrt(e_fold) + d_) ** 2, np.where(e_raw > 0, d_ * d_, 0.0))
        lo_e = hi_e = eff
    else:
        lo_e = hi_e = e_raw

    def sel(e, s):
        c = m["t2e"] * e * s
        return (p1 > 0) & ((mm * mm < c * p1) | (16 * p1 < c))
    must = sel(lo_e, 0.999)     # below the threshold: flagged
    may = sel(hi_e, 1.001)      # above it: not flagged
    # every fp32 tone power exactly 0: flagged unless the window is digital
    # silence (the oracle's powers are then its own rounding noise)
    zero = (p1 == 0) & (e_raw > 0)
    must |= zero
    may |= zero
    if g.shape[1] < 2:
        must = may = np.zeros(W, bool)
    missed = np.flatnonzero(must & ~flag)
    extra = np.flatnonzero(flag & ~may)
    # 3. unflagged decisions equal the oracle's (digital silence: all powers 0
    # in fp32 and in double -> tone 0)
    silent = (g == 0).all(axis=1) & (e_raw == 0)
    wrong = np.flatnonzero(~flag & ~silent & ((sym & 0x7F) != rs))
    return {"case": name, "family": fam, "method": got, "windows": W, "tau": tau,
            "rho_det": m["rho_det"], "rho_ref": m["rho_ref"],
            "worst_ratio_to_model": float(ratio.max()),
            "worst_err_frac_of_tau": float(frac_tau.max()),
            "windows_zero_energy": int(zero_e.sum()),
            "flagged": int(flag.sum()), "flag_missed": int(missed.size), "flag_extra": int(extra.size),
            "unflagged_wrong": int(wrong.size),
            "_detail": (missed[:4].tolist(), extra[:4].tolist(), wrong[:4].tolist())}
