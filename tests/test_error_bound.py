"""The decision rescue's derived error bounds (VERDICT r4 item
1), checked on the CPU window by window.

audio-network_amd/csrc/error_model.cpp derives, for each tone plan, from the
kernels' operation sequences and fp32 constants (no measured constant):
  (1) |sqrt(P_fp32,k) - |X_k||     <= rho_det sqrt(E_det)
  (2) |sigma(P_oracle,k) - |X_k||  <= rho_ref sqrt(sum x^2)
with X_k the exact DFT at the tone (the fold / residue detectors: at its bin),
E_det the energy the kernel sums (raw sum x^2, or sum xf^2 of the n/8 fold).
Here the detectors' fp32 arithmetic is emulated operation for operation
(tests/fp32emu.py; a GPU test ties the emulation to the kernels bit for bit),
X_k is evaluated in long double, the oracle is oracle/fsk_oracle.c, and both
bounds must dominate on every window of the adversarial signal families of
tests/error_model.py plus worst-case inputs built from the bound's own
structure (sign patterns of the tone, full-scale). The worst measured / bound
ratios are printed: the bound is a worst case, typically 10-50x above the
observed error.
"""
import numpy as np
import pytest

import error_model as EM
import fp32emu as E

FS = 48000.0
BIN = FS / 1024

# detector paths x plans: error_model.CASES (direct windows; the segment-
# shared kernels are bit-identical to direct evaluation) and the band edges
CASES = [c for c in EM.CASES if c[4] != 2] + [
    ("fold_dc_nyq", (0.0, 8 * BIN, 512 * BIN), 1024, 1024, 3),
    ("residue_dc_nyq_k5", (0.0, 3 * BIN, 100 * BIN, 509 * BIN, 512 * BIN), 1024, 1024, 4),
    ("plain_bins_1_2", (1 * BIN, 2 * BIN), 1024, 1024, 1),
    ("plain_k16_n4096", tuple(700.0 + 1234.5 * i for i in range(16)), 4096, 4096, 1),
    ("residue_k16_n1024", tuple(BIN * (20 + 7 * i) for i in range(16)), 1024, 1024, 4),
]
FAMILIES = EM.FAMILIES + ["worst_sign", "alt_full"]


def family(name, freqs, n, blocks, seed):
    """error_model.family plus two inputs aimed at the bound: full-scale sign
    patterns of a plan tone (every chain state at its maximum, the windows'
    energy all at the tone), and a full-scale +-32767 alternation."""
    if name == "worst_sign":
        rng = np.random.default_rng(seed)
        t = np.arange(n)
        f = np.asarray(freqs)[rng.integers(0, len(freqs), blocks)]
        ph = rng.uniform(0, 2 * np.pi, (blocks, 1))
        v = np.where(np.cos(2 * np.pi * f[:, None] / FS * t + ph) >= 0, 32767, -32768)
        return v.astype(np.int16).reshape(-1)
    if name == "alt_full":
        t = np.arange(blocks * n)
        return np.where(t % 2 == 0, 32767, -32768).astype(np.int16)
    return EM.family(name, freqs, n, blocks, seed)


def sigma(P):
    return np.sign(P) * np.sqrt(np.abs(P))


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_derived_bounds_dominate(A, O, case):
    name, freqs, n, hop, method = case
    K = len(freqs)
    cfg = A.make_cfg(n=n, hop=n, freqs=freqs, method=method)
    info = A.plan_info(cfg)
    m = A.error_model(cfg)
    got = info["method"]
    assert got != 2
    W = 96 if n == 4096 else 192
    fold = got == 3
    bins = got in (3, 4)
    rc = np.asarray(info["rcoef"], np.float64)
    w_or = np.arccos(rc.astype(np.longdouble) / 2)
    w_b = 2 * E.PI_L * np.round(np.asarray(freqs) * n / FS).astype(np.longdouble) / n
    w_det = w_b if bins else w_or
    worst1 = worst2 = (0.0, None)
    for fi, fam in enumerate(FAMILIES):
        x = family(fam, freqs, n, W, 1000 + fi)[:W * n]
        P = E.detector_powers(info, x, n, n, W, K).astype(np.float64)
        _, Pr = O.goertzel(x, freqs, n, hop=n, fs=FS, threads=4)
        Pr = Pr[:W]
        e_raw, e_fold = E.energies(x, n, n, W)
        e_det = e_fold if fold else e_raw
        X = E.exact_dft_mag(x, n, n, W, w_det)
        b1 = np.broadcast_to(m["rho_det"] * np.sqrt(e_det)[:, None], P.shape)
        b2 = np.broadcast_to(m["rho_ref"] * np.sqrt(e_raw)[:, None], P.shape)
        d1 = np.abs(np.sqrt(P) - X)
        d2 = np.abs(sigma(Pr) - X)
        assert (d1 <= b1).all(), (fam, "detector", float((d1 / np.maximum(b1, 1e-300)).max()))
        assert (d2 <= b2).all(), (fam, "oracle", float((d2 / np.maximum(b2, 1e-300)).max()))
        ok = b1 > 0
        r1 = float((d1[ok] / b1[ok]).max()) if ok.any() else 0.0
        ok = b2 > 0
        r2 = float((d2[ok] / b2[ok]).max()) if ok.any() else 0.0
        if r1 > worst1[0]:
            worst1 = (r1, fam)
        if r2 > worst2[0]:
            worst2 = (r2, fam)
        # the decision the bound licenses is the oracle's: unflagged windows
        # under the kernel's own test carry the oracle's argmax
        if K >= 2:
            Ps = np.sort(P, axis=1)
            p1, p2 = Ps[:, -1], Ps[:, -2]
            e_eff = (np.sqrt(e_fold) + m["amb_d"]) ** 2 if fold else e_raw
            flag = (p1 == 0) & (e_raw > 0) | ((p1 > 0) & ((p1 - p2) ** 2 < m["t2e"] * e_eff * p1))
            sym = np.argmax(P, axis=1)
            ref = np.argmax(Pr, axis=1)
            assert (sym[~flag] == ref[~flag]).all(), fam
    print(f"\n{name}: rho_det {m['rho_det']:.3g} worst {worst1[0]:.3g} of it ({worst1[1]}); "
          f"rho_ref {m['rho_ref']:.3g} worst {worst2[0]:.3g} ({worst2[1]})")


def test_error_model_abi(A):
    """demod_error_model needs no device, rejects what demod_create rejects,
    and its thresholds are the bound's: t2e = 16 rho^2 (x the evaluation's
    safety), tau = sqrt(t2e / n_eff)."""
    cfg = A.make_cfg()
    m = A.error_model(cfg)
    assert m["method"] == A.METHOD_GOERTZEL and m["energy"] == A.ENERGY_RAW
    rho = m["rho_det"] + m["rho_ref"]
    assert 16 * rho ** 2 <= m["t2e"] <= 16 * rho ** 2 * 1.002
    assert abs(m["tau"] - np.sqrt(m["t2e"] / 1024)) <= 1e-12
    assert m["rho_first"] > 0 and m["t2e64"] >= 16 * m["rho_first"] ** 2
    f8 = A.error_model(A.make_cfg(freqs=A.FSK8_FREQS))
    assert f8["method"] == A.METHOD_FOLDED and f8["energy"] == A.ENERGY_FOLDED and f8["amb_d"] > 0
    ff = A.error_model(A.make_cfg(method=A.METHOD_FFT))
    assert ff["energy"] == A.ENERGY_PARSEVAL
    bad = A.make_cfg(n=1000)
    with pytest.raises(A.DemodError):
        A.error_model(bad)
    # every plan's bound is finite (round 4's fitted factor was infinite for a
    # fold plan with a tone at 0 Hz: ADVICE r4 medium)
    for f, meth in (((0.0, 8 * BIN, 512 * BIN), 3), ((0.0, 512 * BIN), 1), ((BIN * 0.01, 3000.0), 1)):
        mm = A.error_model(A.make_cfg(freqs=f, method=meth))
        assert np.isfinite(mm["tau"]) and mm["tau"] > 0, (f, mm)


def _exact_spectrum(xw):
    """|X_b|, b = 0..512, in long double (direct DFT)."""
    n = xw.shape[1]
    tb = np.outer(np.arange(n), np.arange(n // 2 + 1)) % n        # exact phase index
    ph = (2 * E.PI_L / n) * tb.astype(np.longdouble)
    xl = xw.astype(np.longdouble)
    re = xl @ np.cos(ph)
    im = xl @ np.sin(ph)
    return np.sqrt(re * re + im * im).astype(np.float64)


@pytest.mark.parametrize("plan", ["fsk2", "fsk8"])
def test_fft_bounds_dominate(A, O, plan):
    """The FFT detector (fft_quad.hip, emulated operation for operation by
    fp32emu.fft_spectrum): its structural bound on EVERY bin of the 513, and
    the double radix-2 oracle's (oracle_fft_power) against a long-double DFT."""
    freqs = A.FSK2_FREQS if plan == "fsk2" else A.FSK8_FREQS
    n = 1024
    m = A.error_model(A.make_cfg(freqs=freqs, method=A.METHOD_FFT))
    assert m["energy"] == A.ENERGY_PARSEVAL
    bins = np.round(np.asarray(freqs) * n / FS).astype(int)
    worst1 = worst2 = (0.0, None)
    for fi, fam in enumerate(FAMILIES):
        W = 24
        x = family(fam, freqs, n, W, 2000 + fi)[:W * n]
        xw = x.reshape(W, n)
        P = E.fft_spectrum(x, n, W).astype(np.float64)
        Pr = np.stack([O.fft_power(xw[i]) for i in range(W)])
        X = _exact_spectrum(xw)
        nrm = np.sqrt((xw.astype(np.float64) ** 2).sum(axis=1))[:, None]
        d1 = np.abs(np.sqrt(P) - X)
        d2 = np.abs(sigma(Pr) - X)
        b1, b2 = m["rho_det"] * nrm, m["rho_ref"] * nrm
        assert (d1 <= b1).all(), (fam, float((d1 / np.maximum(b1, 1e-300)).max()))
        assert (d2 <= b2).all(), (fam, float((d2 / np.maximum(b2, 1e-300)).max()))
        live = nrm[:, 0] > 0
        if live.any():
            r1 = float((d1[live] / b1[live]).max())
            r2 = float((d2[live] / b2[live]).max())
            worst1 = max(worst1, (r1, fam))
            worst2 = max(worst2, (r2, fam))
        # the kernel's test on its own powers (E = Parseval's 2 sum P): what
        # it leaves unflagged is the oracle's symbol
        Pt = P[:, bins]
        Ps = np.sort(Pt, axis=1)
        p1, p2 = Ps[:, -1], Ps[:, -2]
        epar = 2 * P.sum(axis=1)
        flag = ((p1 == 0) & (epar > 0)) | ((p1 > 0) & ((p1 - p2) ** 2 < m["t2e"] * epar * p1))
        assert (np.argmax(Pt, 1)[~flag] == np.argmax(Pr[:, bins], 1)[~flag]).all(), fam
    print(f"\nfft {plan}: rho_det {m['rho_det']:.3g} worst {worst1[0]:.3g} ({worst1[1]}); "
          f"rho_ref {m['rho_ref']:.3g} worst {worst2[0]:.3g} ({worst2[1]})")
