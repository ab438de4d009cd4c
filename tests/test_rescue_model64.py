"""The in-kernel rescue's first pass (demod_internal.h rescue_rows, pass 0),
its error model checked on the CPU.

Pass 0 re-computes a flagged window's K tone powers in double the way the
fp32 plain bank computes them: each of the row's 16 lanes runs every tone's
recurrence over its own 64 samples, rotates its end state into the window's
phase, and the row sums (xor butterfly). Those powers are not the oracle's
bits (the oracle runs one 1024-step chain per tone), so pass 0 decides a
window only where its top-2 margin clears tau64 sqrt(NE P_max), tau64 = 12
r64, and leaves the rest to the exact chain. That is safe when

    |P_pass0 - P_oracle| <= r64 sqrt(P_max NE) + r64^2 NE          (*)

on every window, with r64 the host's rescue_r64 (demod_api.cpp; mirrored by
r64() below and compared with the handle's demod_rescue_tau64 in
tests/test_gpu_decision.py). This file restates pass 0's arithmetic in numpy
operation for operation (contraction is off in the kernel, so every product
and sum is rounded once, as here; the row sum in the kernel's butterfly
order), runs it on the adversarial signal families of tests/error_model.py
for tone plans from 0.3 bins to 511.7 bins, and asserts (*) against the
double oracle (oracle/fsk_oracle.c through oracle.goertzel) with headroom.
Test infrastructure: imports the oracle as the checker only.
"""
import math

import numpy as np
import pytest

import error_model as EM

FS = 48000.0
N = 1024
BIN = FS / N

# tone plans (Hz): the survey's, off-bin, and the band edges where the double
# recurrences are worst conditioned (the oracle's own error grows like
# 1 / sin^2 w there)
PLANS = {
    "fsk2": (1500.0, 3000.0),
    "fsk8": tuple(1500.0 + 375.0 * i for i in range(8)),
    "nonint8": tuple(1234.5 + 1111.1 * i for i in range(8)),
    "bins_1_2": (1 * BIN, 2 * BIN),
    "bin_0p3_3": (0.3 * BIN, 3 * BIN),
    "nyq_511_510": (511 * BIN, 510 * BIN),
    "nyq_511p7_500": (511.7 * BIN, 500 * BIN),
}


def r64(freqs, fs=FS):
    """demod_api.cpp rescue_r64, restated."""
    s1 = math.sin(2 * math.pi / 1024)
    smin = min(1.0, min(abs(math.sin(2 * math.pi * f / fs)) for f in freqs))
    if smin < 1e-6:
        return 0.0
    r = 2.0 ** -30
    if smin < s1:
        r *= (s1 / smin) ** 2
    return r


def rot64(freqs):
    """The host's [k][16] (A, B) segment rotations, A = e^{-i w (64 j + 63)}."""
    w = 2 * np.pi * np.asarray(freqs, np.float64)[:, None] / FS
    j = np.arange(16)[None, :]
    a, b = -w * (64 * j + 63), -w * (64 * j + 64)
    return np.cos(a), np.sin(a), np.cos(b), np.sin(b)


def butterfly_sum16(v):
    """The kernel's row sum: v += shfl_xor(v, m), m = 1, 2, 4, 8 (every lane
    ends with the same value; lane 0's is returned)."""
    idx = np.arange(16)
    for m in (1, 2, 4, 8):
        v = v + v[:, idx ^ m]
    return v[:, 0]


def pass0_powers(x, freqs):
    """Pass 0's powers of W windows x[W][1024] (int16), operation for operation."""
    W = x.shape[0]
    xs = x.reshape(W, 16, 64).astype(np.float64)
    Ar, Ai, Br, Bi = rot64(freqs)
    P = np.empty((W, len(freqs)))
    for k, f in enumerate(freqs):
        c = 2.0 * math.cos(2.0 * math.pi * f / FS)
        s1 = np.zeros((W, 16))
        s2 = np.zeros((W, 16))
        for i in range(64):
            s = xs[:, :, i] + c * s1
            s = s - s2
            s2, s1 = s1, s
        re = Ar[k] * s1
        im = Ai[k] * s1
        re = re - Br[k] * s2
        im = im - Bi[k] * s2
        re = butterfly_sum16(re)
        im = butterfly_sum16(im)
        P[:, k] = re * re + im * im
    return P


@pytest.mark.parametrize("plan", sorted(PLANS))
def test_pass0_error_model(O, plan):
    freqs = PLANS[plan]
    r = r64(freqs)
    assert r > 0
    worst = (0.0, None)
    for fi, fam in enumerate(EM.FAMILIES):
        W = 384
        x = EM.family(fam, freqs, N, W, seed=100 + fi).reshape(W, N)
        ref_sym, ref_P = O.goertzel(x, freqs, N, fs=FS, threads=4)
        P = pass0_powers(x, freqs)
        xw = x.astype(np.float64)
        NE = N * (xw * xw).sum(axis=1)
        Pm = ref_P.max(axis=1)
        bound = r * np.sqrt(Pm * NE) + r * r * NE
        ok = bound > 0
        dP = np.abs(P - ref_P).max(axis=1)
        assert (dP[~ok] == 0).all(), (fam, "zero-energy windows must give zero powers")
        ratio = (dP[ok] / bound[ok]).max() if ok.any() else 0.0
        if ratio > worst[0]:
            worst = (ratio, fam)
        # what pass 0 decides is the oracle's symbol
        Ps = np.sort(P, axis=1)
        tau = 12.0 * r
        decided = (Ps[:, -1] > 0) & ((Ps[:, -1] - Ps[:, -2]) ** 2 >= tau * tau * NE * Ps[:, -1]) \
            & (16.0 * Ps[:, -1] >= tau * tau * NE)
        sym0 = np.argmax(P, axis=1)
        assert (sym0[decided] == ref_sym[decided]).all(), fam
    print(f"\n{plan}: r64 {r:.3g}, worst |dP| / model {worst[0]:.3g} ({worst[1]})")
    # the model holds with >= 8x to spare (measured: <= ~1/50 at bins 1 and 511)
    assert worst[0] <= 0.125, worst


@pytest.mark.parametrize("plan", ["fsk2", "fsk8", "bins_1_2", "nyq_511_510"])
def test_fft_pass0_error_model(O, plan):
    """The FFT detector's first pass (rescue_fft.h rescue_fft_seg): the same
    segmented recurrence at its tone bins' frequencies, against the oracle's
    double radix-2 FFT powers of those bins (oracle.fft_demod)."""
    bins = [round(f * N / FS) for f in PLANS[plan]]
    freqs = tuple(b * FS / N for b in bins)
    r = r64(freqs)
    worst = (0.0, None)
    for fi, fam in enumerate(EM.FAMILIES):
        W = 384
        x = EM.family(fam, freqs, N, W, seed=200 + fi).reshape(W, N)
        ref_sym, ref_P = O.fft_demod(x, PLANS[plan], N)
        P = pass0_powers(x, freqs)
        xw = x.astype(np.float64)
        NE = N * (xw * xw).sum(axis=1)
        Pm = ref_P.max(axis=1)
        bound = r * np.sqrt(Pm * NE) + r * r * NE
        ok = bound > 0
        dP = np.abs(P - ref_P).max(axis=1)
        ratio = (dP[ok] / bound[ok]).max() if ok.any() else 0.0
        if ratio > worst[0]:
            worst = (ratio, fam)
    print(f"\nfft {plan}: r64 {r:.3g}, worst |dP| / model {worst[0]:.3g} ({worst[1]})")
    assert worst[0] <= 0.125, worst
