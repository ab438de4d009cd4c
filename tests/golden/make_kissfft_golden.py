#!/usr/bin/env python3
"""Regenerate tests/golden/ref_kissfft.npz: outputs of the REFERENCE's own FFT.

    make -f oracle/ref.mk && python tests/golden/make_kissfft_golden.py
    (from the repo root, in the container that has /root/reference)

opus_fft_c (hardware/lib/libopus/src/celt/kiss_fft.c:569-589), compiled in
place from /root/reference with the reference's own config.h (fixed point, no
custom modes) by oracle/ref.mk into oracle/_ref/libkissfft_ref.so, run on
seeded int16 frames for each of its four static sizes (480, 240, 120, 60).
Stored per size N: the input frames x<N> (int16 [F][N]) and the reference's
raw complex output re<N>, im<N> (float64 [F][N]: X/N in its fixed point,
inputs pre-shifted by KISSFFT_PRESHIFT). Plain arrays (allow_pickle=False).

N = 1024, the north-star window, comes from the same kiss_fft.c compiled with
the libopus configure option CUSTOM_MODES (oracle/_ref/libkissfft_custom.so,
oracle/kissfft_custom_harness.c: opus_fft_alloc(1024) + opus_fft_c).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def frames(n: int) -> np.ndarray:
    """Seeded test frames of n samples: 2-FSK and 8-FSK symbols, full-scale
    noise, DC, near-Nyquist, an impulse and a low-level signal."""
    rng = np.random.default_rng(0xF17 + n)
    fs = 48000.0
    rows = []
    p2, _ = O.synth_fsk((1500.0, 3000.0), n, 4, 0x2C5DA044 + n, 8000, 400)
    p8, _ = O.synth_fsk(tuple(1500.0 + 375.0 * i for i in range(8)), n, 4, 0x2C5DA045 + n, 8000, 400)
    rows += list(p2) + list(p8)
    rows.append(rng.integers(-32768, 32768, n))
    rows.append(np.full(n, 12345))
    rows.append(np.round(30000 * np.cos(np.pi * 0.97 * np.arange(n))))
    imp = np.zeros(n)
    imp[n // 3] = 20000
    rows.append(imp)
    rows.append(rng.integers(-50, 51, n))
    t = np.arange(n)
    rows.append(np.round(9000 * np.sin(2 * np.pi * 2250.0 / fs * t + 0.7)))  # off-bin tone at n=480
    return np.stack([np.asarray(r, np.int64) for r in rows]).clip(-32768, 32767).astype(np.int16)


def main():
    if O.ref_kissfft() is None:
        sys.exit("oracle/_ref/libkissfft_ref.so missing: run `make -f oracle/ref.mk` first")
    out = {"preshift": np.int32(O.KISSFFT_PRESHIFT)}
    for which in range(4):
        n = O.ref_kissfft().ref_fft_static_size(which)
        x = frames(n)
        y = np.stack([O.ref_fft_static(which, row) for row in x])
        out[f"x{n}"] = x
        out[f"re{n}"] = y.real
        out[f"im{n}"] = y.imag
        print(f"kfft[{which}]: nfft {n}, {len(x)} frames")
    if O.ref_kissfft_custom() is None:
        sys.exit("oracle/_ref/libkissfft_custom.so missing: run `make -f oracle/ref.mk` first")
    n = 1024
    x = frames(n)
    y = np.stack([O.ref_fft_custom(row) for row in x])
    out[f"x{n}"] = x
    out[f"re{n}"] = y.real
    out[f"im{n}"] = y.imag
    print(f"custom: nfft {n}, {len(x)} frames")
    np.savez_compressed(os.path.join(HERE, "ref_kissfft.npz"), **out)


if __name__ == "__main__":
    main()
