#!/usr/bin/env python3
"""fp32 emulation of the plain tone bank's 64-sample segment chains
(goertzel.hip): |P_fp32 - P| / P for one tone, 2cos(w) form vs the
Reinsch-modified form (RS), against a double-precision direct DFT; and the
fold kernel's 8-sample chains over folded windows (fold.hip). Each fp32
operation is rounded as the kernel rounds it (fma = one rounding). Basis of
the kReinschSin = 0.1 switch in demod_api.cpp.

    python scripts/fp32_goertzel_error.py > profiles/round1/fp32_goertzel_error.log
"""
import numpy as np

f32 = np.float32


def fl(v):
    return float(f32(v))


def chain_2cos(x, w, L):
    c = fl(2 * np.cos(w))
    xr = xi = 0.0
    for j in range(x.size // L):
        s1 = s2 = 0.0
        for v in x[j * L:(j + 1) * L]:
            s1, s2 = fl(c * s1 + fl(v - s2)), s1
        a, b = -w * (L * j + L - 1), -w * (L * j + L)
        xr = fl(xr + fl(fl(np.cos(a)) * s1 - fl(np.cos(b)) * s2))
        xi = fl(xi + fl(fl(np.sin(a)) * s1 - fl(np.sin(b)) * s2))
    return xr * xr + xi * xi


def chain_reinsch(x, w, L):
    sg = 1.0 if np.cos(w) >= 0 else -1.0
    lam = fl(-4 * np.sin(w / 2) ** 2) if sg > 0 else fl(4 * np.cos(w / 2) ** 2)
    xr = xi = 0.0
    for j in range(x.size // L):
        s = d = 0.0
        for v in x[j * L:(j + 1) * L]:
            d = fl(lam * s + fl(sg * d + v))
            s = fl(sg * s + d)
        A, B = np.exp(-1j * w * (L * j + L - 1)), np.exp(-1j * w * (L * j + L))
        C1, C2 = A - sg * B, sg * B
        xr = fl(xr + fl(fl(C1.real) * s + fl(C2.real) * d))
        xi = fl(xi + fl(fl(C1.imag) * s + fl(C2.imag) * d))
    return xr * xr + xi * xi


def dft_power(x, w):
    return abs(np.sum(x * np.exp(-1j * w * np.arange(x.size)))) ** 2


def signal(rng, n, w):
    a = rng.choice([300, 8000, 30000])
    t = np.arange(n)
    return np.clip(np.round(a * np.cos(w * t + rng.uniform(0, 6)) + rng.normal(0, 50, n)),
                   -32768, 32767)


def main():
    rng = np.random.default_rng(1)
    print("plain bank, 64-sample chains: max over 3 signals of |P_fp32 - P| / P")
    print(f"{'n':>5} {'bin':>7} {'|sin w|':>8} {'2cos(w)':>9} {'Reinsch':>9}")
    for n in (256, 1024, 4096):
        h = n // 2
        for b in (0.5, 1, 2, 3, 5, 8, 13, 21, 34, n // 4 - 0.3, h - 13, h - 5, h - 2, h - 1, h - 0.5):
            w = 2 * np.pi * b / n
            e1 = e2 = 0.0
            for _ in range(3):
                x = signal(rng, n, w)
                P = dft_power(x, w)
                e1 = max(e1, abs(chain_2cos(x, w, 64) - P) / P)
                e2 = max(e2, abs(chain_reinsch(x, w, 64) - P) / P)
            print(f"{n:5d} {b:7.1f} {abs(np.sin(w)):8.3f} {e1:9.2e} {e2:9.2e}", flush=True)
    print("\nfold kernel, 8-sample chains over the 8-fold window (bins on multiples of 8)")
    print(f"{'n':>5} {'bin':>7} {'|sin w|':>8} {'2cos(w)':>9}")
    for n in (512, 1024, 4096):
        h = n // 2
        for b in (8, 16, 24, h - 16, h - 8):
            w = 2 * np.pi * b / n
            e = 0.0
            for _ in range(3):
                x = signal(rng, n, w)
                P = dft_power(x, w)
                e = max(e, abs(chain_2cos(x.reshape(8, n // 8).sum(0), w, 8) - P) / P)
            print(f"{n:5d} {b:7d} {abs(np.sin(w)):8.3f} {e:9.2e}", flush=True)


if __name__ == "__main__":
    main()
