"""Measure the fp32 error scale of every detector against the double oracle.

For the decision rescue: a window's fp32 decision can differ
from the exact one only if its top-2 margin is within the error of the two
powers. The error of P_k is modelled as |dP_k| <= r * sqrt(P_max * NE) with
NE = n * sum(x^2) (the window's energy scale: |X_k|^2 <= NE by Cauchy-Schwarz);
for the fold detector NE = (n/8) * sum(xf^2), the folded window's (round 4).
This prints, per detector and signal family, the largest r seen over all
windows and tones, and the largest |dP| / NE (the second-order term).

Usage (GPU box): python scripts/precision_probe.py [--windows W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402
from oracle import oracle as O  # noqa: E402

A = load_pkg()
FS = 48000.0
THREADS = 16


def signals(n, freqs, W, rng):
    """(name, pcm [W*n] int16 flat) families."""
    out = []
    for amp, sig in ((8000, 400), (8000, 2000), (8000, 0), (32767, 2000), (30, 10), (3, 1),
                     (0, 2000), (0, 1)):
        pcm, _ = O.synth_fsk(freqs, n, W, seed=0x51 + amp + sig, amplitude=amp, sigma=sig, fs=FS)
        out.append((f"fsk_a{amp}_s{sig}", pcm.reshape(-1)))
    out.append(("uniform_full", rng.integers(-32768, 32768, W * n, dtype=np.int64)
                .astype(np.int16)))
    # half-half same-tone phase flip (cancellation inside a window at hop n/2)
    t = np.arange(W * n)
    f0 = freqs[0]
    ph = np.where((t // (n // 2)) % 2 == 0, 0.0, np.pi)
    x = np.round(8000 * np.sin(2 * np.pi * f0 * t / FS + ph) + rng.normal(0, 50, t.size))
    out.append(("phase_flip", np.clip(x, -32768, 32767).astype(np.int16)))
    return out


def run_case(name, freqs, n, hop, method, W, rng, fft=False):
    cfg = A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)
    rows = []
    with A.Demodulator(cfg) as d:
        for sname, flat in signals(n, freqs, W, rng):
            nw = (flat.size - n) // hop + 1
            nw = min(nw, W)
            need = (nw - 1) * hop + n
            x = np.ascontiguousarray(flat[:need])
            sym, mag = d.batch(x, n_windows=nw, mags=True)
            if fft:
                rs, rP = O.fft_demod(x, freqs, n, hop=hop, fs=FS, threads=THREADS)
            else:
                rs, rP = O.goertzel(x, freqs, n, hop=hop, fs=FS, threads=THREADS)
            rP = rP[:nw]
            idx = np.arange(nw)[:, None] * hop + np.arange(n)[None, :]
            xw = x[idx].astype(np.float64)
            NE = n * (xw * xw).sum(axis=1)
            if int(d.method) == 3:
                # round 4: the fold detector's energy scale is that of the
                # folded window it transforms, (n/8) sum xf^2 (<= NE)
                xf = xw.reshape(nw, 8, n // 8).sum(axis=1)
                NE = (n / 8) * (xf * xf).sum(axis=1)
            P1 = rP.max(axis=1)
            dP = np.abs(mag.astype(np.float64) - rP).max(axis=1)
            ok = NE > 0
            r = np.zeros(nw)
            r[ok] = dP[ok] / np.sqrt(np.maximum(P1[ok], 1e-300) * NE[ok])
            q = np.zeros(nw)
            q[ok] = dP[ok] / NE[ok]
            Q = float(n) * n * 2.0 ** 30
            rq = dP / np.sqrt(np.maximum(P1, 1e-300) * Q)
            rel = dP / np.maximum(P1, 1e-300)
            i = int(np.argmax(r))
            rows.append({
                "case": name, "signal": sname, "windows": int(nw),
                "method": int(d.method), "r_max": float(r.max()),
                "r_p9999": float(np.quantile(r, 0.9999)),
                "q_max": float(q.max()), "rQ_max": float(rq[P1 > 0].max()) if (P1 > 0).any() else 0.0,
                "rel_maxP_max": float(rel[P1 > 0].max()) if (P1 > 0).any() else 0.0,
                "at_r_max": {"P1_over_NE": float(P1[i] / NE[i]) if NE[i] else 0.0},
                "sym_diff": int((sym != rs[:nw]).sum()),
            })
            print(json.dumps(rows[-1]), flush=True)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=8192)
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    W = a.windows
    f2 = A.FSK2_FREQS
    f8 = A.FSK8_FREQS
    nonint8 = tuple(1500.0 + 377.3 * i for i in range(8))
    odd8 = tuple(48000.0 / 1024 * (32 + 9 * i) for i in range(8))
    k5 = tuple(48000.0 / 1024 * (32 + 9 * i) for i in range(5))
    edge2 = (48000.0 / 1024 * 1.5, 48000.0 / 1024 * 510.5)
    cases = [
        ("plain_k2", f2, 1024, 1024, A.METHOD_GOERTZEL, False),
        ("plain_k2_n256", (1500.0, 3000.0), 256, 256, A.METHOD_GOERTZEL, False),
        ("plain_k2_n4096", f2, 4096, 4096, A.METHOD_GOERTZEL, False),
        ("plain_k8_nonint", nonint8, 1024, 1024, A.METHOD_GOERTZEL, False),
        ("plain_k2_reinsch", edge2, 1024, 1024, A.METHOD_GOERTZEL, False),
        ("slide_k2_h256", f2, 1024, 256, A.METHOD_GOERTZEL, False),
        ("slide_k8_h256", nonint8, 1024, 256, A.METHOD_GOERTZEL, False),
        ("direct_k2_h264", f2, 1024, 264, A.METHOD_GOERTZEL, False),
        ("fold_k2", f2, 1024, 1024, A.METHOD_FOLDED, False),
        ("fold_f16_k8", f8, 1024, 1024, A.METHOD_FOLDED, False),
        ("fold_slide_k8_h256", f8, 1024, 256, A.METHOD_FOLDED, False),
        ("residue_k8_dcls", odd8, 1024, 1024, A.METHOD_RESIDUE, False),
        ("residue_k5_lds", k5, 1024, 1024, A.METHOD_RESIDUE, False),
        # round 4: fold and residue at other window lengths
        ("fold_k2_n256", (1500.0, 3000.0), 256, 256, A.METHOD_FOLDED, False),
        ("fold_k8_n4096", f8, 4096, 4096, A.METHOD_FOLDED, False),
        ("residue_k5_n256", tuple(187.5 * (8 + 3 * i) for i in range(5)), 256, 256, A.METHOD_RESIDUE, False),
        ("residue_k8_n4096", tuple(48000.0 / 4096 * (128 + 9 * i) for i in range(8)), 4096, 4096,
         A.METHOD_RESIDUE, False),
        ("fft_h1024", f2, 1024, 1024, A.METHOD_FFT, True),
        ("fft_h256", f8, 1024, 256, A.METHOD_FFT, True),
    ]
    allrows = []
    t0 = time.time()
    for name, fr, n, hop, m, fft in cases:
        allrows += run_case(name, fr, n, hop, m, W, rng, fft)
    summary = {}
    for r in allrows:
        s = summary.setdefault(r["case"], {"r_max": 0.0, "q_max": 0.0, "rQ_max": 0.0})
        s["r_max"] = max(s["r_max"], r["r_max"])
        s["q_max"] = max(s["q_max"], r["q_max"])
        s["rQ_max"] = max(s["rQ_max"], r["rQ_max"])
    print(json.dumps({"summary": summary, "r_max_all": max(s["r_max"] for s in summary.values()),
                      "seconds": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
