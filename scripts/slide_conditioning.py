#!/usr/bin/env python3
"""Conditioning of sliding windows: on the GPU-synthesised
2-FSK stream, the worst max_k |P - P_ref| / max_k P_ref per hop, for the
segment-shared path (hop 256) and the direct path (hop 1000, 264 — not
multiples of 64) and aligned windows (hop 1024). Windows that straddle a
symbol boundary can put both tone powers ~1e-4 below the window energy
N sum x^2 / 2, and fp32 error scales with that energy, so both paths exceed
1e-5 of max P on a few such windows while aligned windows stay ~3e-6.

    python scripts/slide_conditioning.py
"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
import bench
import oracle as O
A, _ = bench.load_pkg()
n, hop = 1024, 256
src = 1 << 14
cfg = A.make_cfg(freqs=A.FSK2_FREQS, n=n, hop=n)
d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
d_true = torch.empty(src, dtype=torch.uint8, device="cuda")
A.synth_fsk(cfg, 12345, src, 8000, 400, d_pcm, d_true)
x = d_pcm.cpu().numpy().reshape(-1)
for h in (256, 1024, 1000, 264):
    with A.Demodulator(freqs=A.FSK2_FREQS, hop=h) as d:
        W = (x.size - n) // h + 1
        sym, mag = d.batch(x, n_windows=W, mags=True)
    ref_sym, ref_P = O.goertzel(x, A.FSK2_FREQS, n, h)
    denom = np.maximum(ref_P.max(axis=1), 1e-30)
    e = np.abs(mag.astype(np.float64) - ref_P).max(axis=1) / denom
    i = int(e.argmax())
    print(h, W, "max err", e.max(), "at", i, "P", ref_P[i], mag[i], "p99.9", np.quantile(e, 0.999), flush=True)
    # the worst window directly in numpy fp32 emulation of one 1024 chain? print its energy
    xe = x[i * h:i * h + n].astype(np.float64)
    print("   window energy N*sum x^2/2 =", n * (xe * xe).sum() / 2, flush=True)
