#!/usr/bin/env python3
"""Kernel time of the plain tone bank with and without the Reinsch form
(goertzel.hip RS), 2^20 windows of 1024 samples, device-resident, symbols +
|X_k|^2; interleaved rounds, median of HIP-event times on the launch stream.
A plan switches to RS when a tone has |sin w| < 0.1 (demod_api.cpp), so the
pairs below differ by one tone moved from 1500 Hz to 375 Hz (|sin w| = 0.049).

    python scripts/reinsch_cost.py   (GPU)
"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "audio_network_amd", os.path.join(ROOT, "audio-network_amd", "__init__.py"),
    submodule_search_locations=[os.path.join(ROOT, "audio-network_amd")])
A = importlib.util.module_from_spec(spec)
sys.modules["audio_network_amd"] = A
spec.loader.exec_module(A)

W, n = 1 << 20, 1024
plans = {
    "K=2 2cos": (1500.0, 3000.0),
    "K=2 RS": (375.0, 3000.0),
    "K=8 2cos": tuple(1523.4 + 411.1 * i for i in range(8)),
    "K=8 RS": (375.0,) + tuple(1523.4 + 411.1 * i for i in range(1, 8)),
}
d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
cfg = A.make_cfg(freqs=plans["K=2 2cos"], n=n)
A.synth_fsk(cfg, 7, W, 8000, 400, d_pcm)
dems, outs = {}, {}
for name, f in plans.items():
    dems[name] = A.Demodulator(freqs=f, method=A.METHOD_GOERTZEL)
    outs[name] = (torch.empty(W, dtype=torch.uint8, device="cuda"),
                  torch.empty((W, len(f)), dtype=torch.float32, device="cuda"))
s = torch.cuda.current_stream()
times = {k: [] for k in plans}
for rnd in range(12):
    for name in plans:
        sym, mag = outs[name]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        dems[name].batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
        b.record(s)
        b.synchronize()
        if rnd >= 2:
            times[name].append(a.elapsed_time(b) * 1e3)
for name in plans:
    t = np.array(times[name])
    print(f"{name:10s} median {np.median(t):7.1f} us  min {t.min():7.1f} us")
