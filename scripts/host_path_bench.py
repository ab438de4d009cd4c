#!/usr/bin/env python3
"""Host-buffer boundary throughput (the PCIe-inclusive path; never bench.py's
`value`): demod_batch on host numpy windows and streaming demodulate() with
60 ms stereo packets as the reference's playback task would deliver them
(playback.cpp:115-131: 2880 frames per opus_decode call).

    python scripts/host_path_bench.py [--windows 1048576]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--packets", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import bench
    A, _ = bench.load_pkg()
    W, n = args.windows, 1024
    cfg = A.make_cfg(freqs=A.FSK2_FREQS, n=n, hop=n)
    d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
    d_true = torch.empty(W, dtype=torch.uint8, device="cuda")
    A.synth_fsk(cfg, A.BENCH_SEED, W, 8000, 400, d_pcm, d_true)
    torch.cuda.synchronize()
    pcm = d_pcm.cpu().numpy()
    true = d_true.cpu().numpy()
    out = {"windows": W, "bytes": W * n * 2}

    # raw PCIe reference: pinned and pageable H2D of the same bytes
    h_pin = torch.from_numpy(pcm).pin_memory()
    h_page = torch.from_numpy(pcm)
    for name, h in (("h2d_pinned_GBps", h_pin), ("h2d_pageable_GBps", h_page)):
        d_pcm.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            d_pcm.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        out[name] = round(W * n * 2 * args.reps / (time.perf_counter() - t0) / 1e9, 2)

    with A.Demodulator(cfg) as dm:
        sym, mag = dm.batch(pcm, mags=True)  # warm (allocates staging)
        out["batch_symbol_errors"] = int((sym != true).sum())
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            sym, mag = dm.batch(pcm, mags=True)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        out["batch_host_ms"] = round(t * 1e3, 2)
        out["batch_host_Msamples_per_s"] = round(W * n / t / 1e6, 1)
        out["batch_host_GBps"] = round(W * n * 2 / t / 1e9, 2)

    # streaming: 60 ms stereo packets (2880 frames, L = the FSK signal)
    scfg = A.make_cfg(freqs=A.FSK2_FREQS, n=n, hop=n, channels=2)
    P = args.packets
    mono = pcm.reshape(-1)[:P * 2880]
    st = np.empty(2 * mono.size, dtype=np.int16)
    st[0::2] = mono
    st[1::2] = 0
    with A.Demodulator(scfg) as dm:
        dm.demodulate(st[:2 * 2880])
        dm.reset()
        got = []
        t0 = time.perf_counter()
        for p in range(P):
            got.append(dm.demodulate(st[2 * 2880 * p:2 * 2880 * (p + 1)]))
        el = time.perf_counter() - t0
        got = np.concatenate(got)
        out["stream_packets"] = P
        out["stream_us_per_packet"] = round(el / P * 1e6, 1)
        out["stream_realtime_factor"] = round(0.060 * P / el, 1)
        out["stream_symbol_errors"] = int((got != true[:got.size]).sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
