#!/usr/bin/env python3
"""Sliding-window (hop < n) throughput of the Goertzel detectors
over one 2^30-sample int16 stream in HBM: kernel time per launch (HIP events,
median of 20 after 30 warmup launches), the unique-stream rate (2 GiB / t) and
the window-bytes rate (n_windows x 2 KiB / t). At hop = 64 H < n AUTO takes
the segment-shared plain bank (SLIDE) for 2-FSK and the fold detector's
segment-shared form for 8-FSK; the other of the two is timed beside each.
FSKD_NO_SLIDE=1 in the environment times the direct kernels instead.

    python scripts/sliding_probe.py [--samples-log2 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples-log2", type=int, default=30)
    ap.add_argument("--hops", default="1024,1000,512,256,200,128")
    ap.add_argument("--plans", default="fsk2,fsk8", help="comma list of fsk2, fsk8, fsk8odd")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    A, _ = bench.load_pkg()
    n = 1024
    S = 1 << args.samples_log2
    src = S // n
    cfg0 = A.make_cfg(freqs=A.FSK2_FREQS, n=n, hop=n)
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    d_true = torch.empty(src, dtype=torch.uint8, device="cuda")
    A.synth_fsk(cfg0, A.BENCH_SEED, src, 8000, 400, d_pcm, d_true)
    torch.cuda.synchronize()
    odd = tuple(46.875 * (32 + 9 * i) for i in range(8))   # integer bins, every residue class
    cases = {"fsk2": (("fsk2", A.FSK2_FREQS, 0), ("fsk2", A.FSK2_FREQS, A.METHOD_FOLDED)),
             "fsk8": (("fsk8", A.FSK8_FREQS, 0), ("fsk8", A.FSK8_FREQS, A.METHOD_GOERTZEL)),
             "fsk8odd": (("fsk8odd", odd, A.METHOD_GOERTZEL), ("fsk8odd", odd, A.METHOD_RESIDUE))}
    for name, freqs, method in [c for key in args.plans.split(",") for c in cases[key]]:
        for hop in [int(h) for h in args.hops.split(",")]:
            W = (S - n) // hop + 1
            K = len(freqs)
            with A.Demodulator(A.make_cfg(freqs=freqs, n=n, hop=hop, method=method)) as d:
                sym = torch.empty(W, dtype=torch.uint8, device="cuda")
                mag = torch.empty(W * K, dtype=torch.float32, device="cuda")
                s = torch.cuda.current_stream()
                for _ in range(30):
                    d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(20)]
                for a, b in ev:
                    a.record(s)
                    d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
                    b.record(s)
                torch.cuda.synchronize()
                ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
                print(json.dumps({"cfg": name, "hop": hop, "windows": W, "method": d.method,
                                  "kernel_ms": round(ms, 4),
                                  "stream_GBps": round(S * 2 / (ms / 1e3) / 1e9, 1),
                                  "window_bytes_GBps": round(W * 2 * n / (ms / 1e3) / 1e9, 1),
                                  "Mwindows_per_s": round(W / (ms / 1e3) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
