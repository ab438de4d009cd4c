#!/usr/bin/env python3
"""8-tone plans on integer bins with different spacings at hop = n: the
detector AUTO picks and its kernel time against the plain bank (HIP events,
median of 20 after 30 warmups, 2^20 windows), plus the read-only ceiling of
the same buffer. Spacing 1 and odd spacings hit every residue class mod 8
evenly (the residue kernel's compile-time classes); even spacings leave
classes empty or uneven (its LDS class file); multiples of 8 fold.

    python scripts/plan_probe.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    A, _ = bench.load_pkg()
    n, W = 1024, 1 << 20
    d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(), 3, W, 8000, 400, d_pcm)
    s = torch.cuda.current_stream()
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    mag = torch.empty(W * 8, dtype=torch.float32, device="cuda")

    def timed(fn):
        for _ in range(30):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(20)]
        for a, b in ev:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    ceil = timed(lambda: A.read_ceiling_async(d_pcm, W * n * 2, stream=s.cuda_stream))
    print(json.dumps({"read_ceiling_ms": round(ceil, 4)}), flush=True)
    for spacing in (1, 2, 3, 4, 6, 8, 9, 12):
        freqs = tuple(46.875 * (32 + spacing * i) for i in range(8))
        for method in (A.METHOD_AUTO, A.METHOD_GOERTZEL):
            with A.Demodulator(freqs=freqs, method=method) as d:
                ms = timed(lambda: d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream))
                print(json.dumps({"spacing": spacing, "bins": [32 + spacing * i for i in range(8)],
                                  "requested": method, "method": d.method,
                                  "launches": d.batch_launches(W), "kernel_ms": round(ms, 4),
                                  "frac_8TBps": round(W * 2081 / (ms / 1e3) / 8e12, 3),
                                  "frac_ceiling": round(ceil / ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
