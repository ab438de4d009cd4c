#!/usr/bin/env python3
"""Where bench.py's ms_per_step exceeds kernel_ms (2-FSK configs[1]): 100
back-to-back demod_batch_async steps timed as a whole, with and without the
per-step HIP event pairs bench.py records for kernel_ms. 80 warmups,
round-robin x 6, median of the per-step time.

    python scripts/step_gap_probe.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    A, _ = bench.load_pkg()
    W, n, steps = 1 << 20, 1024, 100
    d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(), 7, W, 8000, 400, d_pcm)
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    mag = torch.empty((W, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    with A.Demodulator() as d:
        for _ in range(80):
            d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
        for rnd in range(6):
            for mode in ("events per step", "no events"):
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(steps)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    if mode == "events per step":
                        evs[i][0].record(s)
                    d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
                    if mode == "events per step":
                        evs[i][1].record(s)
                torch.cuda.synchronize()
                el = (time.perf_counter() - t0) / steps * 1e3
                res.setdefault(mode, []).append(el)
                if mode == "events per step":
                    res.setdefault("kernel (events)", []).append(
                        float(np.mean([a.elapsed_time(b) for a, b in evs])))
    for k, v in res.items():
        print(f"{k:18s} median {np.median(v) * 1e3:6.1f} us per step", flush=True)


if __name__ == "__main__":
    main()
