#!/usr/bin/env python3
"""8-FSK (fold F16, configs[2]) magnitude write cost vs launch size: the same
2^20 windows demodulated as 1, 2, 4 or 8 back-to-back launches over
contiguous slices (outputs to the same buffers), time from HIP events
around the whole group; 80 warmup batches, then the variants round-robin
(6 rounds x 8), median.

    python scripts/split_launch_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    A, _ = bench.load_pkg()
    W, n = 1 << 20, 1024
    for name, freqs in (("fsk8", A.FSK8_FREQS), ("fsk2", A.FSK2_FREQS)):
        K = len(freqs)
        d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
        A.synth_fsk(A.make_cfg(freqs=freqs), 7, W, 8000, 400, d_pcm)
        sym = torch.empty(W, dtype=torch.uint8, device="cuda")
        mag = torch.empty((W, K), dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream()
        res = {}
        with A.Demodulator(freqs=freqs) as d:
            def group(parts, mags, ev=None):
                per = W // parts
                if ev:
                    ev[0].record(s)
                for i in range(parts):
                    d.batch_async(d_pcm[i * per:(i + 1) * per], per, sym[i * per:(i + 1) * per],
                                  mag[i * per:(i + 1) * per] if mags else None,
                                  stream=s.cuda_stream)
                if ev:
                    ev[1].record(s)
            for _ in range(80):                  # past the power-management transient
                group(1, True)
            for rnd in range(6):                 # round-robin over the variants
                for parts in (1, 2, 4, 8, 16):
                    for mags in (True, False):
                        ev = [(torch.cuda.Event(enable_timing=True),
                               torch.cuda.Event(enable_timing=True)) for _ in range(8)]
                        for e in ev:
                            group(parts, mags, e)
                        torch.cuda.synchronize()
                        res.setdefault((parts, mags), []).extend(a.elapsed_time(b) * 1e3 for a, b in ev)
        for (parts, mags), t in sorted(res.items()):
            print(f"{name} {parts:2d} launch(es) {'mags' if mags else 'no mags':8s} "
                  f"median {np.median(t):6.1f} us  (each launch may slice further: "
                  f"demod_batch_launches)", flush=True)
        del d_pcm


if __name__ == "__main__":
    main()
