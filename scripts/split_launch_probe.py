#!/usr/bin/env python3
"""8-FSK (fold F16, configs[2]) magnitude write cost vs launch size: the same
2^20 windows demodulated as 1, 2, 4 or 8 back-to-back launches over
contiguous slices (outputs to the same buffers), kernel-to-kernel time from
HIP events around the whole group, median of 40 after 20 warmups.

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
        with A.Demodulator(freqs=freqs) as d:
            for parts in (1, 2, 4, 8, 16):
                for mags in (True, False):
                    per = W // parts
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(60)]
                    for a, b in ev:
                        a.record(s)
                        for i in range(parts):
                            d.batch_async(d_pcm[i * per:(i + 1) * per], per, sym[i * per:(i + 1) * per],
                                          mag[i * per:(i + 1) * per] if mags else None,
                                          stream=s.cuda_stream)
                        b.record(s)
                    torch.cuda.synchronize()
                    t = np.array([a.elapsed_time(b) for a, b in ev[20:]]) * 1e3
                    print(f"{name} {parts:2d} launch(es) {'mags' if mags else 'no mags':8s} "
                          f"median {np.median(t):6.1f} us", flush=True)
        del d_pcm


if __name__ == "__main__":
    main()
