#!/usr/bin/env python3
"""FFT detector (configs[3], hop 256) as 1/2/4/8 back-to-back launches over
window slices of one 2^30-sample stream, with and without tone powers:
does the output write-back cost that slicing removes for 8-FSK
(scripts/split_launch_probe.py) show here too? 80 warmup batches, then the
variants round-robin (6 rounds x 5), median.

    python scripts/split_launch_fft.py
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
    n, hop, src = 1024, 256, 1 << 20
    W = (src * n - n) // hop + 1
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(freqs=A.FSK2_FREQS), 7, src, 8000, 400, d_pcm)
    flat = d_pcm.view(-1)
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    mag = torch.empty((W, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    with A.Demodulator(freqs=A.FSK2_FREQS, hop=hop, method=A.METHOD_FFT) as d:
        def group(parts, mags, ev=None):
            per = (W + parts - 1) // parts
            if ev:
                ev[0].record(s)
            for w0 in range(0, W, per):
                c = min(per, W - w0)
                d.batch_async(flat[w0 * hop:w0 * hop + (c - 1) * hop + n], c, sym[w0:w0 + c],
                              mag[w0:w0 + c] if mags else None, stream=s.cuda_stream)
            if ev:
                ev[1].record(s)
        for _ in range(80):                      # past the power-management transient
            group(1, True)
        # round-robin, so every variant sees the same clock history
        for rnd in range(6):
            for parts in (1, 2, 4, 8):
                for mags in (True, False):
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(5)]
                    for e in ev:
                        group(parts, mags, e)
                    torch.cuda.synchronize()
                    res.setdefault((parts, mags), []).extend(a.elapsed_time(b) * 1e3 for a, b in ev)
        for (parts, mags), t in sorted(res.items()):
            print(f"fft hop {hop} {parts} launch(es) {'mags' if mags else 'no mags':8s} "
                  f"median {np.median(t):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
