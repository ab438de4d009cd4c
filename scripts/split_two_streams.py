#!/usr/bin/env python3
"""8-FSK (configs[2]) as 4 output slices of 2^18 windows (each one launch,
below the library's slicing threshold): on one stream (what
demod_batch_async does) vs alternating over two streams forked from and
joined to the timing stream, so one slice's drain overlaps the next one's
fill. 80 warmups, round-robin, median.

    python scripts/split_two_streams.py
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
    W, n, parts = 1 << 20, 1024, 4
    freqs = A.FSK8_FREQS
    d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(freqs=freqs), 7, W, 8000, 400, d_pcm)
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    mag = torch.empty((W, 8), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    per = W // parts
    res = {}
    with A.Demodulator(freqs=freqs) as d:
        assert d.batch_launches(per) == 1

        def run(mode, ev=None):
            if ev:
                ev[0].record(s)
            if mode == "one stream":
                for i in range(parts):
                    d.batch_async(d_pcm[i * per:(i + 1) * per], per, sym[i * per:(i + 1) * per],
                                  mag[i * per:(i + 1) * per], stream=s.cuda_stream)
            else:
                for st in side:
                    st.wait_stream(s)
                for i in range(parts):
                    st = side[i % 2]
                    d.batch_async(d_pcm[i * per:(i + 1) * per], per, sym[i * per:(i + 1) * per],
                                  mag[i * per:(i + 1) * per], stream=st.cuda_stream)
                for st in side:
                    s.wait_stream(st)
            if ev:
                ev[1].record(s)

        for _ in range(80):
            run("one stream")
        for rnd in range(8):
            for mode in ("one stream", "two streams"):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(8)]
                for e in ev:
                    run(mode, e)
                torch.cuda.synchronize()
                res.setdefault(mode, []).extend(a.elapsed_time(b) * 1e3 for a, b in ev)
    for mode, t in res.items():
        print(f"fsk8 {parts} slices, {mode:12s} median {np.median(t):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
