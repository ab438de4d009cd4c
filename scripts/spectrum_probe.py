#!/usr/bin/env python3
"""Full-spectrum output of the FFT detector (demod_batch_spectrum_async,
SURVEY §8 f3): kernel time per launch with |X[b]|^2 for all 513 bins stored
(2052 B per window) against symbols + tone powers only, over one 2^30-sample
stream at hop 1024 and 256. Median of 20 after 30 warmups; the written
spectrum rate is n_windows x 2052 B / t. "spectrum" is a 16-byte-aligned
output (linear power slab, 16-byte stores of each group's contiguous run),
"spectrum_unaligned" the same output 4 bytes further (quad_slot slab, dword
stores).

    python scripts/spectrum_probe.py
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
    n, src = 1024, 1 << 20
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(), 7, src, 8000, 400, d_pcm)
    s = torch.cuda.current_stream()
    for hop in (1024, 256):
        W = (src * n - n) // hop + 1
        sym = torch.empty(W, dtype=torch.uint8, device="cuda")
        mag = torch.empty((W, 2), dtype=torch.float32, device="cuda")
        spec_buf = torch.empty(W * 513 + 4, dtype=torch.float32, device="cuda")
        spec = spec_buf[:W * 513]
        spec_un = spec_buf[1:1 + W * 513]
        with A.Demodulator(freqs=A.FSK2_FREQS, hop=hop, method=A.METHOD_FFT) as d:
            for label, run in (("tones", lambda: d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)),
                               ("spectrum", lambda: d.batch_spectrum_async(d_pcm, W, sym, mag, spec,
                                                                           stream=s.cuda_stream)),
                               ("spectrum_unaligned", lambda: d.batch_spectrum_async(
                                   d_pcm, W, sym, mag, spec_un, stream=s.cuda_stream))):
                for _ in range(30):
                    run()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(20)]
                for a, b in ev:
                    a.record(s)
                    run()
                    b.record(s)
                torch.cuda.synchronize()
                ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
                out = W * (513 * 4 if label.startswith("spectrum") else 9)
                print(json.dumps({"hop": hop, "windows": W, "output": label, "kernel_ms": round(ms, 4),
                                  "write_GBps": round(out / (ms / 1e3) / 1e9, 1),
                                  "read_GBps": round(src * n * 2 / (ms / 1e3) / 1e9, 1)}), flush=True)
        # write-only reference: torch's fill of the same 2052 B x W buffer
        for _ in range(5):
            spec_buf.fill_(1.0)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(10)]
        for a, b in ev:
            a.record(s)
            spec_buf.fill_(1.0)
            b.record(s)
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        print(json.dumps({"hop": hop, "output": "write_only_fill", "bytes": spec_buf.numel() * 4,
                          "kernel_ms": round(ms, 4),
                          "write_GBps": round(spec_buf.numel() * 4 / (ms / 1e3) / 1e9, 1)}), flush=True)
        del spec, spec_un, spec_buf, mag, sym
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
