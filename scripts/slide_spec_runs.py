#!/usr/bin/env python3
"""Short fixed workloads for rocprofv3 passes over the round-2 additions:
8-FSK (survey plan) at hop 256 through the fold detector's segment-shared
form (fold_slide_kernel) and the FFT detector at hop 256 with the full
spectrum stored (linear slab). One 2^30-sample stream, 3 warmup + 5 launches
each; prints the HIP-event median per workload.

    rocprofv3 --kernel-trace --stats -- python3 scripts/slide_spec_runs.py
    rocprofv3 --pmc FETCH_SIZE -- python3 scripts/slide_spec_runs.py
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
    n, src, hop = 1024, 1 << 20, 256
    d_pcm = torch.empty((src, n), dtype=torch.int16, device="cuda")
    A.synth_fsk(A.make_cfg(freqs=A.FSK8_FREQS), 7, src, 8000, 400, d_pcm)
    W = (src * n - n) // hop + 1
    s = torch.cuda.current_stream()
    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
    for name, freqs, method, spec in (("fsk8_fold_slide_hop256", A.FSK8_FREQS, A.METHOD_AUTO, False),
                                      ("fft_spectrum_hop256", A.FSK2_FREQS, A.METHOD_FFT, True)):
        K = len(freqs)
        mag = torch.empty((W, K), dtype=torch.float32, device="cuda")
        d_spec = torch.empty((W, 513), dtype=torch.float32, device="cuda") if spec else None
        with A.Demodulator(freqs=freqs, hop=hop, method=method) as d:
            def run():
                if spec:
                    d.batch_spectrum_async(d_pcm, W, sym, mag, d_spec, stream=s.cuda_stream)
                else:
                    d.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream)
            for _ in range(3):
                run()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(5)]
            for a, b in ev:
                a.record(s)
                run()
                b.record(s)
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            out = W * (1 + 4 * K + (2052 if spec else 0))
            print(json.dumps({"workload": name, "method": d.method, "windows": W, "kernel_ms": round(ms, 4),
                              "alg_bytes": src * n * 2 + out,
                              "alg_GBps": round((src * n * 2 + out) / (ms / 1e3) / 1e9, 1)}), flush=True)
        del mag, d_spec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
