#!/usr/bin/env python3
"""The rescue worst case of one detector alone (for rocprofv3 PMC passes and
kernel traces): bench.rescue_worst's two-tone stream, every window flagged.
    python3 scripts/rescue_probe.py fsk2_slide_hop256 [steps]
Cases: fsk2, fsk8, fft_hop256, fsk2_slide_hop256, fsk8_slide_hop256, fsk8odd
(residue detector). FSKD_NO_RESCUE=1 in the environment: the step without
the rescue (for the slowdown). Prints
the step time (HIP events over the timed steps) and the flagged fraction."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "fsk2_slide_hop256"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import torch
    A, _ = bench.load_pkg()
    cases = {"fsk2": (A.FSK2_FREQS, 0, 1, A.METHOD_AUTO, 1024),
             "fsk8": (A.FSK8_FREQS, 2, 5, A.METHOD_AUTO, 1024),
             "fft_hop256": (A.FSK8_FREQS, 2, 5, A.METHOD_FFT, 256),
             "fsk2_slide_hop256": (A.FSK2_FREQS, 0, 1, A.METHOD_AUTO, 256),
             "fsk8_slide_hop256": (A.FSK8_FREQS, 2, 5, A.METHOD_AUTO, 256),
             # 8 tones on integer bins 32 + 9 i (not multiples of 8): the residue detector
             "fsk8odd": (tuple(46.875 * (32 + 9 * i) for i in range(8)), 2, 5, A.METHOD_AUTO, 1024)}
    freqs, a, b, method, hop = cases[case]
    W, n = 1 << 20, 1024
    dev = torch.device("cuda", 0)
    d_pcm = torch.empty((W, n), dtype=torch.int16, device=dev)
    bench.two_tone_stream(torch, d_pcm, freqs, a, b)
    n_eval = (W * n - n) // hop + 1
    sym = torch.empty(n_eval, dtype=torch.uint8, device=dev)
    mag = torch.empty((n_eval, len(freqs)), dtype=torch.float32, device=dev)
    d = A.Demodulator(A.make_cfg(freqs=freqs, n=n, hop=hop, method=method))
    with d:
        fn = lambda: d.batch_async(d_pcm, n_eval, sym, mag)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
    print(f"{case}: {ms:.4f} ms/step, detector {d.method}, "
          f"flagged {float((sym >= 128).sum().item()) / n_eval:.4f} (after rescue: should be 0)")


if __name__ == "__main__":
    main()
