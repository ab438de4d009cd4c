#!/usr/bin/env python3
"""Many live streams through demod_streams_push (one batch per push) against
one demodulate() call per stream: S streams, each pushed one 60 ms packet
(2880 frames at 48 kHz, the playback.cpp:10 packet) per round; wall time per
round (median of the timed rounds) and the real-time factor
S x 60 ms / round time. Mono and interleaved stereo (left channel), hop = n
and hop 256.

    python scripts/streams_push_bench.py [--streams 1024] [--rounds 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--lib", default=None, help="load this build of libfskdemod.so instead (A/B)")
    args = ap.parse_args()
    import bench
    A, _ = bench.load_pkg()
    if args.lib:
        A.load_library(args.lib)
    S, R, F = args.streams, args.rounds, 2880
    rng = np.random.default_rng(1)
    for channels, hop in ((1, 1024), (2, 1024), (1, 256)):
        pk = rng.integers(-8000, 8000, size=(S, (R + 3) * F * channels)).astype(np.int16)
        kw = dict(freqs=A.FSK2_FREQS, hop=hop, channels=channels)
        with A.Streams(S, **kw) as ms:
            times, syms = [], 0
            for r in range(R + 3):
                pkts = [pk[s, r * F * channels:(r + 1) * F * channels] for s in range(S)]
                t0 = time.perf_counter()
                out = ms.push(pkts)
                dt = time.perf_counter() - t0
                if r >= 3:
                    times.append(dt)
                    syms += sum(o.size for o in out)
        t_push = float(np.median(times))
        # the same packets as one 2-D array (rows = streams, a column slice)
        with A.Streams(S, **kw) as ms:
            times2 = []
            for r in range(R + 3):
                t0 = time.perf_counter()
                ms.push(pk[:, r * F * channels:(r + 1) * F * channels])
                dt = time.perf_counter() - t0
                if r >= 3:
                    times2.append(dt)
        t_rows = float(np.median(times2))
        # the same pushes through the C ABI alone: pointer arrays and output
        # buffers built outside the timer (what a C caller pays)
        import ctypes
        lib = A.load_library()
        with A.Streams(S, **kw) as ms:
            times_abi = []
            frames = np.full(S, F, dtype=np.uintp)
            cap = S * (F // hop + 2)
            sym = np.empty(cap, dtype=np.uint8)
            counts = np.zeros(S, dtype=np.uint32)
            for r in range(R + 3):
                base = pk[:, r * F * channels:(r + 1) * F * channels]
                ptrs = (ctypes.c_void_p * S)(*[base[s].ctypes.data for s in range(S)])
                t0 = time.perf_counter()
                rc = lib.demod_streams_push(ms._h, ctypes.cast(ptrs, ctypes.c_void_p), frames.ctypes.data,
                                            sym.ctypes.data, None, cap, counts.ctypes.data)
                dt = time.perf_counter() - t0
                assert rc >= 0, rc
                if r >= 3:
                    times_abi.append(dt)
        t_abi = float(np.median(times_abi))
        singles = [A.Demodulator(**kw) for _ in range(S)]
        times1 = []
        for r in range(min(R, 5) + 2):
            t0 = time.perf_counter()
            for s in range(S):
                singles[s].demodulate(pk[s, r * F * channels:(r + 1) * F * channels])
            if r >= 2:
                times1.append(time.perf_counter() - t0)
        for d in singles:
            d.close()
        t_one = float(np.median(times1))
        print(json.dumps({"lib": args.lib or "in-tree", "streams": S, "channels": channels, "hop": hop, "packet_frames": F,
                          "push_ms": round(t_push * 1e3, 3),
                          "push_abi_ms": round(t_abi * 1e3, 3),
                          "push_rows_ms": round(t_rows * 1e3, 3),
                          "per_stream_calls_ms": round(t_one * 1e3, 3),
                          "speedup": round(t_one / t_push, 1),
                          "realtime_factor_push": round(S * 0.06 / t_push, 1),
                          "symbols_per_push": syms // R}), flush=True)


if __name__ == "__main__":
    main()
