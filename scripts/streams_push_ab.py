#!/usr/bin/env python3
"""A/B of the demod_streams_push staging variants.

copy   — the push stages every stream's run into pinned memory (persistent
         staging threads for large pushes), one H2D copy, the detector (+ the
         rescue), one D2H copy of the results;
mapped — FSKD_STREAMS_MAPPED=1: the same staging into mapped pinned memory
         that the detector reads in place over PCIe and writes its results
         back to (no copies; one launch and one synchronize).

S streams, one 60 ms packet (2880 frames) per stream per push, timed through
the C ABI alone (pointer arrays built outside the timer, as a C caller has
them), the variants interleaved round by round; the symbols of both must be
identical. Mono and stereo at hop = n, mono at hop 256.

    python scripts/streams_push_ab.py [--streams 1024] [--rounds 30]
"""
import argparse
import ctypes
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
    ap.add_argument("--rounds", type=int, default=30)
    args = ap.parse_args()
    import bench
    A, _ = bench.load_pkg()
    lib = A.load_library()
    S, R, F = args.streams, args.rounds, 2880
    rng = np.random.default_rng(1)
    for channels, hop in ((1, 1024), (2, 1024), (1, 256)):
        pk = rng.integers(-8000, 8000, size=(S, (R + 3) * F * channels)).astype(np.int16)
        kw = dict(freqs=A.FSK2_FREQS, hop=hop, channels=channels)
        handles = {}
        for name in ("copy", "mapped"):
            if name == "mapped":
                os.environ["FSKD_STREAMS_MAPPED"] = "1"
            try:
                handles[name] = A.Streams(S, **kw)
            finally:
                os.environ.pop("FSKD_STREAMS_MAPPED", None)
        frames = np.full(S, F, dtype=np.uintp)
        cap = S * (F // hop + 2)
        outs = {k: np.empty(cap, dtype=np.uint8) for k in handles}
        counts = {k: np.zeros(S, dtype=np.uint32) for k in handles}
        times = {k: [] for k in handles}
        equal = True
        for r in range(R + 3):
            base = pk[:, r * F * channels:(r + 1) * F * channels]
            ptrs = (ctypes.c_void_p * S)(*[base[s].ctypes.data for s in range(S)])
            order = ("copy", "mapped") if r % 2 == 0 else ("mapped", "copy")
            got = {}
            for k in order:
                t0 = time.perf_counter()
                rc = lib.demod_streams_push(handles[k]._h, ctypes.cast(ptrs, ctypes.c_void_p),
                                            frames.ctypes.data, outs[k].ctypes.data, None, cap,
                                            counts[k].ctypes.data)
                dt = time.perf_counter() - t0
                assert rc >= 0, (k, rc)
                got[k] = outs[k][:rc].copy()
                if r >= 3:
                    times[k].append(dt)
            equal &= bool(np.array_equal(got["copy"], got["mapped"]))
        for h in handles.values():
            h.close()
        print(json.dumps({"streams": S, "channels": channels, "hop": hop, "packet_frames": F,
                          "rounds": R,
                          "copy_ms_p50": round(float(np.median(times["copy"])) * 1e3, 3),
                          "mapped_ms_p50": round(float(np.median(times["mapped"])) * 1e3, 3),
                          "copy_ms_p10_p90": [round(float(np.percentile(times["copy"], q)) * 1e3, 3)
                                              for q in (10, 90)],
                          "mapped_ms_p10_p90": [round(float(np.percentile(times["mapped"], q)) * 1e3, 3)
                                                for q in (10, 90)],
                          "symbols_identical": equal}), flush=True)


if __name__ == "__main__":
    main()
