#!/usr/bin/env python3
"""Copy the results of scripts/gpu_check.sh (merged into gpurun_out/) into
profiles/round1/: bench lines appended to bench_<cfg>.jsonl, the pytest and
smoke logs, the rocprofv3 kernel statistics, and per-dispatch kernel traces
with the mean of the 20 timed dispatches (kernel_trace_timed_*.json).

    python scripts/store_gpu_check.py
"""
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles", "round1")
BENCH = {"fsk2": "bench", "fsk8": "bench_fsk8", "fft": "bench_fft", "fft1024": "bench_fft1024",
         "streams": "bench_streams", "fsk8_odd": "bench_fsk8_odd",
         "fsk8_odd_plain": "bench_fsk8_odd_plain"}


def last_json_line(path):
    lines = [l for l in open(path) if l.startswith("{")]
    return lines[-1] if lines else None


def main():
    for cfg, log in BENCH.items():
        src = os.path.join(OUT, log + ".log")
        line = last_json_line(src) if os.path.exists(src) else None
        if line:
            with open(os.path.join(P, f"bench_{cfg}.jsonl"), "a") as f:
                f.write(line if line.endswith("\n") else line + "\n")
    for name in ("pytest_gpu.log", "smoke.log"):
        shutil.copy(os.path.join(OUT, name), os.path.join(P, name))
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"),
                os.path.join(P, "kernel_stats_bench_default.csv"))
    shutil.copy(os.path.join(OUT, "prof_fft", "run_kernel_stats.csv"),
                os.path.join(P, "kernel_stats_fft.csv"))
    for sub, tag, key in (("prof", "fsk2", "goertzel_tile_kernel"),
                          ("prof_fft", "fft", "fft1024_quad_kernel")):
        rows = sorted((r for r in csv.DictReader(open(os.path.join(OUT, sub, "run_kernel_trace.csv")))
                       if key in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        out = {"kernel": key,
               "source": "rocprofv3 --kernel-trace of bench.py --steps 20 (scripts/gpu_check.sh)",
               "dispatches": len(us), "mean_all_us": sum(us) / len(us),
               "mean_warmup_us": sum(us[:-20]) / len(us[:-20]),
               "mean_timed_last20_us": sum(us[-20:]) / 20, "series_us": [round(u, 1) for u in us]}
        json.dump(out, open(os.path.join(P, f"kernel_trace_timed_{tag}.json"), "w"), indent=1)
        print(key, "timed mean", round(out["mean_timed_last20_us"], 1), "us")


if __name__ == "__main__":
    main()
