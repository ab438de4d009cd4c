#!/usr/bin/env python3
"""Per-grid summary of a rocprofv3 --kernel-trace CSV: the bench command's
detector kernels run at several sizes (the timed batch, the extras, the
rescue worst case), so rocprof's per-name average mixes them. Groups by
(kernel, grid size) and prints count, mean and median duration (us).

    python scripts/kt_by_grid.py gpurun_out/r4z/kt/run_kernel_trace.csv > profiles/round4/r4z/kernel_trace_by_grid.csv
"""
import csv
import statistics
import sys
from collections import defaultdict

groups = defaultdict(list)
with open(sys.argv[1]) as fh:
    for r in csv.DictReader(fh):
        if "fskd::" not in r["Kernel_Name"]:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        groups[(r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]))].append(d)
w = csv.writer(sys.stdout)
w.writerow(["kernel", "grid_size_x", "dispatches", "mean_us", "median_us", "min_us"])
for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, grid, len(v), round(statistics.mean(v), 2), round(statistics.median(v), 2),
                round(min(v), 2)])
