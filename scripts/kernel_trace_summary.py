#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace.

The --stats table averages every dispatch of a kernel, so one kernel launched
with several workloads in one bench.py run (the headline batch, the configs[4]
streams batch, host-path chunks) reads as one mixed mean. This splits the
trace by kernel name and grid size, so the headline dispatches can be
compared with the bench line's kernel_ms.

    python scripts/kernel_trace_summary.py gpurun_out/<dir>/kt/run_kernel_trace.csv [out.csv]
"""
import csv
import sys
from collections import defaultdict

import numpy as np


def main(path, out=None):
    groups = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if not r["Kernel_Name"].startswith(("void fskd::", "fskd::")):
                continue
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
            groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        d = np.array(d)
        rows.append({"kernel": name, "grid_x": grid, "workgroup_x": wg, "calls": d.size,
                     "mean_us": round(float(d.mean()), 2), "median_us": round(float(np.median(d)), 2),
                     "min_us": round(float(d.min()), 2), "max_us": round(float(d.max()), 2)})
    for r in rows:
        print(f'{r["calls"]:6d} {r["mean_us"]:10.2f} {r["median_us"]:10.2f} {r["min_us"]:10.2f} '
              f'grid {r["grid_x"]:>9d} x {r["workgroup_x"]:<4d} {r["kernel"][:110]}')
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main(*sys.argv[1:])
