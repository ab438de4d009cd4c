#!/usr/bin/env python3
"""Wait-state shares of one kernel from a rocprofv3 --pmc counter CSV
(scripts/gpu_run.sh sqw): SQ_WAIT_ANY (waves parked at s_waitcnt / barrier),
SQ_WAIT_INST_ANY (issue-stalled; SQ_WAIT_INST_LDS its LDS part) and
SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md
§rocprofv3 PMC), VALU busy = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8), mean over the kernel's dispatches.
    python3 scripts/sq_wait_summary.py <run_counter_collection.csv> [kernel-substring]"""
import csv
import json
import sys
from collections import defaultdict

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "fft1024_quad_kernel"
acc = defaultdict(lambda: defaultdict(float))
name = {}
for r in csv.DictReader(open(path)):
    if pat not in r["Kernel_Name"]:
        continue
    d = int(r["Dispatch_Id"])
    acc[d][r["Counter_Name"]] += float(r["Counter_Value"])
    name[d] = r["Kernel_Name"]
if not acc:
    sys.exit("no dispatch of " + pat)
keys = sorted({k for v in acc.values() for k in v})
mean = {k: sum(v.get(k, 0.0) for v in acc.values()) / len(acc) for k in keys}
wc = mean.get("SQ_WAVE_CYCLES", 0.0)
out = {"kernel": next(iter(name.values())), "dispatches": len(acc), "counters_mean": mean}
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
        if k in mean:
            out[k + "_frac_of_wave_cycles"] = round(mean[k] / wc, 4)
if "SQ_INSTS_VALU" in mean and "GRBM_GUI_ACTIVE" in mean:
    out["valu_busy_frac_4cyc"] = round(mean["SQ_INSTS_VALU"] * 4 / 1024 / (mean["GRBM_GUI_ACTIVE"] / 8), 4)
print(json.dumps(out, indent=1))
