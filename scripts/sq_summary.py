#!/usr/bin/env python3
"""Summarise the SQ/GRBM passes of scripts/gpu_pmc_sq.sh (removed in round 6; git show 8b49018:scripts/gpu_pmc_sq.sh) (gpurun_out/sq_*/):
per-dispatch means of the kernel each pass profiled, and the derived issue
fractions, into profiles/round1/pmc_sq_kernels.json.

    python scripts/sq_summary.py

Derived (MI355X_MICROARCH.md §Counters): SQ_ACTIVE_INST_* and SQ_BUSY_CYCLES
count in quad-cycles summed over SIMDs/SEs as rocprofv3 reports them;
fractions here are ratios of counters of the same kind, and the effective
clock is GRBM_GUI_ACTIVE / 8 (XCDs) / the dispatch's wall time.
"""
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"residue": "residue_tile_kernel", "goertzel": "goertzel_tile_kernel",
        "fold": "fold_tile_kernel"}


def main():
    out = {}
    for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "sq_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        tag = os.path.basename(d)[3:].strip("_")
        key = next(v for k, v in KEYS.items() if tag.startswith(k))
        sums, cnt, wall = collections.defaultdict(float), collections.Counter(), {}
        for r in csv.DictReader(open(f)):
            if key not in r["Kernel_Name"]:
                continue
            sums[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
            wall[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
        c = {k: sums[k] / cnt[k] for k in sums}
        mean_wall = sum(wall.values()) / len(wall)
        d_out = {"kernel": key, "dispatches": len(wall), "mean_dispatch_us": mean_wall * 1e6,
                 "counters": c}
        if c.get("SQ_ACTIVE_INST_ANY"):
            d_out["valu_share_of_issue"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_ACTIVE_INST_ANY"]
            d_out["lds_share_of_issue"] = c["SQ_ACTIVE_INST_LDS"] / c["SQ_ACTIVE_INST_ANY"]
        if c.get("GRBM_GUI_ACTIVE"):
            d_out["effective_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / mean_wall / 1e9
        out[tag] = d_out
        print(tag, {k: round(v, 3) for k, v in d_out.items() if isinstance(v, float)})
    out["_source"] = ("rocprofv3 --pmc (9 counters, one pass per kernel) over scripts/bin/probe "
                      "1048576 1 3 with PROBE_FILTER per kernel (scripts/gpu_pmc_sq.sh)")
    json.dump(out, open(os.path.join(ROOT, "profiles", "round1", "pmc_sq_kernels.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
