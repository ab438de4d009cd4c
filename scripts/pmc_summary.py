#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc passes for one kernel.

    python scripts/pmc_summary.py <kernel-substring> <pass-dir>... [--groups G] [--out json]

Each <pass-dir> holds run_counter_collection.csv. Prints the counters (mean
over that kernel's dispatches), per-group values (/ G when given) and the
derived ratios: the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall) and the
SQ issue shares (MI355X_MICROARCH.md §rocprofv3 PMC slots; SQ_* cycle
counters are quad-cycles).
"""
import argparse
import collections
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--groups", type=float, default=0.0)
    ap.add_argument("--out")
    ap.add_argument("--what", default="")
    a = ap.parse_args()
    sums, cnt, wall = collections.defaultdict(float), collections.Counter(), {}
    name = None
    for d in a.dirs:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            key = (d, r["Dispatch_Id"])
            sums[(d, r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(d, r["Counter_Name"])] += 1
            if "End_Timestamp" in r:
                wall[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    c = {}
    for (d, k), v in sums.items():
        # a counter's value per dispatch is the sum over its dimension rows;
        # rows per dispatch = rows / dispatches of that pass
        disp = len({kk for kk in wall if kk[0] == d}) or 1
        c.setdefault(k, v / disp)
    mean_wall = sum(wall.values()) / max(len(wall), 1)
    out = {"what": a.what, "kernel": name, "dispatches_per_pass": len(wall) // max(len(a.dirs), 1),
           "mean_dispatch_us": mean_wall * 1e6, "counters": c}
    if a.groups:
        out["per_group"] = {k: v / a.groups for k, v in c.items()
                            if k.startswith("SQ_INSTS") or k in ("SQ_WAVES",)}
    if c.get("SQ_ACTIVE_INST_ANY"):
        for k in ("VALU", "LDS", "MISC", "VMEM", "SCA"):
            if f"SQ_ACTIVE_INST_{k}" in c:
                out[f"{k.lower()}_share_of_issue"] = c[f"SQ_ACTIVE_INST_{k}"] / c["SQ_ACTIVE_INST_ANY"]
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                out[k.lower() + "_share_of_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
    if c.get("GRBM_GUI_ACTIVE") and mean_wall:
        out["effective_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / mean_wall / 1e9
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
    js = json.dumps(out, indent=1)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
