#!/usr/bin/env python3
"""Summarise the bench.py lines of a gpu_run.sh directory (ab / bench steps):
    python3 scripts/ab_summary.py gpurun_out/<dir>"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    lines = [ln for ln in open(f, errors="replace") if ln.startswith("{")]
    if not lines:
        continue
    try:
        j = json.loads(lines[-1])
    except ValueError:
        continue
    if "ms_per_step" not in j:
        continue
    rf = j.get("roofline", {})
    rv = j.get("roofline_valu", {})
    print(f"{os.path.basename(f):24s} {j['config']['workload'][:38]:38s} ms/step {j['ms_per_step']:.4f} "
          f"kernel {j.get('kernel_ms', 0):.4f} p50 {j.get('kernel_ms_p10_p50_p90', [0, 0, 0])[1]:.4f} "
          f"frac {rf.get('frac', 0):.4f}{(' valu %.4f' % rv['frac']) if rv else ''} "
          f"launches {rf.get('launches_per_step')} err {j.get('symbol_errors')}")
