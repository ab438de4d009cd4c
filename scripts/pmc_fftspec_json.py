#!/usr/bin/env python3
"""profiles/pmc_fftspec.json (bench.py's roofline.traffic of the
fft_hop256_spectrum extra) from the FETCH_SIZE / WRITE_SIZE passes of
scripts/gpu_prof_slide_spec.sh (gpurun_out/<dir>/pmc_{FETCH,WRITE}_SIZE),
averaged over the spectrum kernel's launches; copies the CSVs to
profiles/round2/<dir>/.

    python scripts/pmc_fftspec_json.py prof_ss2

bytes = KB * 1024; FETCH_SIZE doubled (gfx950 counts half of 16 B/lane
streaming reads, MI355X_MICROARCH.md §HBM).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "fft1024_quad_kernel<4, 4, 0, true"


def per_launch(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if KERNEL in r["Kernel_Name"]]
    vals = {}
    for r in rows:
        vals.setdefault(r["Dispatch_Id"], 0.0)
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return rows[0]["Kernel_Name"], sorted(vals.values()), rows


def main(tag):
    d = os.path.join(ROOT, "gpurun_out", tag)
    name, fetch, rows = per_launch(d, "FETCH_SIZE")
    _, write, wrows = per_launch(d, "WRITE_SIZE")
    W, hop, n = 1 << 20, 256, 1024
    Wev = (W * n - n) // hop + 1
    fkb, wkb = sum(fetch) / len(fetch), sum(write) / len(write)
    rd, wr = 2 * fkb * 1024, wkb * 1024
    alg = W * n * 2 + Wev * (1 + 2 * 4 + 513 * 4)  # input once + symbols + 2 tone powers + spectrum
    out = {"config": "fftspec", "windows": W, "hop": hop, "windows_evaluated": Wev,
           "kernel": name, "launches_sampled": len(fetch),
           "FETCH_SIZE_kb_per_launch": fkb, "WRITE_SIZE_kb_per_launch": wkb,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg,
           "traffic_over_alg": (rd + wr) / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                     "scripts/slide_spec_runs.py (scripts/gpu_prof_slide_spec.sh): FFT detector, hop "
                     "256, full spectrum stored through the linear slab; bytes = KB*1024, FETCH "
                     "doubled per MI355X_MICROARCH.md §HBM",
           "source": f"profiles/round2/{tag}/pmc_FETCH_SIZE.csv, pmc_WRITE_SIZE.csv"}
    dst = os.path.join(ROOT, "profiles", "round2", tag)
    os.makedirs(dst, exist_ok=True)
    for c, rs in (("FETCH_SIZE", rows), ("WRITE_SIZE", wrows)):
        with open(os.path.join(dst, f"pmc_{c}.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rs[0].keys()))
            w.writeheader()
            w.writerows(rs)
    with open(os.path.join(ROOT, "profiles", "pmc_fftspec.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "prof_ss2")
