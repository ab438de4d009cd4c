#!/usr/bin/env python3
"""profiles/pmc_fft.json and profiles/pmc_fftspec.json (bench.py's
roofline.traffic of the fft_hop256 and fft_hop256_spectrum entries) from the
FETCH_SIZE / WRITE_SIZE passes of `scripts/gpu_run.sh <dir> pmc`
(gpurun_out/<dir>/pmc_{fft,fftspec}_{FETCH,WRITE}_SIZE): the FFT detector
with the decision rescue inside the kernel. Averaged over every
launch of the detector kernel in `bench.py --config fft [--spectrum]
--no-rescue-ab`; the counter CSVs are copied to profiles/<round>/<dir>/.

    python scripts/pmc_fft_r3_json.py r4z [round4]

bytes = KB * 1024; FETCH_SIZE doubled (gfx950 counts half of streaming
reads, MI355X_MICROARCH.md §HBM; the hop-1024 run of round 2 confirmed the
rule for these 4 B/lane loads at 1.0009x the stream).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, spec):
    key = "fft1024_quad_kernel<4, 4, 0, true" if spec else "fft1024_quad_kernel<4, 4, 0, false"
    vals, name = {}, None
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if key in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    v = list(vals.values())
    return name, sum(v) / len(v), len(v)


def main(tag="r4z", rnd="round4"):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", rnd, tag)
    os.makedirs(dst, exist_ok=True)
    W, hop, n = 1 << 20, 256, 1024
    Wev = (W * n - n) // hop + 1
    for cfg, spec in (("fft", False), ("fftspec", True)):
        if not os.path.exists(os.path.join(src, f"pmc_{cfg}_FETCH_SIZE")):
            continue
        got = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            path = os.path.join(src, f"pmc_{cfg}_{c}", "run_counter_collection.csv")
            got[c] = per_launch(path, spec)
            shutil.copy(path, os.path.join(dst, f"pmc_{cfg}_{c}.csv"))
        name, fkb, launches = got["FETCH_SIZE"]
        wkb = got["WRITE_SIZE"][1]
        rd, wr = 2 * fkb * 1024, wkb * 1024
        # input once + symbols + 2 tone powers (+ the 513-float spectrum)
        alg = W * n * 2 + Wev * (1 + 2 * 4 + (513 * 4 if spec else 0))
        out = {"config": cfg, "windows": W, "hop": hop, "windows_evaluated": Wev, "kernel": name,
               "launches_sampled": launches, "FETCH_SIZE_kb_per_launch": fkb,
               "WRITE_SIZE_kb_per_launch": wkb, "read_bytes_per_launch": rd,
               "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
               "alg_bytes_per_launch": alg, "traffic_over_alg": (rd + wr) / alg,
               "method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                          "bench.py --config fft" + (" --spectrum" if spec else "") +
                          " --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5 "
                          f"(scripts/gpu_run.sh {tag} pmc); bytes = KB*1024, FETCH doubled per "
                          "MI355X_MICROARCH.md §HBM; the decision rescue inside the kernel"),
               "source": f"profiles/{rnd}/{tag}/pmc_{cfg}_FETCH_SIZE.csv, pmc_{cfg}_WRITE_SIZE.csv"}
        with open(os.path.join(ROOT, "profiles", f"pmc_{cfg}.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        print(cfg, launches, round(out["traffic_over_alg"], 5), round(rd / 1e9, 4), round(wr / 1e9, 4))


if __name__ == "__main__":
    main(*sys.argv[1:])
