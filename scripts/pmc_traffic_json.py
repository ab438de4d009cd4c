#!/usr/bin/env python3
"""Per-launch HBM traffic of the detector kernels from the PMC passes of
`scripts/gpu_run.sh <dir> pmc` (merged into gpurun_out/<dir>/): writes
profiles/pmc_<cfg>.json (read by bench.py for roofline.traffic) and copies the
counter CSVs to profiles/<round>/.

    python scripts/pmc_traffic_json.py round4/r4z r4z   # a closing check:
        # passes under gpurun_out/r4z/, CSVs to profiles/round4/r4z/
        # (the FFT passes: scripts/pmc_fft_r3_json.py)

Round 2 (scripts/gpu_profile_r2.sh, scripts/gpu_r2_fft.sh) adds the FFT
detector at hop 256 (configs[3]) and hop 1024.

bytes = KB * 1024; FETCH_SIZE doubled (gfx950 counts half of 16 B/lane
streaming reads, MI355X_MICROARCH.md §HBM).
"""
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = 1 << 20
MAX_BATCHES = 69  # bench.py --warmup 2 --steps 5: 64 effective warmup batches + 5 timed
CFGS = {"fsk2": (2, "goertzel_tile_kernel", 1024), "fsk8": (8, "fold_tile_kernel", 1024),
        "fsk8odd": (8, "residue_tile_kernel", 1024), "fft": (2, "fft1024_quad_kernel", 256),
        "fft1024": (2, "fft1024_quad_kernel", 1024)}


def main(rnd="round1", sub=""):
    base = os.path.join(ROOT, "gpurun_out", sub)
    os.makedirs(os.path.join(ROOT, "profiles", rnd), exist_ok=True)
    for tag, (k, kname, hop) in CFGS.items():
        if sub and tag.startswith("fft"):
            continue  # round 3: the FFT passes go through scripts/pmc_fft_r3_json.py
        if not os.path.exists(os.path.join(base, f"pmc_{tag}_FETCH_SIZE")):
            continue
        vals, name = {}, None
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            src = os.path.join(base, f"pmc_{tag}_{c}", "run_counter_collection.csv")
            rows = sorted((r for r in csv.DictReader(open(src)) if r["Counter_Name"] == c),
                          key=lambda r: int(r["Dispatch_Id"]))
            name = next(r["Kernel_Name"] for r in rows if kname in r["Kernel_Name"])
            # one batch = `per` consecutive detector launches: the bench line of
            # the pass gives launches_per_step, less the rescue's launch when
            # the trace has one (round-2 launch slices: 4 + 1; round 3: 1 + 1,
            # or 1 where the detector rescues in its own kernel); round 3
            # keeps the first MAX_BATCHES (warmup + timed steps): the bench's
            # sustained phase re-reads the same input back to back
            det = [float(r["Counter_Value"]) for r in rows if kname in r["Kernel_Name"]]
            per = 1
            if sub:
                line = [ln for ln in open(os.path.join(base, f"pmc_{tag}_{c}.log"))
                        if ln.startswith("{")][-1]
                lps = int(json.loads(line)["roofline"]["launches_per_step"])
                per = max(1, lps - (1 if any("rescue_kernel" in r["Kernel_Name"] for r in rows) else 0))
            v = [sum(det[i:i + per]) for i in range(0, len(det) - per + 1, per)]
            if sub:
                v = v[:MAX_BATCHES]
            vals[c] = (sum(v) / len(v), len(v))
            dst = os.path.join(ROOT, "profiles", rnd, f"pmc_{tag}_{c}.csv")
            if sub and tag == "fsk2":  # the sustained phase's ~30k rows are not kept
                with open(src) as fi, open(dst, "w") as fo:
                    fo.writelines(line for i, line in enumerate(fi) if i <= 200)
            else:
                shutil.copy(src, dst)
        rd = vals["FETCH_SIZE"][0] * 1024 * 2
        wr = vals["WRITE_SIZE"][0] * 1024
        n_eval = (W * 1024 - 1024) // hop + 1
        alg = W * 2048 + n_eval * (1 + 4 * k)
        out = {
            "config": tag, "windows": W, "hop": hop, "windows_evaluated": n_eval, "kernel": name,
            "batches_sampled": vals["FETCH_SIZE"][1],
            "FETCH_SIZE_kb_per_batch": vals["FETCH_SIZE"][0],
            "WRITE_SIZE_kb_per_batch": vals["WRITE_SIZE"][0],
            "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            # "per launch" as bench.py reads it: one batch, all its detector launches
            "hbm_bytes_per_launch": rd + wr, "alg_bytes_per_launch": alg,
            "traffic_over_alg": (rd + wr) / alg,
            "method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                       "bench.py (" + (f"scripts/gpu_run.sh {sub} pmc, closing check" if sub else
                                       "round 2 profiling scripts")
                       + "); bytes = KB*1024, FETCH doubled "
                       "per MI355X_MICROARCH.md §HBM (gfx950 counts 1/2 of 16 B/lane streaming "
                       "reads); calibration: the 16 B/lane synth_kernel write of 2 GiB reads "
                       "WRITE_SIZE 2105344 KB = 2.0078 GiB"),
            "source": f"profiles/{rnd}/pmc_{tag}_FETCH_SIZE.csv, pmc_{tag}_WRITE_SIZE.csv"
                      + (" (first 200 dispatches kept in the copy)" if sub and tag == "fsk2" else ""),
        }
        json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
        print(tag, name[:60], out["batches_sampled"], round(out["traffic_over_alg"], 5))


if __name__ == "__main__":
    import sys
    main(*sys.argv[1:])
