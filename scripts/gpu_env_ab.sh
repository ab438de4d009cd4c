#!/bin/bash
# Interleaved env A/B of the headline step (no extras): scripts/gpu_env_ab.sh
# <outdir> <rounds> "<bench args>" "<ENV=V ...>" ["<ENV=V ...>" ...]
# ("-" for no environment). One line per run: label, ms_per_step, kernel p10/p50/p90.
set -o pipefail
out=gpurun_out/$1; rounds=$2; args=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  i=0
  for ev in "$@"; do
    i=$((i + 1))
    e=$ev; [ "$e" = "-" ] && e="X_NONE=1"
    env $e timeout -k 10 200 python3 bench.py $args --no-extras --no-cpu-baseline --sustain 0 --no-rescue-ab \
        > "$out/v${i}_$r.json" 2> "$out/v${i}_$r.err" || exit $?
    python3 -c "import json; d=json.loads(open('$out/v${i}_$r.json').read().strip().splitlines()[-1]); print('$ev', '$args', $r, d['detector'], d['ms_per_step'], d['kernel_ms_p10_p50_p90'], d['symbol_errors'])"
  done
done
