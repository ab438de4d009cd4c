#!/bin/bash
# Interleaved A/B of the shipped library against a variant build (FSKD_LIB)
# on one bench configuration: scripts/gpu_lib_ab.sh <outdir> <variant.so> <bench args...>
set -o pipefail
out=gpurun_out/$1; var=$2; shift 2
mkdir -p "$out"
for rep in 1 2 3; do
  for v in shipped variant; do
    if [ $v = variant ]; then export FSKD_LIB=$var; else unset FSKD_LIB; fi
    timeout -k 10 240 python -u bench.py "$@" --no-extras --no-cpu-baseline --sustain 0 --no-rescue-ab \
        > "$out/${v}_$rep.json" 2> "$out/${v}_$rep.err" || exit $?
    python -c "import json; d=json.loads(open('$out/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, d['detector'], d['ms_per_step'], d['kernel_ms'], d['kernel_ms_p10_p50_p90'], d['symbol_errors'], d['roofline']['frac'])"
  done
done
