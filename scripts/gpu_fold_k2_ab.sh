#!/bin/bash
# the fold detector against the plain bank on the 2-FSK
# survey plan (bins 32 / 64), configs[1] at full size, interleaved A/B runs
# of the headline step (no extras), 200 timed steps each.
set -o pipefail
out=gpurun_out/${1:-r6fold}
mkdir -p "$out"
for rep in 1 2 3; do
  for m in auto folded; do
    timeout -k 10 240 python -u bench.py --method $m --no-extras --no-cpu-baseline --sustain 0 \
        --no-rescue-ab --steps 200 --warmup 20 > "$out/${m}_$rep.json" 2> "$out/${m}_$rep.err" || exit $?
    python -c "import json,sys; d=json.loads(open('$out/${m}_$rep.json').read().strip().splitlines()[-1]); print('$m', $rep, d['detector'], d['ms_per_step'], d['kernel_ms'], d['kernel_ms_p10_p50_p90'], d['symbol_errors'], d['roofline']['frac'])"
  done
done
