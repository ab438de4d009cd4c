set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for m in goertzel folded; do
  timeout -k 10 300 python -u bench.py --method $m --warmup 20 --steps 200 --no-cpu-baseline > $R/gpurun_out/sustain_fsk2_$m.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --config fsk8 --method $m --warmup 20 --steps 200 --no-cpu-baseline > $R/gpurun_out/sustain_fsk8_$m.log 2>&1 || exit 1
done
timeout -k 10 300 $R/scripts/bin/probe 1048576 5 10 > $R/gpurun_out/probe.log 2>&1
