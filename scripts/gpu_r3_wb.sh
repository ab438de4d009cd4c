# Round 3, late: one launch with L2 write-back bursts (GoertzelParams::wb_bursts)
# for Goertzel-family batches with > 10 MiB of output, against the round-2
# launch slices (FSKD_WB_BURSTS=0): the probe's variants, then bench.py A/B per
# config (interleaved, two runs each way), then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3wb}
mkdir -p $O
cd $R
timeout -k 10 200 scripts/bin/mag_probe 8 5 wb > $O/mag_probe_wb.log 2>&1 || exit $?
B="python3 bench.py --no-cpu-baseline --no-rescue-ab --steps 20 --warmup 5"
for i in 1 2; do
  for cfg in "--config fsk8" "--config fsk8 --plan odd" "--config streams"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 200 $B $cfg > $O/bench_${tag}_wb_$i.log 2>&1 || exit $?
    FSKD_WB_BURSTS=0 timeout -k 10 200 $B $cfg > $O/bench_${tag}_slices_$i.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
