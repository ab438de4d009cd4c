# Tuning probe + bench + kernel-trace profile on the GPU box.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 $R/scripts/bin/probe 1048576 5 10 > $R/gpurun_out/probe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5 > $R/gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 --steps 20 --warmup 5 --cpu-seconds 5 > $R/gpurun_out/bench_fsk8.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
