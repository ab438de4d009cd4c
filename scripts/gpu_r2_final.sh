# Round-2 final check: whole GPU suite, smoke, default bench (with CPU
# baseline), configs[4] streams with RCCL at N = 1, the sliding probe.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
cd $R
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'; cat /sys/fs/cgroup/cpu.max 2>&1; } > $O/cpu_share.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config streams --force-dist > $O/bench_streams.log 2>&1 && \
timeout -k 10 300 python -u scripts/sliding_probe.py > $O/sliding.log 2>&1
