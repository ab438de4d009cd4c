# Round 2: new GPU tests first, then the whole GPU suite, smoke, default bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'; cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > $O/cpu_share.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r2_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
