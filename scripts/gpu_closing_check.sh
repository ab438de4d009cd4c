# Round-2 closing check of the tree (threaded streams staging included):
# whole GPU suite, smoke, default bench (with CPU baseline and
# the three extras), configs[4] with RCCL at N = 1, kernel-trace stats of the
# default bench command.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final13
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config streams --force-dist > $O/bench_streams.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $R/bench.py --no-cpu-baseline > $O/kt_default.log 2>&1
