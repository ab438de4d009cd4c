# bench.py with kernel events on every 4th timed step: default twice, streams
# with RCCL, the streams / multi-rank GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/evev_1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/evev_2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config streams --force-dist > gpurun_out/evev_streams.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/evev_pytest.log 2>&1
