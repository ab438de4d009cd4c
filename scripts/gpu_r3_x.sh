# Round 3: bench.py with the N > 1 watchdog: the streams GPU tests (self-launch
# over gloo, with and without the watchdog firing) and the driver's N = 1 command.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3x}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_streams.py > $O/pytest_streams.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
