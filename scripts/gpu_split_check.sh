# Output-size launch split: split probe, default bench twice, streams, GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/split_launch_probe.py > gpurun_out/split_launch2.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/split_def_$i.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --config streams > gpurun_out/split_streams.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
