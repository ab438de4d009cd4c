# GPU parity suite + host-buffer boundary throughput.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u scripts/host_path_bench.py > $R/gpurun_out/host.log 2>&1
