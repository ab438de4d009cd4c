set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 && \
PROBE_FILTER=fft1024 timeout -k 10 300 $R/scripts/bin/probe 1048576 5 10 > $R/gpurun_out/probe.log 2>&1
