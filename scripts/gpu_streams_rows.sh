# Streams.push with a 2-D array of packets (row addresses computed) and the
# list path's leaner marshalling: streams GPU tests and the push bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/streams_rows
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_streams_push.py > $O/pytest_streams.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py > $O/push_bench.log 2>&1
