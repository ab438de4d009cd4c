# demod_streams_push staging each stream within its own hops, on several host
# threads for large pushes: streams GPU tests (incl. 1024 streams) and the
# push bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-streams_mt}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_streams_push.py tests/test_native.py tests/test_gpu_streams.py > $O/pytest_streams.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py > $O/push_bench.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py > $O/push_bench2.log 2>&1
