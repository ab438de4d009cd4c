# demod_streams_push writing each packet straight into the pinned staging
# buffer (one host copy): the streams GPU tests, the native C test, and the
# push bench for this build and the previous one (scripts/bin/libfskdemod_prev.so)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/streams_direct
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_streams_push.py tests/test_native.py > $O/pytest_streams.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py > $O/push_bench_new.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py --lib scripts/bin/libfskdemod_prev.so > $O/push_bench_prev.log 2>&1 && \
timeout -k 10 300 python -u scripts/streams_push_bench.py > $O/push_bench_new2.log 2>&1
