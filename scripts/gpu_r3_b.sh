# Round 3, second check: GPU suite, default bench (CPU baseline included),
# the FFT probe's OVL variants at hop 256 / 1024, the streams-push staging A/B.
# A test failure (rc 1) is not a GPU fault; any other non-zero status stops.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3b}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 6 10 "ovl:" > $O/probe_ovl_256.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 1024 6 10 "ovl:" > $O/probe_ovl_1024.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/streams_push_ab.py > $O/push_ab.log 2>&1 || exit $?
exit $rc
