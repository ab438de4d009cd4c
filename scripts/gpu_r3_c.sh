# Round 3, third check: GPU suite, default bench, kernel-trace stats of the
# default bench command (profiles/), the FFT probe's spectrum variants (PF 2).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3c}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 4 10 "spl:" spec > $O/probe_spl_256.log 2>&1 || exit $?
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $R/bench.py --no-cpu-baseline > $O/kt_default.log 2>&1 || exit $?
exit $rc
