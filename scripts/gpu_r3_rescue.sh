# Round 3: the decision rescue on the GPU — whole GPU suite (failures listed,
# not stopping at the first), then the default bench with and without the
# rescue (FSKD_NO_RESCUE=1) to price it. A test failure (rc 1) is not a GPU
# fault and lets the benches run; anything else stops the script.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3a}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
FSKD_NO_RESCUE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_norescue.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench2.log 2>&1 || exit $?
exit $rc
