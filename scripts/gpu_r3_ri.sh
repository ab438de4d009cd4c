# Round 3, late: the 2-FSK plain bank's decision rescue inside the detector
# kernel (rescue_row) against the separate rescue launch
# (FSKD_RESCUE_LAUNCH=1): bench.py interleaved, three rounds; then the GPU
# suite (near ties on the 2-FSK path now rescued in the kernel) and smoke.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3ri}
mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --steps 40 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 120 $B > $O/fsk2_inline_$i.log 2>&1 || exit $?
  FSKD_RESCUE_LAUNCH=1 timeout -k 10 120 $B > $O/fsk2_launch_$i.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
