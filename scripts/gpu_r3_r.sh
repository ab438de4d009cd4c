# Round 3: non-temporal K >= 8 magnitude stores, 8-FSK in one launch: the GPU
# suite, configs[2] through bench.py, and the store-policy probe again.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3r}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config fsk8 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_fsk8.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/mag_probe 6 5 > $O/mag_probe.log 2>&1 || exit $?
