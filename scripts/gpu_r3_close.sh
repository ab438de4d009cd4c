# Round 3 closing check on the final tree: the GPU suite, smoke, the
# driver's bench command, rocprofv3 kernel-trace stats of that command, and
# the HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) of the FFT
# detector at hop 256, tones only and with the spectrum (the in-kernel rescue
# changed that kernel this round).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3close}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain 0 > $O/kt.log 2>&1 || exit $?
B="python3 $R/bench.py --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_fft_$c -o run -- $B > $O/pmc_fft_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_fftspec_$c -o run -- $B --spectrum > $O/pmc_fftspec_$c.log 2>&1 || exit $?
done
