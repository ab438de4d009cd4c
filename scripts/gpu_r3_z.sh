# Round 3 closing check on the final tree: the GPU suite, smoke, the driver's
# bench command, rocprofv3 kernel-trace stats of that command, the HBM PMC
# passes (FETCH_SIZE, WRITE_SIZE in separate runs) of the 2-FSK / 8-FSK
# detectors and of the FFT detector at hop 256 (tones only, with the
# spectrum), and one SQ pass of the tones-only FFT kernel (issue counts per
# group after the gathered tone pick).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3z}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit $?
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain 0 > $O/kt.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  for cfg in fsk2 fsk8; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${cfg}_$c -o run -- python3 $R/bench.py --config $cfg --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5 > $O/pmc_${cfg}_$c.log 2>&1 || exit $?
  done
  B="python3 $R/bench.py --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5"
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_fft_$c -o run -- $B > $O/pmc_fft_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_fftspec_$c -o run -- $B --spectrum > $O/pmc_fftspec_$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq_fft -o run -- python3 $R/bench.py --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5 > $O/sq_fft.log 2>&1 || exit $?
