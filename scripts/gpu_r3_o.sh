# Round 3: plain loads in the FFT rescue's read-back, XCD-aware chunks in the
# Goertzel rescue: FFT / decision / Goertzel parity tests, FFT PMC traffic,
# kernel-trace durations of the headline step (detector + rescue).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3o}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "fft or FFT or decision or near_ties or parity" > $O/pytest_gpu.log 2>&1 || exit $?
cd /tmp
B="python3 $R/bench.py --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_fft_$c -o run -- $B > $O/pmc_fft_$c.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --sustain 0 > $O/kt.log 2>&1 || exit $?
