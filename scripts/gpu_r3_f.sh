# Round 3: the FFT rescue inside the detector (rescue_fft.h): the GPU suite,
# the FFT rescue cost by signal, bench --config fft at hop 256 (tones only and
# with the full spectrum).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3g}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "fft or FFT or decision or near_ties or spectrum" > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/rescue_cost.py --only fft > $O/rescue_cost.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config fft --hop 256 --no-cpu-baseline --steps 50 > $O/bench_fft.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config fft --hop 256 --spectrum --no-cpu-baseline --steps 50 > $O/bench_fft_spec.log 2>&1 || exit $?
