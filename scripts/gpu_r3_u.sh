# Round 3: the gathered FFT tone pick shipped (PICK 1): the GPU suite and the
# configs[3] line (hop 256, tones only).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3u}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config fft --steps 20 --warmup 5 > $O/bench_fft.log 2>&1 || exit $?
