# Round 3: FFT rescue cost (bench --config fft), the rescue cost by detector
# and signal (scripts/rescue_cost.py), the FFT probe's TW3R variants.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3e}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --config fft --hop 256 --no-cpu-baseline --steps 50 > $O/bench_fft.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/rescue_cost.py > $O/rescue_cost.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 6 10 "tw3:" > $O/probe_tw3_256.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 4 10 "tw3:" spec > $O/probe_tw3_256_spec.log 2>&1 || exit $?
