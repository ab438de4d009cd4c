# Round 2: FFT detector parity (all FFT GPU tests), A/B probe, bench line and
# kernel-trace stats of the shipped kernel.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -k "fft or FFT or near_ties or dc_and_nyquist or threads or sweep" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_fft.log 2>&1 && \
timeout -k 10 200 scripts/bin/fft_probe 256 5 10 > $O/fft_probe.log 2>&1 && \
timeout -k 10 100 scripts/bin/fft_probe 1024 4 10 >> $O/fft_probe.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config fft --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench_fft.log 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fft -o run -- python3 $R/bench.py --config fft --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_fft.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fft_FETCH_SIZE -o run -- python3 $R/bench.py --config fft --no-cpu-baseline --warmup 2 --steps 5 > $O/pmc_fft_FETCH_SIZE.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_fft_WRITE_SIZE -o run -- python3 $R/bench.py --config fft --no-cpu-baseline --warmup 2 --steps 5 > $O/pmc_fft_WRITE_SIZE.log 2>&1
