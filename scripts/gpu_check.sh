# GPU tests + smoke + bench lines for every config + kernel-trace profile.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rocm-smi --showproductname > $R/gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > $R/gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $R/gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 > $R/gpurun_out/bench_fsk8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 --plan odd --cpu-seconds 5 > $R/gpurun_out/bench_fsk8_odd.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 --plan odd --method goertzel --no-cpu-baseline > $R/gpurun_out/bench_fsk8_odd_plain.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config streams --cpu-seconds 3 > $R/gpurun_out/bench_streams.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --cpu-seconds 5 > $R/gpurun_out/bench_fft.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --hop 1024 --cpu-seconds 5 > $R/gpurun_out/bench_fft1024.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 20 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fft -o run -- python3 $R/bench.py --config fft --steps 20 --no-cpu-baseline > $R/gpurun_out/prof_fft.log 2>&1
