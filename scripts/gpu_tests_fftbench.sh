set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > $R/gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --cpu-seconds 5 > $R/gpurun_out/bench_fft.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --hop 1024 --cpu-seconds 3 > $R/gpurun_out/bench_fft1024.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 --method goertzel --cpu-seconds 3 > $R/gpurun_out/bench_fsk8_plain.log 2>&1
