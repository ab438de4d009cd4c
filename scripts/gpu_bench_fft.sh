set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 $R/scripts/bin/probe 1048576 5 10 > $R/gpurun_out/probe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --cpu-seconds 5 > $R/gpurun_out/bench_fft.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fft --hop 1024 --cpu-seconds 3 > $R/gpurun_out/bench_fft1024.log 2>&1
