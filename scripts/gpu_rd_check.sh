# FFT detector: unpaired LDS reads (RD 1) and lane-major twiddle tables (RD 2) against the shipped kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 250 scripts/bin/fft_probe 256 8 10 > gpurun_out/probe_rd_256.log 2>&1 || exit 1
timeout -k 10 150 scripts/bin/fft_probe 1024 6 10 > gpurun_out/probe_rd_1024.log 2>&1
