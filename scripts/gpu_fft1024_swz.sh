# FFT detector at hop 1024 with the XCD swizzle (bench.py --config fft --hop 1024), twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --config fft --hop 1024 > gpurun_out/fft1024_swz_$i.log 2>&1 || exit 1
done
