# quad-layout FFT detector: GPU parity (FFT tests through the C ABI), then the probe A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "fft or FFT" > $O/pytest_fftq.log 2>&1 || exit 1
PROBE_FILTER=fft timeout -k 10 300 $R/scripts/bin/probe 1048576 6 10 > $O/probe_fftq.log 2>&1
