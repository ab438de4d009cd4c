# FFT detector with direct spectrum stores: FFT GPU tests, spectrum probe, probe A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "fft or FFT or spectrum" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_spec.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/spectrum_probe.py > gpurun_out/spectrum2.log 2>&1 || exit 1
timeout -k 10 250 scripts/bin/fft_probe 256 6 10 > gpurun_out/probe_spec.log 2>&1
