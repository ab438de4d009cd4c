# Spectrum FFT kernel after the spill fix (SPL slab addresses formed from a
# fenced lane id): FFT parity tests, the spectrum probe, the probe's PF / MINW
# variants against the shipped kernel, and the default bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spec_nospill
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "fft or spectrum" > $O/pytest_fft.log 2>&1 && \
timeout -k 10 300 python -u scripts/spectrum_probe.py > $O/spectrum_probe.log 2>&1 && \
timeout -k 10 120 scripts/bin/fft_probe 256 6 10 pfx > $O/fft_probe_pfx.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
