# FFT full-spectrum store through the linear power slab: FFT GPU tests, then
# the spectrum probe (aligned = linear slab, unaligned = quad_slot slab).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spec_lin
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fft" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_fft.log 2>&1 && \
timeout -k 10 300 python -u scripts/spectrum_probe.py > $O/spectrum_probe.log 2>&1
