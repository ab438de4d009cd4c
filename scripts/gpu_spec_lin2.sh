# Spectrum store: linear slab with plain vs nt 16-byte stores, and a
# write-only fill of the same buffer as the write reference. (Run when
# launch_fft_quad read FSKD_SPL_NT to pick the nt variant; nt shipped and the
# switch is gone, so both passes now run the shipped kernel.)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spec_lin
mkdir -p $O
cd $R
timeout -k 10 300 python -u scripts/spectrum_probe.py > $O/spectrum_probe2.log 2>&1 && \
FSKD_SPL_NT=1 timeout -k 10 300 python -u scripts/spectrum_probe.py > $O/spectrum_probe2_nt.log 2>&1
