# Round 3: FFT probe A/B of the decision rescue inside the detector (rsc
# variants: compiled out / in and off / flags only / per-wave / per-block),
# tones only and with the spectrum, hop 256.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3j}
mkdir -p $O
cd $R
timeout -k 10 300 scripts/bin/fft_probe 256 8 10 rsc > $O/probe_rsc_256.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 6 10 rsc spec > $O/probe_rsc_256_spec.log 2>&1 || exit $?
