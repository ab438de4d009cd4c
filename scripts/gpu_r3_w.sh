# Round 3: FFT input as wide loads staged through LDS (WL 1) against the
# shipped 32 dword loads: hop 256 with the spectrum and tones only, hop 512
# with the spectrum.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3w}
mkdir -p $O
cd $R
timeout -k 10 200 scripts/bin/fft_probe 256 5 5 "wl" spec > $O/probe_wl_256_spec.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 256 5 8 "wl" > $O/probe_wl_256.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 512 5 5 "wl" spec > $O/probe_wl_512_spec.log 2>&1 || exit $?
