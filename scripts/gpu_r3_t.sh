# Round 3: lane 0's post-pass pairing through masked LDS (L0 1) against the
# shipped selects; tones only at hop 256 / 1024, and the spectrum at hop 256.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3t}
mkdir -p $O
cd $R
timeout -k 10 200 scripts/bin/fft_probe 256 6 10 "l0" > $O/probe_l0_256.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 1024 6 10 "l0" > $O/probe_l0_1024.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 256 4 5 "l0" spec > $O/probe_l0_256_spec.log 2>&1 || exit $?
