# Round 3: FFT detector tone pick gathered by ds_bpermute (PICK 1) against the
# shipped register pick, hop 256 and 1024, interleaved in one process.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3s}
mkdir -p $O
cd $R
timeout -k 10 200 scripts/bin/fft_probe 256 6 10 "pick" > $O/probe_pick_256.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 1024 6 10 "pick" > $O/probe_pick_1024.log 2>&1 || exit $?
