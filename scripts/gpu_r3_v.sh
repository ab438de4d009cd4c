# Round 3: the spectrum kernel's memory floor with wide reads (each group's
# span once, 16 B per lane) against the detector's 32 dword loads.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3v}
mkdir -p $O
cd $R
timeout -k 10 300 scripts/bin/spec_mem_probe 4 5 > $O/spec_mem_probe.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 256 4 5 "pick" spec > $O/probe_spec_256.log 2>&1 || exit $?
