# Round 3: default bench line (parity over the whole timed output, sustained
# phase), and on the same box the spectrum kernel against the memory floor
# of its own traffic (scripts/spec_mem_probe.hip).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3m}
mkdir -p $O
cd $R
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/spec_mem_probe 4 4 > $O/spec_mem_probe.log 2>&1 || exit $?
timeout -k 10 200 scripts/bin/fft_probe 256 4 5 "quad shipped" spec > $O/probe_spec_256.log 2>&1 || exit $?
