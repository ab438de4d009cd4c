# Round 3: the 8-FSK magnitude stream by store policy and launch slicing
# (scripts/mag_probe.hip).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3q}
mkdir -p $O
cd $R
timeout -k 10 300 scripts/bin/mag_probe 6 5 > $O/mag_probe.log 2>&1 || exit $?
