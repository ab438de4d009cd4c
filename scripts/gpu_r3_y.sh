# Round 3: 8-FSK input load cache policy with the magnitude stream
# (scripts/mag_probe.hip loads).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3y}
mkdir -p $O
cd $R
timeout -k 10 300 scripts/bin/mag_probe 6 5 loads > $O/mag_probe_loads.log 2>&1 || exit $?
