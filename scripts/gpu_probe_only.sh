set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 $R/scripts/bin/probe 1048576 8 10 > $R/gpurun_out/probe.log 2>&1
