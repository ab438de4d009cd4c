set -o pipefail
R=$GRAFT_REPO_ROOT
for v in "fold WS LDST K=8 WPB=2" "fold WS PK LDST K=8 WPB=2" "fold WS LDST K=8 WPB=2" "fold WS PK LDST K=8 WPB=2"; do
  PROBE_FILTER="$v" timeout -k 10 100 $R/scripts/bin/probe 1048576 2 60 >> $R/gpurun_out/sustained.log 2>&1 || exit 1
done
