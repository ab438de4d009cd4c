# SQ/GRBM counters of the shipped 8-tone kernels (one probe variant per pass):
# issue utilisation by instruction type and effective clock.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
for f in "residue K=8o WPB=4" "goertzel PK WS K=8o" "fold WS LDST K=8 WPB=2" "goertzel K2 K=2 WPB=2"; do
  tag=$(echo "$f" | tr -c 'A-Za-z0-9' '_')
  PROBE_FILTER="$f" timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/sq_$tag -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/sq_$tag.log 2>&1 || exit 1
done
