# SQ/GRBM counters for the VALU-bound kernels (plain Goertzel K=8, FFT quad
# hop 256): issue utilisation and effective clock. One pass per counter set.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
for f in "PK [default] K=8" "hop=256 swz=0 QUAD-new"; do
  tag=$(echo "$f" | tr -c 'A-Za-z0-9' '_')
  PROBE_FILTER="$f" timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_$tag -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_$tag.log 2>&1 || exit 1
done
