# SQ counters for the FFT detector kernel (hop 256) and the plain K=8 Goertzel.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
for f in "hop=256 swz=1" "goertzel [default] K=8"; do
  tag=$(echo "$f" | tr -c 'a-zA-Z0-9' '_')
  PROBE_FILTER="$f" timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc_$tag -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_$tag.log 2>&1 || exit 1
done
