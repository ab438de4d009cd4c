# HBM traffic per launch of the shipped detector kernels (rocprofv3 PMC):
# FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit one TCC pass),
# bench.py --no-cpu-baseline --warmup 2 --steps 5 (70 launches: 64 forced warmup + 5 + ...).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --warmup 2 --steps 5"
for spec in "fsk2:--config fsk2" "fsk8:--config fsk8" "fsk8odd:--config fsk8 --plan odd"; do
  tag=${spec%%:*}; args=${spec#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${tag}_$c -o run -- $B $args > $O/pmc_${tag}_$c.log 2>&1 || exit 1
  done
done
