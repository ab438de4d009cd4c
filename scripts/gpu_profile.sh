# Round profiles: bench lines, kernel-trace stats, and PMC traffic passes
# (FETCH_SIZE and WRITE_SIZE in separate runs: they do not fit one TCC pass).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --warmup 2 --steps 5"
for cfg in fsk2 fsk8; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$cfg -o run -- python3 $R/bench.py --config $cfg --warmup 20 --steps 100 --no-cpu-baseline > $O/kt_$cfg.log 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${cfg}_$c -o run -- $B --config $cfg > $O/pmc_${cfg}_$c.log 2>&1 || exit 1
  done
done
cd $R && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_fsk2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config fsk8 --steps 20 --warmup 5 > $O/bench_fsk8.log 2>&1
