# Round-2 profiles of the shipped tree: kernel-trace stats of the default
# bench.py run (configs[1] + the fsk8 / fft_hop256 extras), then per-launch HBM
# traffic (FETCH_SIZE and WRITE_SIZE in separate passes: they do not fit one
# TCC pass) for every detector the bench line reports.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 $R/bench.py --no-cpu-baseline > $O/kt_default.log 2>&1 || exit 1
B="python3 $R/bench.py --no-cpu-baseline --no-extras --warmup 2 --steps 5"
for spec in "fsk2:--config fsk2" "fsk8:--config fsk8" "fsk8odd:--config fsk8 --plan odd" "fft:--config fft --hop 256" "fft1024:--config fft --hop 1024"; do
  tag=${spec%%:*}; args=${spec#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${tag}_$c -o run -- $B $args > $O/pmc_${tag}_$c.log 2>&1 || exit 1
  done
done
