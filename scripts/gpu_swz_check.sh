# XCD-swizzled tiles at hop = n: default bench (2-FSK + extras), 8-FSK odd plan
# (residue), configs[4] streams, each twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/swzc_def_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --config fsk8 --plan odd > gpurun_out/swzc_odd_$i.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --config streams > gpurun_out/swzc_streams_$i.log 2>&1 || exit 1
done
