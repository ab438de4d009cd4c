# Default bench twice with the swizzled 2-wave read-ceiling reference.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 > gpurun_out/ceil_$i.log 2>&1 || exit 1
done
