# The GPU random sweep with more case sets (FSKD_SWEEP_SEED 1..3, or the list in FSKD_SEEDS).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for s in ${FSKD_SEEDS:-1 2 3}; do
FSKD_SWEEP_SEED=$s timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sweep_seed$s.log 2>&1 || exit 1
done
