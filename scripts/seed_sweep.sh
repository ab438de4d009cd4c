# GPU box: the random sweep and the all-family rescued-decision sweep at extra
# seeds (each step under its own time limit; the first failure ends the run).
#   gpurun -- bash scripts/seed_sweep.sh <outdir> <seed> [<seed> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:?outdir}
shift
mkdir -p "$O"
cd "$R"
for s in "$@"; do
  echo "[$(date +%T)] seed $s" | tee -a "$O/steps.log"
  FSKD_SWEEP_SEED=$s timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_sweep.py > "$O/seed${s}_sweep.log" 2>&1 || exit $?
  FSKD_SWEEP_SEED=$s FSKD_SWEEP_ALL=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_error_model.py -k rescued > "$O/seed${s}_rescued_all_families.log" 2>&1 || exit $?
done
echo "[$(date +%T)] done" | tee -a "$O/steps.log"
