# More seeds of the GPU random sweeps (parity breadth; results under
# gpurun_out/<prefix>_<seed>/): tests/test_gpu_sweep.py (random plans,
# levels, hops, batch sizes) and the rescued-decision sweep over all ten
# signal families (FSKD_SWEEP_ALL=1).
#   gpurun -- bash scripts/sweep_seeds.sh <prefix> <seed> [<seed> ...]
pre=${1:?prefix}
shift
export FSKD_SWEEP_ALL=1
for sd in "$@"; do
  FSKD_SWEEP_SEED=$sd bash scripts/gpu_run.sh ${pre}_$sd \
    "pyt:600:-m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_sweep.py" \
    "pyt:300:-m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_error_model.py::test_rescued_decisions_every_window" || exit $?
done
