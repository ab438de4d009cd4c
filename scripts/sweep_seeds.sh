export FSKD_SWEEP_ALL=1
for sd in 101 202 303 404; do
  FSKD_SWEEP_SEED=$sd bash scripts/gpu_run.sh r4t_$sd "pyt:300:-m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_error_model.py -k rescued" || exit $?
done
