# Residue-class detector: GPU parity tests, then interleaved A/B vs the plain
# bank and the multiple-of-8 fold (scripts/probe.hip), one process.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_residue.log 2>&1 && \
PROBE_FILTER="${PROBE_FILTER:-residue|goertzel PK [default]|goertzel [default]|goertzel PK K=|fold K=8|read-only one-shot tile (8 KiB/wave, nt, 4}" timeout -k 10 300 $R/scripts/bin/probe 1048576 6 10 > $R/gpurun_out/probe_residue.log 2>&1
