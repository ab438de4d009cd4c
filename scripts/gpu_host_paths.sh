# Host-pointer paths (zero-copy / pinned round trip / chunked) against the
# device-pointer call, every detector, boundary sizes.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/host_paths
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_host_paths.py > $O/pytest_host_paths.log 2>&1
