# Packet-sized host calls through mapped coherent pinned memory (no copies):
# whole GPU suite, then the host-path bench with and without the zero-copy
# path (FSKD_NO_ZERO_COPY=1), twice each, interleaved.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/zero_copy
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u scripts/host_path_bench.py > $O/host_path_zc1.log 2>&1 && \
FSKD_NO_ZERO_COPY=1 timeout -k 10 300 python -u scripts/host_path_bench.py > $O/host_path_copy1.log 2>&1 && \
timeout -k 10 300 python -u scripts/host_path_bench.py > $O/host_path_zc2.log 2>&1 && \
FSKD_NO_ZERO_COPY=1 timeout -k 10 300 python -u scripts/host_path_bench.py > $O/host_path_copy2.log 2>&1
