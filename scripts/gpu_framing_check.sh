# GPU parity suite + config-5 bench (device framing) at 1 rank and a 2-rank
# gloo rehearsal of the frame gather on the one-GPU box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config streams --cpu-seconds 3 > $R/gpurun_out/bench_streams.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config streams --steps 3 --warmup 1 --dist-backend gloo > $R/gpurun_out/dist_streams_2.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --windows 65536 --dist-backend gloo > $R/gpurun_out/dist_2.log 2>&1
