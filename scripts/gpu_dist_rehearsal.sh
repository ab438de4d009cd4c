# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 and 3 ranks share the
# GPU, collectives over gloo (the real node uses RCCL). Small batches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for np in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $np --steps 5 --warmup 2 --windows 65536 --dist-backend gloo > $R/gpurun_out/dist_$np.log 2>&1 || exit 1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus $np --config streams --steps 3 --warmup 1 --dist-backend gloo > $R/gpurun_out/dist_streams_$np.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --cpu-seconds 3 > $R/gpurun_out/bench.log 2>&1
