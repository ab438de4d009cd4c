"""Can two RCCL ranks share one GPU here? (probe: if so, bench.py's N > 1
configs[4] graph bucket can be exercised on the one-GPU box)."""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank), device=dev)
out = torch.empty(4 * world, device=dev)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: {out.tolist()}", flush=True)
dist.destroy_process_group()
sys.exit(0)
