"""Probe: can two RCCL ranks share one GPU on this box? (all_gather_into_tensor of
a few ints). Prints one line per rank; exits non-zero if the collective fails.
Run as: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/nccl_same_dev.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda")
out = torch.empty(4 * world, dtype=torch.int64, device="cuda")
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: {out.tolist()}", flush=True)
dist.barrier()
dist.destroy_process_group()
