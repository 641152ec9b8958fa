"""Two processes on one GPU (torchrun --nproc-per-node 2, gloo): how a plain
HBM-bound torch kernel (a 2 GiB device copy) shares the chip, to put K1's
two-process time (tools/lookback_contention.sh) beside the platform's own.
Prints per rank the copy time alone (rank 1 idle) and with both ranks copying."""
import os
import time

import torch
import torch.distributed as dist

rank = int(os.environ.get("RANK", "0"))
torch.cuda.set_device(0)
dist.init_process_group("gloo")
src = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
iters = 20


def run(active):
    dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    if active:
        for _ in range(iters):
            dst.copy_(src)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / iters * 1e3
    dist.barrier()
    return el


run(True)
solo = run(rank == 0)
both = run(True)
print(f"rank {rank}: 2 GiB copy alone {solo:.3f} ms, both ranks copying {both:.3f} ms "
      f"({both / solo:.2f}x)" if rank == 0 else f"rank {rank}: both {both:.3f} ms", flush=True)
dist.destroy_process_group()
