import os
print("before", len(os.sched_getaffinity(0)), flush=True)
import numpy as np
print("numpy", len(os.sched_getaffinity(0)), flush=True)
import torch
print("torch", len(os.sched_getaffinity(0)), torch.get_num_threads(), flush=True)
x = torch.randn(1000, 1000); y = x @ x
print("torch op", len(os.sched_getaffinity(0)), flush=True)
torch.cuda.init(); torch.zeros(1, device="cuda")
print("cuda", len(os.sched_getaffinity(0)), flush=True)
print({k: v for k, v in os.environ.items() if "OMP" in k or "KMP" in k or "GOMP" in k or "MKL" in k})
