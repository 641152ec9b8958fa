"""PCIe ceiling of the E2E leg on this box: 1.5 GB device -> pinned host, pinned host
-> device, and both at once on two streams (the pipe's shape: header windows in,
records out), torch copies on pinned (hipHostMalloc) memory, best of 5."""
import time

import torch

n = 1_500_000_000
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def best(fn):
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return min(ts)


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


a, b, c = best(h2d), best(d2h), best(both)
print(f"H2D {n / a / 1e9:.1f} GB/s, D2H {n / b / 1e9:.1f} GB/s, both at once "
      f"{n / c / 1e9:.1f} GB/s each way ({c * 1e3:.1f} ms for 2 x 1.5 GB)", flush=True)
