"""Same box: bench.host_e2e (as in bench.py) in different process states:
before torch touches the GPU, after torch's CUDA init, after a device-resident
bench leg — with the cgroup's CPU throttling (cpu.stat) over each run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def cpu_stat():
    try:
        return dict(l.split() for l in open("/sys/fs/cgroup/cpu.stat"))
    except OSError:
        return {}


def run(tag):
    a = cpu_stat()
    r = bench.host_e2e("imix", 1, 10_000, 0x7CBEE)
    b = cpu_stat()
    print(tag, {k: v["mpkts"] for k, v in r.items() if isinstance(v, dict) and "mpkts" in v},
          "throttled_usec", int(b.get("throttled_usec", 0)) - int(a.get("throttled_usec", 0)),
          flush=True)


run("fresh")
import torch  # noqa: E402
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
run("torch-cuda")
torch.cuda.set_stream(torch.cuda.Stream())
bench.run_device(torch, None, 0, 1, 20_000_000, "imix", 1, 10_000, 5, 2, 0x7CBEE)
run("after-device-leg")
run("again")
