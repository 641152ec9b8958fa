"""Same box: bench.host_e2e (torch imported, as in bench.py) twice, with the
cgroup's CPU throttling (cpu.stat) over each run."""
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


for thr in (16, 12, 16, 12):
    a = cpu_stat()
    r = bench.host_e2e("imix", 1, 10_000, 0x7CBEE, threads=thr)
    b = cpu_stat()
    r["cpu_stat_delta"] = {k: int(b[k]) - int(a[k]) for k in b if k in a}
    print(json.dumps(r), flush=True)
