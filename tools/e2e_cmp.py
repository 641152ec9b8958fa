"""Same box: bench.host_e2e (torch imported, as in bench.py) twice."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

for _ in range(2):
    print(json.dumps(bench.host_e2e("imix", 1, 10_000, 0x7CBEE)), flush=True)
