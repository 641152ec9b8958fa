"""E2E from host RAM (bench.host_e2e's calibrated 64-B-window pipe) in one process,
for A/B of two builds of libtcbee_amd.so in alternating processes
(TCBEE_AB_OPTIN=1 TCBEE_AB_LIB=... python tools/e2e_ab.py)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

r = bench.host_e2e("imix", 1, 10_000, 0x7CBEE, n=int(os.environ.get("E2E_FRAMES", "20000000")),
                   reps=int(os.environ.get("E2E_REPS", "5")))
print(json.dumps({k: v["mpkts"] for k, v in r.items() if isinstance(v, dict) and "mpkts" in v}))
