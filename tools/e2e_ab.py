#!/usr/bin/env python3
"""E2E (host RAM -> GPU -> host RAM) pipeline rate of the tcbee_amd package under
ROOT (argv[1]); header-window 80 and whole-frame staging, 20M IMIX frames."""
import os
import sys
import time

import numpy as np

root = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else ".")
sys.path.insert(0, root)
import tcbee_amd  # noqa: E402
from tcbee_amd.pipeline import Pipeline  # noqa: E402

n = 20_000_000
tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=10_000)
rec = np.empty((n, 74), np.uint8)
ids = np.empty(n, np.uint32)
pfs = [v for v in os.environ.get("PF_LIST", "").split(",") if v]
nts = [v for v in os.environ.get("NT_LIST", "").split(",") if v]
runs = ([(80, v, None) for v in pfs] + [(80, None, v) for v in nts]) or [(80, None, None),
                                                                       (0, None, None)]
for window, pf, nt in runs:
    if pf is not None:
        os.environ["TCBEE_PIPE_PF"] = pf
    if nt is not None:
        os.environ["TCBEE_PIPE_NT"] = nt
    with Pipeline(device=0, chunk_frames=1 << 20, window=window, depth=4, threads=16,
                  chunk_bytes=(1 << 29), max_flows=40_000) as p:
        p.run(tr, out_rec=rec, out_id=ids)
        ts = []
        for _ in range(5):
            p.reset_flows()
            t0 = time.perf_counter()
            p.run(tr, out_rec=rec, out_id=ids)
            ts.append(time.perf_counter() - t0)
    print(root, "window", window, "pf", pf, "nt", nt, "Mpkt/s", round(n / float(np.median(ts)) / 1e6, 1), flush=True)
