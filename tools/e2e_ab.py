#!/usr/bin/env python3
"""A/B of the host-RAM end-to-end pipeline (tcbee_pipe) settings on one trace:
header window bytes, staging depth, chunk size, gather threads."""
import argparse
import json
import os
# TCBEE_* variants / ablations are dispatched by the variants build only
os.environ.setdefault("TCBEE_AB_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tcbee_amd", "lib", "libtcbee_amd_variants.so"))
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20_000_000)
    ap.add_argument("--variants", default="80:4:20:16,64:4:20:16,80:4:21:16,80:6:20:16,80:4:20:12")
    ap.add_argument("--reps", type=int, default=9)
    args = ap.parse_args()
    import tcbee_amd
    from tcbee_amd.pipeline import Pipeline
    n = args.frames
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=10_000, seed=0x7CBEE)
    rec = np.empty((n, 74), np.uint8)
    ids = np.empty(n, np.uint32)
    res = {}
    pipes = {}
    for v in args.variants.split(","):
        f = [int(x) for x in v.split(":")]
        w, depth, cbits, thr = f[:4]
        if len(f) > 4:  # copy-out threads (TCBEE_PIPE_CTHREADS, read at create)
            os.environ["TCBEE_PIPE_CTHREADS"] = str(f[4])
        else:
            os.environ.pop("TCBEE_PIPE_CTHREADS", None)
        pipes[v] = Pipeline(device=0, chunk_frames=1 << cbits, window=w, depth=depth, threads=thr,
                            chunk_bytes=(1 << 29), max_flows=40_000)
        pipes[v].run(tr, out_rec=rec, out_id=ids)  # warm-up
    ts = {v: [] for v in pipes}
    for _ in range(args.reps):  # interleaved: box drift hits every variant alike
        for v, p in pipes.items():
            p.reset_flows()
            t0 = time.perf_counter()
            r = p.run(tr, out_rec=rec, out_id=ids)
            ts[v].append(time.perf_counter() - t0)
            assert r.n == n
    for v, p in pipes.items():
        el = float(np.median(ts[v]))
        res[v] = {"mpkts": round(n / el / 1e6, 1),
                  "min_max": [round(n / max(ts[v]) / 1e6, 1), round(n / min(ts[v]) / 1e6, 1)]}
        print(v, res[v], flush=True)
        p.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
