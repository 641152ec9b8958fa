#!/usr/bin/env python3
"""E2E from host RAM, same process, interleaved: tcbee_pipe with the caller's output
arrays registered (direct D2H) or staged, by header window and host thread count.

  python tools/e2e_threads.py [--frames N] [--reps R] [--configs 64:12:reg,64:16:reg,...]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--configs", default="64:12:reg,64:16:reg,80:12:reg,80:16:reg,64:12:staged")
    args = ap.parse_args()
    import tcbee_amd
    from tcbee_amd.pipeline import Pipeline
    n = args.frames
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=10_000)
    rec = np.empty((n, 74), np.uint8)
    ids = np.empty(n, np.uint32)
    cfgs = []
    for c in args.configs.split(","):
        w, t, mode = c.split(":")
        cfgs.append((int(w), int(t), mode == "reg"))
    res = {c: [] for c in cfgs}
    for _ in range(args.rounds):
        for c in cfgs:
            w, t, reg = c
            with Pipeline(device=0, chunk_frames=1 << 20, window=w, depth=4, threads=t,
                          chunk_bytes=1 << 29, max_flows=40_000) as p:
                if reg:
                    p.register_output(rec, ids)
                p.run(tr, out_rec=rec, out_id=ids)
                for _ in range(args.reps):
                    p.reset_flows()
                    t0 = time.perf_counter()
                    p.run(tr, out_rec=rec, out_id=ids)
                    res[c].append(time.perf_counter() - t0)
    for c in cfgs:
        el = float(np.median(res[c]))
        print(f"window {c[0]} threads {c[1]} {'registered' if c[2] else 'staged'}: "
              f"{n / el / 1e6:.1f} Mpkt/s (median of {len(res[c])}, "
              f"min {n / max(res[c]) / 1e6:.1f} max {n / min(res[c]) / 1e6:.1f})", flush=True)


if __name__ == "__main__":
    main()
