"""Config 2 (1M x 64-B frames, one flow) timed with bench.py's own run_device at
different warm-up / step counts, alternating, in one process: how much of the leg's
ms/step is the GPU clock ramping up after the previous leg's idle validation.
  python tools/c2_warm.py [--rounds R]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--idle", type=float, default=2.0, help="seconds idle before each leg")
    ap.add_argument("--legs", default="3:20,200:200,3:200,1000:1000", help="warmup:steps,...")
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    res = {}
    for r in range(args.rounds):
        for w, s in [tuple(int(x) for x in l.split(":")) for l in args.legs.split(",")]:
            time.sleep(args.idle)  # the idle gap bench.py's validation leaves
            el, k1, n, chk, _ = bench.run_device(torch, None, 0, 1, 1_000_000, "64", 0, 1, s, w,
                                                 0x7CBEE, full_check=(r == 0))
            key = f"warmup={w} steps={s}"
            res.setdefault(key, []).append((round(el / s * 1e3, 4), round(k1, 4)))
            print(key, res[key][-1], chk.get("full_bit_exact"), "host issue ms/step",
                  chk.get("host_issue_ms_per_step"), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
