#!/usr/bin/env python3
"""A/B sweep of the parse path in ONE process (interleaved rounds): K1 time and
whole-step time per variant (frames-per-lane tiling, flows on/off) per workload.

  python tools/k1_sweep.py [--frames N] [--rounds R] [--iters I]
"""
import argparse
import itertools
import json
import os
# TCBEE_* variants / ablations are dispatched by the variants build only
os.environ.setdefault("TCBEE_AB_OPTIN", "1")
os.environ.setdefault("TCBEE_AB_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tcbee_amd", "lib", "libtcbee_amd_variants.so"))
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fpl", default="1,2,4")
    ap.add_argument("--workloads", default="imix10k,imix1,64B1")
    ap.add_argument("--var", default="", help="extra env A/B of a variants-build test hook, e.g. TCBEE_TEST_K3_WIDE=0,1")
    ap.add_argument("--flows-only", action="store_true", help="only the flows-on variants")
    ap.add_argument("--cap-mult", default="4", help="max_flows = mult x flows (comma list: A/B)")
    ap.add_argument("--warm", action="store_true", help="keep the flow table across steps (no reset)")
    ap.add_argument("--min-table", type=int, default=4096, help="max_flows floor (bench.py: 64)")
    args = ap.parse_args()
    import torch
    import tcbee_amd
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())  # non-NULL: NULL means "the ctx's stream"
    stream = torch.cuda.current_stream().cuda_stream
    wl_defs = {"imix10k": ("imix", 1, 10_000), "imix1": ("imix", 0, 1), "64B1": ("64", 0, 1),
               "imix1M": ("imix", 1, 1_000_000), "64B10k": ("64", 1, 10_000),
               "imix125k": ("imix", 1, 125_000), "imix20k": ("imix", 1, 20_000),
               "imix30k": ("imix", 1, 30_000), "imix45k": ("imix", 1, 45_000),
               "imix60k": ("imix", 1, 60_000), "imix6v6": ("imix6", 3, 10_000)}
    results = {}
    for wl in args.workloads.split(","):
        sizes, kind, nf = wl_defs[wl]
        n = args.frames
        off, ln, ts, alen = tcbee_amd.synth_index(n, sizes=sizes)
        d_arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(off.view(np.int64)).cuda()
        d_len = torch.from_numpy(ln.view(np.int32)).cuda()
        d_ts = torch.from_numpy(ts.view(np.int64)).cuda()
        tcbee_amd.gen_frames_device(d_arena, d_off, d_len, n, kind, nf, 0x7CBEE, stream=stream)
        d_rec = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
        d_hash = torch.empty(n, dtype=torch.int32, device="cuda")
        d_id = torch.empty(n, dtype=torch.int32, device="cuda")
        d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
        d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
        var_name, _, var_vals = args.var.partition("=")
        vvals = var_vals.split(",") if var_name else [""]
        variants = list(itertools.product(args.fpl.split(","),
                                          [True] if args.flows_only else [True, False], vvals,
                                          [float(x) for x in args.cap_mult.split(",")]))
        parsers = {}
        for fpl, flows, vv, cm in variants:
            os.environ["TCBEE_FPL"] = fpl
            if var_name:
                os.environ[var_name] = vv
            parsers[(fpl, flows, vv, cm)] = tcbee_amd.PacketParser(
                max_frames=n, max_flows=max(int(cm * nf), args.min_table))
        times = {v: [] for v in variants}
        k1 = {v: [] for v in variants}
        for r in range(args.rounds):
            for v in variants:
                p = parsers[v]
                if var_name:  # (set again per variant: a hook read at launch sees its own value)
                    os.environ[var_name] = v[2]
                def step():
                    if not args.warm:
                        p.reset_flows(stream=stream, sync=False)  # one fresh trace per step, as bench.py
                    p.parse_device(d_arena, alen, d_off, d_len, d_ts, n, d_rec, n,
                                   d_hash if v[1] else None, d_id if v[1] else None, d_n, d_ctr,
                                   flows=v[1], stream=stream)
                step()
                torch.cuda.synchronize()
                p.profile(True)
                t0 = time.perf_counter()
                for _ in range(args.iters):
                    step()
                torch.cuda.synchronize()
                el = (time.perf_counter() - t0) / args.iters
                ms, k = p.profile_read()
                p.profile(False)
                times[v].append(el * 1e3)
                k1[v].append(ms / max(k, 1))
        for v in variants:
            key = (f"{wl} fpl={v[0]} flows={int(v[1])}" + (f" {var_name}={v[2]}" if var_name else "")
                   + (f" cap={v[3]:g}x" if "," in args.cap_mult else ""))
            step_ms = float(np.median(times[v]))
            k1_ms = float(np.median(k1[v]))
            results[key] = {"step_ms": round(step_ms, 4), "k1_ms": round(k1_ms, 4),
                            "mpkts": round(n / step_ms / 1e3, 1),
                            "k1_alg_GBs": round(n * 156 / k1_ms / 1e6, 1)}
            print(key, results[key], flush=True)
        for p in parsers.values():
            p.close()
        del d_arena, d_rec, d_off, d_len, d_ts, d_hash, d_id
        torch.cuda.empty_cache()
    print(json.dumps(results))


if __name__ == "__main__":
    main()
