#!/usr/bin/env python3
"""Cost of the N>1 per-step flow-table merge, simulated on ONE GPU: one rank's
exported table stands in for all `world` segments (what the RCCL all-gather
delivers), then merge_device + the local->global id remap over the rank's
records — the device work a rank does per step besides the collectives.

  python tools/merge_bench.py [--world 8] [--frames 100000000] [--flows 10000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--frames", type=int, default=100_000_000)
    ap.add_argument("--flows", type=int, default=10_000)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    import tcbee_amd
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())  # non-NULL: NULL means "the ctx's stream"
    stream = torch.cuda.current_stream().cuda_stream
    n, nf, world = args.frames, args.flows, args.world
    off, ln, ts, alen = tcbee_amd.synth_index(n, sizes="imix")
    d_arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    d_ts = torch.from_numpy(ts.view(np.int64)).cuda()
    tcbee_amd.gen_frames_device(d_arena, d_off, d_len, n, 1, nf, 0x7CBEE, stream=stream)
    d_rec = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    d_hash = torch.empty(n, dtype=torch.int32, device="cuda")
    d_id = torch.empty(n, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    cap = max(4 * nf, 1 << 12)
    out = {}
    with tcbee_amd.PacketParser(max_frames=n, max_flows=cap) as p, \
            tcbee_amd.PacketParser(max_frames=1024, max_flows=world * cap) as m:
        p.parse_device(d_arena, alen, d_off, d_len, d_ts, n, d_rec, n, d_hash, d_id, d_n, d_ctr,
                       stream=stream)
        ent = torch.zeros((cap, 8), dtype=torch.int64, device="cuda")
        meta = torch.zeros(2, dtype=torch.int64, device="cuda")
        p.export_device(ent, cap, meta, stream=stream)
        torch.cuda.synchronize()
        nflows = int(meta[0].item())
        for name, stride in (("stride_cap", cap), ("stride_flows", nflows)):
            all_ent = ent[:stride].repeat(world, 1).contiguous()
            all_meta = meta.repeat(world).contiguous()
            ids = torch.empty(world * stride, dtype=torch.int32, device="cuda")
            def once():
                m.merge_device(all_ent, world, stride, all_meta, world * n, ids, stream=stream)
                tcbee_amd.parser.remap_ids_device(d_id, n, d_n, ids[:stride], stride, stream=stream)
            once()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                once()
            torch.cuda.synchronize()
            t_all = (time.perf_counter() - t0) / args.iters
            t0 = time.perf_counter()
            for _ in range(args.iters):
                m.merge_device(all_ent, world, stride, all_meta, world * n, ids, stream=stream)
            torch.cuda.synchronize()
            t_merge = (time.perf_counter() - t0) / args.iters
            out[name] = {"stride": stride, "merge_ms": round(t_merge * 1e3, 4),
                         "merge_remap_ms": round(t_all * 1e3, 4)}
            print(name, out[name], flush=True)
    print(json.dumps({"world": world, "frames": n, "flows": nf, **out}))


if __name__ == "__main__":
    main()
