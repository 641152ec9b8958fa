#!/usr/bin/env python3
"""Zero-copy A/B for the end-to-end path: K1-K3 reading frames (and optionally the
index, and writing the outputs) straight from/to pinned host memory over PCIe,
instead of staging header windows through H2D copies (tcbee_pipe).

  python tools/zerocopy_ab.py [--frames 20000000] [--reps 5]

Legs (IMIX, 10k flows; time = one tcbee_parse_batch_device + sync):
  dev        everything in HBM (the device-resident reference point)
  arena      arena pinned on the host, index + outputs in HBM
  arena_idx  arena + index pinned on the host, outputs in HBM
  all_host   arena, index and outputs (records, hashes, ids) pinned on the host
Each leg's records/ids are compared with the dev leg's.
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
    ap.add_argument("--frames", type=int, default=20_000_000)
    ap.add_argument("--flows", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import tcbee_amd
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    n = args.frames
    t0 = time.perf_counter()
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=args.flows)
    print(f"trace {n} frames, {len(tr.arena) / 1e9:.2f} GB in {time.perf_counter() - t0:.1f}s",
          flush=True)

    def host(a):
        t = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = a.view(np.uint8).reshape(-1)
        return t

    t0 = time.perf_counter()
    h_arena = host(tr.arena)
    h_off, h_len, h_ts = host(tr.offset), host(tr.caplen), host(tr.ts_ns)
    print(f"pinned copies in {time.perf_counter() - t0:.1f}s", flush=True)
    d_arena = h_arena.cuda()
    d_off, d_len, d_ts = h_off.cuda(), h_len.cuda(), h_ts.cuda()

    def outs(on_host):
        kw = dict(dtype=torch.uint8, pin_memory=True) if on_host else dict(dtype=torch.uint8,
                                                                           device="cuda")
        return (torch.empty(n * 74 + 64, **kw), torch.empty(n * 4, **kw),
                torch.empty(n * 4, **kw), torch.zeros(8, **kw))

    d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    legs = {"dev": (d_arena, (d_off, d_len, d_ts), False),
            "arena": (h_arena, (d_off, d_len, d_ts), False),
            "arena_idx": (h_arena, (h_off, h_len, h_ts), False),
            "all_host": (h_arena, (h_off, h_len, h_ts), True)}
    res, ref = {}, None
    with tcbee_amd.PacketParser(max_frames=n, max_arena=0, max_flows=4 * args.flows) as p:
        for name, (arena, idx, oh) in legs.items():
            rec, hs, ids, nn = outs(oh)
            ts = []
            for _ in range(args.reps + 1):
                p.reset_flows(stream=stream, sync=False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                p.parse_device(arena, len(tr.arena), idx[0], idx[1], idx[2], n, rec, n, hs, ids,
                               nn, d_ctr, stream=stream)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            el = float(np.median(ts[1:]))
            r = rec[: n * 74].cpu().numpy()
            i = ids.cpu().numpy()
            if ref is None:
                ref = (r.copy(), i.copy())
            same = bool(np.array_equal(r, ref[0]) and np.array_equal(i, ref[1]))
            res[name] = {"ms": round(el * 1e3, 2), "mpkts": round(n / el / 1e6, 1),
                         "same_as_dev": same}
            print(name, res[name], flush=True)
            del rec, hs, ids, nn
    print(json.dumps({"frames": n, "arena_GB": round(len(tr.arena) / 1e9, 2), **res}))


if __name__ == "__main__":
    main()
