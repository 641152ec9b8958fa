#!/usr/bin/env python3
"""Eager launches vs one hipGraph per step (captured through torch.cuda.CUDAGraph):
ms per step of the device-resident path for config 2 (1M x 64 B, launch-bound)
and config 3 (100M IMIX, 10k flows)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import tcbee_amd
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    out = {}
    for name, n, sizes, kind, nf, iters in (("config2", 1_000_000, "64", 0, 1, 200),
                                            ("config3", 100_000_000, "imix", 1, 10_000, 20)):
        s = torch.cuda.current_stream().cuda_stream
        off, ln, ts, alen = tcbee_amd.synth_index(n, sizes=sizes)
        arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(off.view(np.int64)).cuda()
        d_len = torch.from_numpy(ln.view(np.int32)).cuda()
        d_ts = torch.from_numpy(ts.view(np.int64)).cuda()
        tcbee_amd.gen_frames_device(arena, d_off, d_len, n, kind, nf, 0x7CBEE, stream=s)
        rec = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
        hsh = torch.empty(n, dtype=torch.int32, device="cuda")
        ids = torch.empty(n, dtype=torch.int32, device="cuda")
        nd = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
        with tcbee_amd.PacketParser(max_frames=n, max_flows=max(4 * nf, 4096)) as p:
            def step():
                cs = torch.cuda.current_stream().cuda_stream
                p.reset_flows(stream=cs, sync=False)
                p.parse_device(arena, alen, d_off, d_len, d_ts, n, rec, n, hsh, ids, nd, ctr,
                               stream=cs)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                step()
            torch.cuda.synchronize()
            eager = (time.perf_counter() - t0) / iters * 1e3
            ref = rec[:n * 74].clone()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            rec.zero_()
            t0 = time.perf_counter()
            for _ in range(iters):
                g.replay()
            torch.cuda.synchronize()
            graph = (time.perf_counter() - t0) / iters * 1e3
            same = bool(torch.equal(rec[:n * 74], ref)) and int(nd.item()) == n
            out[name] = {"eager_ms": round(eager, 4), "graph_ms": round(graph, 4),
                         "same_output": same}
            print(name, out[name], flush=True)
            del g
        del arena, rec
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
