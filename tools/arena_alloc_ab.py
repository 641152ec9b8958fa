#!/usr/bin/env python3
"""A/B of the frame arena's memory type: K1 time (and, under rocprofv3 --pmc,
the L2 read-request sizes) with the arena from torch (hipMalloc, coarse-grained,
cached) vs hipExtMallocWithFlags fine-grained / uncached. The header window is
40 B of each 576/1500-B frame; a cached fill costs a whole 128-B line.

  python tools/arena_alloc_ab.py [--frames N] [--kinds default,fine,uncached]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=100_000_000)
    ap.add_argument("--flows", type=int, default=10_000)
    ap.add_argument("--kinds", default="default,fine,uncached")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    import torch
    import tcbee_amd
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    hip = C.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipMemsetAsync.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]
    n, nf = args.frames, args.flows
    off, ln, ts, alen = tcbee_amd.synth_index(n, sizes="imix")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    d_ts = torch.from_numpy(ts.view(np.int64)).cuda()
    d_rec = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    d_hash = torch.empty(n, dtype=torch.int32, device="cuda")
    d_id = torch.empty(n, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    ref = None
    out = {}
    with tcbee_amd.PacketParser(max_frames=n, max_flows=max(4 * nf, 4096)) as p:
        for kind in args.kinds.split(","):
            keep = None
            if kind == "default":
                keep = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
                arena = keep.data_ptr()
            else:
                ptr = C.c_void_p()
                flag = {"fine": 0x1, "uncached": 0x3}[kind]
                rc = hip.hipExtMallocWithFlags(C.byref(ptr), alen + 64, flag)
                if rc != 0:
                    print(kind, "alloc failed", rc, flush=True)
                    continue
                arena = ptr.value
                hip.hipMemsetAsync(C.c_void_p(arena), 0, alen + 64, C.c_void_p(stream))
            tcbee_amd.gen_frames_device(arena, d_off, d_len, n, 1, nf, 0x7CBEE, stream=stream)
            torch.cuda.synchronize()

            def step():
                p.reset_flows(stream=stream, sync=False)
                p.parse_device(arena, alen, d_off, d_len, d_ts, n, d_rec, n, d_hash, d_id, d_n,
                               d_ctr, stream=stream)
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
            h = torch.sum(d_hash.to(torch.int64)).item()
            same = ref is None or h == ref
            ref = h if ref is None else ref
            out[kind] = {"step_ms": round(el * 1e3, 4), "k1_ms": round(ms / max(k, 1), 4),
                         "same_output": bool(same)}
            print(kind, out[kind], flush=True)
            if keep is None:
                hip.hipFree(C.c_void_p(arena))
            del keep
            torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
