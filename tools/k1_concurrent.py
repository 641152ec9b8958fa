"""K1 beside other kernels in ONE process: two parser contexts on two streams
parsing the same device-resident trace at once, against one context alone.

  python tools/k1_concurrent.py [--frames 10000000] [--iters 20] [--pairs 3]

K1's decoupled look-back assumes nothing about dispatch order, but it polls a
predecessor's status word before recounting it; when another kernel holds part of
the chip (a second stream, another process, a collective), some XCDs fall behind
and their successors wait on them. This prints, per round, the wall time of
`iters` batches on one stream and of `iters` batches on each of two streams at
once (2x the frames), and checks both contexts' outputs against the solo run.
TCBEE_AB_LIB selects another build of libtcbee_amd.so (tools/lib_ab.sh).
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
    ap.add_argument("--frames", type=int, default=10_000_000)
    ap.add_argument("--flows", type=int, default=10_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pairs", type=int, default=3)
    a = ap.parse_args()
    import torch
    import tcbee_amd
    from bench import build_device_trace
    torch.cuda.set_device(0)
    n = a.frames
    s0 = torch.cuda.Stream()
    arena, alen, off, ln, ts = build_device_trace(torch, n, "imix", 1, a.flows, 0x7CBEE, 0,
                                                  s0.cuda_stream)
    streams = [s0, torch.cuda.Stream()]
    ctxs, outs = [], []
    for _ in range(2):
        ctxs.append(tcbee_amd.PacketParser(max_frames=n, max_flows=a.flows + a.flows // 32 + 64))
        outs.append({"rec": torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda"),
                     "id": torch.empty(n, dtype=torch.int32, device="cuda"),
                     "n": torch.zeros(1, dtype=torch.int64, device="cuda"),
                     "ctr": torch.zeros(4, dtype=torch.int64, device="cuda")})

    def launch(k):
        o, s = outs[k], streams[k].cuda_stream
        with torch.cuda.stream(streams[k]):
            o["ctr"].zero_()  # the counters accumulate across calls
        ctxs[k].reset_flows(stream=s, sync=False)
        ctxs[k].parse_device(arena, alen, off, ln, ts, n, o["rec"], n, None, o["id"], o["n"],
                             o["ctr"], stream=s)

    def timed(both):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            launch(0)
            if both:
                launch(1)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.iters * 1e3

    timed(True)
    rows = []
    for _ in range(a.pairs):
        rows.append((timed(False), timed(True)))
    solo = float(np.median([r[0] for r in rows]))
    conc = float(np.median([r[1] for r in rows]))
    # outputs: both contexts of a concurrent pair vs context 0 run alone
    launch(0)
    torch.cuda.synchronize()
    ref = {k: v.clone() for k, v in outs[0].items()}
    torch.cuda.synchronize()  # the clones (current stream) before the next zeroing
    launch(0)
    launch(1)
    torch.cuda.synchronize()
    diffs = []
    for c in range(2):
        for k in ("n", "ctr", "id", "rec"):
            x, y = outs[c][k], ref[k]
            if k == "rec":
                m = int(ref["n"].item()) * 74
                x, y = x[:m], y[:m]
            if not torch.equal(x, y):
                bad = int((x != y).sum().item())
                diffs.append(f"ctx{c}.{k}: {bad} elements differ"
                             + (f" ({x.tolist()} vs {y.tolist()})" if k in ("n", "ctr") else ""))
        st = ctxs[c].status()
        if st:
            diffs.append(f"ctx{c} status {st}")
    same = not diffs
    print(f"lib {os.environ.get('TCBEE_AB_LIB', 'tree')}: one stream {solo:.3f} ms/batch, "
          f"two streams {conc:.3f} ms per pair of batches ({conc / solo:.2f}x the solo batch; "
          f"2.00x = the chip shared perfectly); outputs identical: {same} {diffs}; rounds "
          + " ".join(f"{x:.3f}/{y:.3f}" for x, y in rows), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
