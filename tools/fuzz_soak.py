"""Soak of the random-frame fuzz (tests/test_gpu_parity.py::_fuzz_trace) over many
seeds: random caplens around every accept boundary, random ethertypes/protocols,
keys from pools of 0 (a distinct key per frame) / 40 / 3000 / 60000, FILTER_PORT on
every other seed; each trace through one batch and through three batches of a kept
table, everything bit-exact vs the oracle. Prints one line per seed and a summary;
exits 1 on the first mismatch.

  python tools/fuzz_soak.py [--seeds 60] [--seed0 1000] [--frames 300000]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def same(res, orc, flows=None, table=None):
    rec, fh, fi, ctr, _ = orc
    ok = res.n == len(rec) and res.counters == ctr
    ok = ok and (len(rec) == 0 or np.array_equal(res.records, rec))
    ok = ok and np.array_equal(res.flow_hash, fh) and np.array_equal(res.flow_id, fi)
    if flows is not None:
        ok = ok and np.array_equal(flows, table)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=60)
    ap.add_argument("--seed0", type=int, default=1000, help="first seed")
    ap.add_argument("--frames", type=int, default=300_000)
    a = ap.parse_args()
    import tcbee_amd
    from oracle_py import Oracle
    from test_gpu_parity import _fuzz_trace
    oracle = Oracle()
    pools = [0, 40, 3000, 60_000]
    t0 = time.time()
    frames = 0
    for seed in range(a.seed0, a.seed0 + a.seeds):
        pool = pools[seed % len(pools)]
        port = 4242 if seed % 2 else 0
        n = a.frames
        tr = _fuzz_trace(seed, n, pool, port)
        orc = oracle.parse(tr, filter_port=port)
        cap = 256 if pool == 40 else max(len(orc[4]), 16) + 64
        with tcbee_amd.PacketParser(max_frames=n, max_arena=len(tr.arena), max_flows=cap) as p:
            ok = same(p.parse(tr, filter_port=port), orc, p.flows(), orc[4]) and p.status() == 0
            p.reset_flows()
            ft = oracle.new_flowtab(1 << 20)
            base = 0
            try:
                cuts = sorted({0, n, *np.random.default_rng(seed).integers(1, n, 2).tolist()})
                for lo, hi in zip(cuts[:-1], cuts[1:]):
                    part = tr.select(np.arange(lo, hi))
                    o = oracle.parse(part, ft=ft, record_base=base, filter_port=port)
                    ok = ok and same(p.parse(part, filter_port=port), o)
                    base += len(o[0])
                ok = ok and np.array_equal(p.flows(), oracle.flows(ft)) and p.status() == 0
            finally:
                oracle.free_flowtab(ft)
        frames += 2 * n
        print(f"seed {seed} pool {pool} port {port}: {len(orc[0])} records, "
              f"{len(orc[4])} flows, cuts {cuts[1:-1]}: {'ok' if ok else 'MISMATCH'}", flush=True)
        if not ok:
            sys.exit(1)
    print(f"fuzz soak: {a.seeds} seeds, {frames} frames parsed, all bit-exact "
          f"({time.time() - t0:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
