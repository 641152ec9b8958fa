#!/usr/bin/env python3
"""Benchmark of the device-resident packet-record path (BASELINE.json metric).

Workload (config 3 of BASELINE.json, the largest single-GPU config): per GPU,
100M synthetic IPv4/TCP frames, IMIX 64/576/1500 B at 7:4:1 (35.4 GB arena),
10k flows, all resident in HBM before the timed region. A step = one
``tcbee_parse_batch_device`` over the whole batch: parse + 74-B records +
flow hash + flow classification (table upsert, dense first-seen ids) +
counters. Each step is one fresh trace (the flow table starts empty). With
--gpus N (weak scaling, no frame exchange) each rank parses its flow-hash shard
of one global trace of N x --frames frames (north_star's partition, the NIC-RSS
view): between K2 and K3 one RCCL all-gather of every rank's first-frame array
gives the global dense first-seen ids, which K3 writes directly
(tcbee_amd.dist.FlowHashExchange); the counters are all-reduced; the timed region
ends after all of it. --shard contig: contiguous shards, each flow merged at its
hash owner (OwnerExchange; TCBEE_BENCH_EXCHANGE=merge: the all-gather merge
overlapped with the next parse, OverlappedMerge).

Prints ONE JSON line (rank 0). See DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkt/s device-resident TCP header parse+flow-classify, 64–1500B frames"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
IDX_BYTES = 8 + 4 + 8          # offset u64 + caplen u32 + ts_ns u64 read per frame
V4_HDR_BYTES = 54              # eth + ipv4 + tcp header bytes the hook reads
OUT_BYTES = 74 + 4 + 4         # record + flow hash + flow id (slot) written per record


_T0 = time.perf_counter()


def log(*a):
    """Progress on stderr (the JSON line alone goes to stdout): every leg and every
    long check reports, so a multi-minute default run is never silent."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s]", *a, file=sys.stderr, flush=True)


def build_device_trace(torch, n, sizes, kind, n_flows, seed, first_index, stream):
    """Synthetic trace straight into HBM: index on the host (numpy), headers by the
    device generator (bit-identical to the host generator)."""
    import tcbee_amd
    off, ln, ts, alen = tcbee_amd.synth_index(n, sizes=sizes, seed=seed, first_index=first_index)
    d_arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    d_ts = torch.from_numpy(ts.view(np.int64)).cuda()
    tcbee_amd.gen_frames_device(d_arena, d_off, d_len, n, kind, n_flows, seed, stream=stream,
                                first_index=first_index)
    torch.cuda.synchronize()
    return d_arena, alen, d_off, d_len, d_ts


RSS_WINDOW = 16_000_000  # frames of observed traffic an RSS table is balanced on


RSS_SKEW_LIMIT = 1.25  # max / mean flows per rank a flow-hash run accepts (before timing)


def rss_for(torch, n_global, world, kind, n_flows, seed, stream):
    """The NIC's RSS indirection table (4096 hash buckets -> GPUs) balanced on the
    bucket loads of RSS_WINDOW frames of the same synthetic stream OUTSIDE the
    measured trace (global frames [n_global, n_global + RSS_WINDOW): held out, as
    receive-side scaling is rebalanced from earlier load — ADVICE r3: balancing on
    the measured frames made the imbalance in-sample), via
    tcbee_gen_rss_load_range_device and tcbee_amd.rss_table; the same table on every
    rank. Every flow still lands on one GPU. Returns the table on the device (None:
    the modulo placement fold32(hash) % world; TCBEE_BENCH_RSS=0), what the line
    reports, and the flows each rank will hold (tcbee_amd.rss_flows_per_rank: the
    flows routed to it, known before any frame is parsed), from which the table and
    exchange capacities are sized. A partition whose busiest rank holds more than
    RSS_SKEW_LIMIT x the mean flows is refused HERE, before anything is timed, on
    every rank alike (the same table everywhere: no rank waits in a collective).
    TCBEE_BENCH_RSS=skew (test hook): every bucket but one on rank 0."""
    import tcbee_amd
    mode = os.environ.get("TCBEE_BENCH_RSS", "1")
    table = None
    info = {"rss": None}
    if world >= 2 and mode == "skew":
        table = np.zeros(tcbee_amd.RSS_BUCKETS, dtype=np.uint16)
        table[1:world] = np.arange(1, world, dtype=np.uint16)
        info = {"rss": {"buckets": len(table), "skewed_test_table": True}}
    elif world >= 2 and mode != "0":
        win = RSS_WINDOW
        counts = torch.empty(tcbee_amd.RSS_BUCKETS, dtype=torch.int64, device="cuda")
        tcbee_amd.gen_rss_load_device(win, kind, n_flows, seed, counts, stream=stream,
                                      first_frame=n_global)
        load = counts.cpu().numpy()
        table = tcbee_amd.rss_table(load, world)
        per = np.bincount(table, weights=load, minlength=world)
        info = {"rss": {"buckets": len(table), "balanced_on_frames": [n_global, n_global + win],
                        "held_out": True,
                        "window_imbalance": round(float(per.max() / per.mean()), 5)}}
        if len(table) % world == 0:  # the modulo placement on the same window, for reference
            mod = np.bincount(np.arange(len(table)) % world, weights=load, minlength=world)
            info["rss"]["window_imbalance_modulo"] = round(float(mod.max() / mod.mean()), 5)
    # (the multi-flow IPv4 kind: each flow's key from its number; any other kind is
    #  bounded by its flow count on every rank)
    flows_per_rank = (tcbee_amd.rss_flows_per_rank(n_flows, world, seed, table)
                      if kind == 1 else np.full(world, n_flows, np.int64))
    skew = float(flows_per_rank.max() / max(flows_per_rank.mean(), 1e-9))
    if world >= 2 and kind == 1:
        info["flows_per_rank"] = [int(flows_per_rank.min()), int(flows_per_rank.max())]
        info["flows_imbalance"] = round(skew, 4)  # max / mean flows per rank
        if skew > RSS_SKEW_LIMIT:
            raise RuntimeError(
                f"flow-hash partition refused before the timed region: its busiest rank "
                f"holds {int(flows_per_rank.max())} of {n_flows} flows, {skew:.2f}x the mean "
                f"(limit {RSS_SKEW_LIMIT}); rebalance the RSS table")
    dev = torch.from_numpy(table.view(np.int16)).cuda() if table is not None else None
    return dev, info, flows_per_rank


def build_shard_trace(torch, n_global, world, rank, sizes, kind, n_flows, seed, stream,
                      rss=None):
    """This rank's flow-hash shard of the global synthetic trace [0, n_global) (the
    NIC-RSS view of config 4), built on the device: global indices + caplens
    (tcbee_gen_shard_index_device; with an RSS table, _rss_device), offsets by a
    prefix sum, headers by the device generator at each frame's global index."""
    import tcbee_amd
    scratch = torch.empty(tcbee_amd.gen_shard_scratch_words(n_global), dtype=torch.int64,
                          device="cuda")
    n_out = torch.zeros(1, dtype=torch.int64, device="cuda")
    # count pass first (cap 0: nothing written), then the exact buffers: a shard's
    # size is (its flows / all flows) x n_global, and with 10k flows over 8 ranks the
    # flows per rank spread by ~3 % (1210..1287 at the default seed), far more than
    # the sampling noise of the frame draw
    tcbee_amd.gen_shard_index_device(n_global, world, rank, kind, n_flows, seed,
                                     sizes == "imix", None, None, 0, scratch, n_out,
                                     stream=stream, rss=rss)
    cap = int(n_out.item())
    if cap < 0:  # TCBEE_RSS_INVALID: the device found a table entry >= world
        raise RuntimeError("RSS table refused by the device (an entry >= world)")
    gidx = torch.empty(max(cap, 1), dtype=torch.int64, device="cuda")
    clen = torch.empty(max(cap, 1), dtype=torch.int32, device="cuda")
    tcbee_amd.gen_shard_index_device(n_global, world, rank, kind, n_flows, seed,
                                     sizes == "imix", gidx, clen, cap, scratch, n_out,
                                     stream=stream, rss=rss)
    m = int(n_out.item())
    if m != cap:
        raise RuntimeError(f"shard of {m} frames, counted {cap}")
    gidx, clen = gidx[:m], clen[:m]
    off = torch.zeros(m, dtype=torch.int64, device="cuda")
    if m > 1:
        torch.cumsum(clen[:-1].to(torch.int64), 0, out=off[1:])
    alen = int(off[-1].item() + clen[-1].item()) if m else 0
    ts = gidx * 1000 + 1_000_000_000  # TS_BASE_NS + TS_STEP_NS * global index
    arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
    tcbee_amd.gen_frames_index_device(arena, off, clen, gidx, m, kind, n_flows, seed,
                                      stream=stream)
    torch.cuda.synchronize()
    del scratch
    return arena, alen, off, clen, ts, gidx, m


def run_device(torch, dist, rank, world, n, sizes, kind, n_flows, steps, warmup, seed,
               multi=None, full_check=False, flowhash=False, vworld=0, warm=False):
    import tcbee_amd
    stream = torch.cuda.current_stream().cuda_stream
    log(f"rank {rank}: building {n} frames ({sizes}, {n_flows} flows, "
        f"{'flow-hash' if flowhash else 'contiguous'} shard)")
    # multi: the N>1 exchange runs (also at N=1 under TCBEE_BENCH_FORCE_MERGE=1, a
    # one-GPU rehearsal of its cost and of the overlap)
    multi = world > 1 if multi is None else multi
    first = rank * n
    # vworld (N=1 only): emulate rank 0 of a vworld-GPU flow-hash run (its shard and
    # its share of the flows), without the exchange
    sw = vworld if (flowhash and vworld and world == 1) else world
    n_global = n * sw
    gidx = None
    if flowhash:
        # n frames per GPU on average: rank `rank` parses the frames of ITS flows out of
        # a global trace of n * world frames (sizes differ by a few hundred)
        rss, rss_info, flows_per_rank = rss_for(torch, n_global, sw, kind, n_flows, seed, stream)
        d_arena, alen, d_off, d_len, d_ts, gidx, n = build_shard_trace(
            torch, n_global, sw, rank, sizes, kind, n_flows, seed, stream, rss=rss)
        first = 0
    else:
        d_arena, alen, d_off, d_len, d_ts = build_device_trace(torch, n, sizes, kind, n_flows,
                                                               seed, first, stream)
    # N>1, flow-hash shards: disjoint tables, the global-id exchange runs between K2
    # and K3 (FlowHashExchange; TCBEE_BENCH_EXCHANGE=merge: the general table merge)
    exch = os.environ.get("TCBEE_BENCH_EXCHANGE", "auto")
    fhx = multi and flowhash and exch in ("auto", "fhx")
    # N>1 contiguous shards: each flow merged at its hash owner (OwnerExchange, between
    # K2 and K3) instead of every rank merging every table (TCBEE_BENCH_EXCHANGE=merge:
    # the all-gather merge, overlapped on a side stream). World-1 rehearsal, config 4
    # contiguous (1M flows): 10.54 ms/step owner vs 11.00 merge (whose side stream
    # slows the next K1 7.46 -> 8.78 ms); at N=8 an owner merges 1/8 of the entries
    ownx = multi and not flowhash and exch in ("auto", "owner")
    # N>1 contiguous shards (every rank sees every flow): the table merge; two output
    # slots, so that step i's exchange (side stream) overlaps step i+1's parse
    overlap = (multi and not fhx and not ownx
               and os.environ.get("TCBEE_BENCH_OVERLAP", "1") != "0")
    nbuf = 2 if overlap else 1
    # TCBEE_BENCH_ASYNC=1: K3 (ids, pkts/bytes, counters) of step i on a side stream
    # beside step i+1's K1 (TCBEE_EX_ASYNC_IDS). Off by default: measured slower
    # (config 3 4.52 -> 4.65 ms/step, config-4 share 7.39 -> 7.66): K3's 1024-thread,
    # 144 KiB-LDS workgroups take whole CUs from the HBM-bound K1
    ids_side = (torch.cuda.Stream() if os.environ.get("TCBEE_BENCH_ASYNC", "0") == "1"
                and (not multi or fhx) else None)
    ids_stream = ids_side.cuda_stream if ids_side is not None else None
    slots = [{"rec": torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda"),
              "hash": torch.empty(n, dtype=torch.int32, device="cuda"),
              "id": torch.empty(n, dtype=torch.int32, device="cuda"),
              "n": torch.zeros(1, dtype=torch.int64, device="cuda"),
              "ctr": torch.zeros(4, dtype=torch.int64, device="cuda")} for _ in range(nbuf)]
    # flow-hash shards: the flows routed to each rank are known before any frame is
    # parsed (rss_for); the exchange carries `xcap` entries per rank, sized for the
    # busiest rank (every rank's all-gather block has the same size)
    flows_here = int(flows_per_rank[rank]) if flowhash else n_flows
    # table: max_flows = the shard's expected flows + 3 % + 64 (a flow-hash shard of
    # config 3 at N=8 holds up to +3 % of the mean; claims past max_flows are
    # refused). The compact table (round 3) keeps 8 slots per max_flow (load <=
    # 1/8), 6 slots per 128-B line: 176 MB at 1M flows (rounds 1-2: 64-B slots at
    # max_flows = 4x flows, 512 MiB), and a tight max_flows keeps the K1 -> K3 word
    # packed (claim | caplen) up to 2^20 flows
    # (flow-hash shards: flows_here is exact, an upper bound the shard reaches once
    # every one of its flows has appeared; 1M flows stay below 2^20 = packed K1 -> K3
    # words)
    cap = max(flows_here + flows_here // 32 + 64, 64)
    # (the exchange carries up to xcap entries per rank: the busiest rank's flows, or a
    # quarter more than a contiguous shard's)
    xcap = (int(flows_per_rank.max()) + 64 if flowhash
            else max(int(1.25 * flows_here) + 4096, 1 << 12))
    p = tcbee_amd.PacketParser(device=torch.cuda.current_device(), max_frames=n, max_arena=0,
                               max_flows=cap)
    merged = om = fm = fx = ox = None
    if ownx:
        from tcbee_amd.dist import OwnerExchange
        merged = tcbee_amd.PacketParser(device=torch.cuda.current_device(), max_frames=1024,
                                        max_arena=0, max_flows=world * xcap)
        ocap = int(1.25 * n_flows / world) + 4096  # flows one owner merges
        owner_ctx = tcbee_amd.PacketParser(device=torch.cuda.current_device(), max_frames=1024,
                                           max_arena=0, max_flows=ocap)
        ox = OwnerExchange(p, owner_ctx, seg_cap=int(1.25 * flows_here / world) + 4096,
                           owner_cap=ocap, map_cap=xcap, max_total_records=world * n)
    elif fhx:
        from tcbee_amd.dist import FlowHashExchange
        merged = tcbee_amd.PacketParser(device=torch.cuda.current_device(), max_frames=1024,
                                        max_arena=0, max_flows=world * xcap)
        fx = FlowHashExchange(p, xcap, gidx)
    elif multi:
        from tcbee_amd.dist import FlowMerge, OverlappedMerge
        merged = tcbee_amd.PacketParser(device=torch.cuda.current_device(), max_frames=1024,
                                        max_arena=0, max_flows=world * xcap)
        fm = FlowMerge(p, merged, xcap, n_global if flowhash else world * n, nbuf=nbuf)
        fm.gidx = gidx
        om = (OverlappedMerge(fm, nbuf=nbuf, timing=os.environ.get("TCBEE_BENCH_XTIME", "1") != "0")
              if overlap else None)
    count = [0]

    def step():
        # one step = one fresh trace: empty flow table, parse + classify the shard,
        # then (N>1) the RCCL flow-table merge, the local->global id remap and the
        # counter all-reduce, overlapping the next step's parse
        k = count[0] % nbuf
        count[0] += 1
        b = slots[k]
        if ox is not None:
            b["ctr"].zero_()
            p.reset_flows(stream=stream, sync=False)
            ox.step(d_arena, alen, d_off, d_len, d_ts, n, b["rec"], n, b["hash"], b["id"],
                    b["n"], b["ctr"], stream)
            dist.all_reduce(b["ctr"])
            return
        if fx is not None:
            cs = ids_side if ids_side is not None else torch.cuda.current_stream()
            with torch.cuda.stream(cs):  # the counters live on K3's stream
                b["ctr"].zero_()
            p.reset_flows(stream=stream, sync=False)
            fx.reset()
            fx.step(d_arena, alen, d_off, d_len, d_ts, n, b["rec"], n, b["hash"], b["id"],
                    b["n"], b["ctr"], stream, ids_stream=ids_stream)
            with torch.cuda.stream(cs):
                dist.all_reduce(b["ctr"])  # global INGRESS/HANDLED/DROPPED
            return
        if multi:
            if om is not None:
                om.acquire(k)
            b["ctr"].zero_()
        if not warm:  # warm (N=1 extra leg): the table persists, a recorder's steady state
            p.reset_flows(stream=stream, sync=False)
        p.parse_device(d_arena, alen, d_off, d_len, d_ts, n, b["rec"], n, b["hash"], b["id"],
                       b["n"], b["ctr"], stream=stream, ids_stream=ids_stream)
        if om is not None:
            om.submit(k, b["id"], b["n"], n, ctr=b["ctr"])
        elif fm is not None:  # TCBEE_BENCH_OVERLAP=0: the exchange in line, one stream
            fm.step(b["id"], b["n"], n, stream=stream)
            dist.all_reduce(b["ctr"])

    log(f"rank {rank}: {n} frames resident; {warmup} warm-up + {steps} timed steps")
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    p.profile(True)
    if om is not None:
        om.spans.clear()
    if fx is not None:
        fx.timing = os.environ.get("TCBEE_BENCH_XTIME", "1") != "0"
        fx.spans.clear()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t_issue = time.perf_counter()  # the host's issue time (a step rate near it: host-bound)
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    t1 = time.perf_counter()
    k1_ms, k1_launches = p.profile_read()
    elapsed = t1 - t0
    log(f"rank {rank}: {steps} steps in {elapsed * 1e3:.1f} ms; validating")
    fx_ms = fx.exchange_ms() if fx is not None else None
    status = p.status()

    # validation (untimed): counts, flow table, and a bit-exact sample vs the oracle
    last = slots[(count[0] - 1) % nbuf]
    nrec = int(last["n"].item())
    if multi and p.flow_count() > xcap:
        raise RuntimeError(f"rank {rank}: {p.flow_count()} flows exceed the exchange cap {xcap}")
    if fx is not None:
        # the global table, assembled once after the timed steps (not part of a step)
        flows = fx.merged_flows(merged, last["n"], n, n_global)
    elif ox is not None:
        flows = ox.merged_flows(merged, last["n"], n)
    else:
        flows = (merged if merged is not None else p).flows()
    check = {"records": nrec, "flows": int(len(flows)), "status": status,
             "pkts_total": int(flows["pkts"].sum()),
             "host_issue_ms_per_step": round((t_issue - t0) / steps * 1e3, 4)}
    if multi:
        check["ingress_global"] = int(last["ctr"][0].item())
        if fx is not None:
            check["exchange"] = ("flow-hash: first-frame all-gather (8 B x "
                                 f"{xcap + 2} per rank) + global ids between K2 and K3")
            # in-line span per step on the rank's stream (first frames .. global ids)
            check["exchange_ms"] = round(fx_ms, 4) if fx_ms is not None else None
        if ox is not None:
            check["exchange"] = (f"owner: all-to-all of {ox.seg_cap}-entry owner segments, "
                                 "owner merge, first_seen all-gather, ids all-to-all back, "
                                 "between K2 and K3")
        if om is not None:
            # side-stream span of one step's exchange (RCCL all-gather of the tables,
            # merge, id remap, counter all-reduce), overlapping the next parse
            xm = om.exchange_ms()
            check["exchange_ms"] = round(xm, 4) if xm is not None else None
            check["exchange_entries_per_rank"] = xcap
    if flowhash:
        check["frames_local"] = n
        check.update(rss_info)
        if full_check and not multi:
            # one GPU's share (no exchange): every record, hash, shard-local id and the
            # whole table, the oracle fed the very frames the GPU parsed
            check.update(validate_shard_full(torch, d_arena, d_off, d_len, d_ts, last["rec"],
                                             last["hash"], last["id"], n, nrec, flows))
        elif full_check and fx is not None:
            # N>1: every rank checks ALL of its shard — records, hashes, global ids
            # against a host recomputation of the global first-seen order, and its rows
            # of the merged table (collective)
            log(f"rank {rank}: full check of {n} shard records")
            check.update(validate_shard_global(torch, dist, d_arena, d_off, d_len, d_ts,
                                               last["rec"], last["hash"], last["id"], gidx, n,
                                               nrec, flows))
        else:
            # every rank checks its own shard (global ids included) against the oracle
            check.update(validate_shard(torch, last["rec"], last["hash"], last["id"], gidx, n,
                                        sizes, kind, n_flows, seed, nrec, global_ids=multi))
    elif rank == 0 and full_check and not multi:
        check.update(validate_full(torch, last["rec"], last["hash"], last["id"], n, sizes, kind,
                                   n_flows, seed, nrec, flows,
                                   table_mult=count[0] if warm else 1))
    else:
        check.update(validate_sample(torch, last["rec"], last["hash"], n, sizes, kind, n_flows,
                                     seed, first, nrec))
    if multi:
        check.update(all_ranks_check(torch, dist, check, status, n, n_global if flowhash
                                     else world * n, flows, last["ctr"]))
    if ox is not None:
        ox.owner.close()
    p.close()
    if merged is not None:
        merged.close()
    del d_arena, slots
    torch.cuda.empty_cache()
    return elapsed, k1_ms / max(k1_launches, 1), nrec, check, n


def all_ranks_check(torch, dist, check, status, n_local, n_global, flows, ctr):
    """One verdict for the whole job (collective): every rank's own oracle check and
    context status, MIN-reduced into all_ranks_bit_exact; the global table and
    counters against the global frame count (every synthetic frame is accepted);
    the flow-hash shard imbalance (max / mean local frames), which bounds weak-scaling
    efficiency."""
    full = "full_bit_exact" in check
    ok = bool(check.get("full_bit_exact", check.get("sample_bit_exact", False))) and status == 0
    if "merged_rows_exact" in check:
        ok = ok and bool(check["merged_rows_exact"])
    v = torch.tensor([int(ok)], dtype=torch.int64, device="cuda")
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    # every rank's own verdict and check kind, for the line (rank order)
    flags = [torch.zeros(2, dtype=torch.int64, device="cuda") for _ in range(dist.get_world_size())]
    dist.all_gather(flags, torch.tensor([int(ok), int(full)], dtype=torch.int64, device="cuda"))
    mx = torch.tensor([n_local], dtype=torch.int64, device="cuda")
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    sm = torch.tensor([n_local], dtype=torch.int64, device="cuda")
    dist.all_reduce(sm)
    world = dist.get_world_size()
    mean = int(sm.item()) / world
    per = [f.cpu().tolist() for f in flags]
    return {"all_ranks_bit_exact": bool(v.item()), "ranks_checked": world,
            "ranks_full_bit_exact": [bool(a) and bool(b) for a, b in per],
            "all_ranks_checked_in_full": all(bool(b) for _, b in per),
            "frames_local_max": int(mx.item()), "frames_local_mean": round(mean, 1),
            "shard_imbalance": round(int(mx.item()) / mean, 4) if mean else None,
            "global_frames_ok": int(sm.item()) == n_global,
            "global_pkts_ok": int(flows["pkts"].sum()) == n_global,
            "global_ingress_ok": int(ctr[0].item()) == n_global}


def validate_shard(torch, d_rec, d_hash, d_id, gidx, n, sizes, kind, n_flows, seed, nrec,
                   sample=200_000, global_ids=True):
    """Flow-hash shard: the first `sample` local records (hash, flow id) vs the
    oracle over the global trace prefix that holds them (a flow's global id only
    depends on the first-seen order up to its own first frame; without the
    exchange the ids are the shard's own first-seen order)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tcbee_amd
    from oracle_py import Oracle
    k = min(sample, n)
    g = gidx[:k].cpu().numpy().astype(np.int64)
    glob = tcbee_amd.synth_trace(int(g[-1]) + 1, sizes=sizes, kind=kind, n_flows=n_flows,
                                 seed=seed)
    rec, fh, fi, _, _ = Oracle().parse(glob)  # every synthetic frame is accepted
    want = fi[g]
    if not global_ids and k:
        # the shard's own dense ids: order of first appearance within the shard
        u, first = np.unique(want, return_index=True)
        local = np.empty(len(u), dtype=np.uint32)
        local[np.argsort(first, kind="stable")] = np.arange(len(u), dtype=np.uint32)
        want = local[np.searchsorted(u, want)]
    ok = (nrec == n
          and np.array_equal(d_rec[:k * 74].cpu().numpy().reshape(-1, 74), rec[g])
          and np.array_equal(d_hash[:k].cpu().numpy().view(np.uint32), fh[g])
          and np.array_equal(d_id[:k].cpu().numpy().view(np.uint32), want))
    return {"sample_bit_exact": bool(ok), "sample_frames": k,
            "sample_global_prefix": int(g[-1]) + 1 if k else 0}


def validate_shard_full(torch, d_arena, d_off, d_len, d_ts, d_rec, d_hash, d_id, n, nrec,
                        gpu_flows, chunk=2_000_000):
    """A flow-hash shard parsed alone (N=1, no exchange): every record, flow hash and
    shard-local flow id, and the whole flow table, vs the oracle run over the SAME
    frames (copied back from the device arena chunk by chunk, one oracle flow table
    carried across the chunks). The device generator's frames equal the host
    generator's (tests/test_manifest.py); here the shard's global frame indices are
    scattered, so the frames are taken from where the GPU read them."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import Oracle
    from tcbee_amd.trace import Trace
    orc = Oracle()
    ft = orc.new_flowtab(1 << 18)
    t0 = time.perf_counter()
    ok = nrec == n
    bad_at = None
    try:
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            off = d_off[lo:hi].cpu().numpy().view(np.uint64)
            ln = d_len[lo:hi].cpu().numpy().view(np.uint32)
            a0, a1 = int(off[0]), int(off[-1]) + int(ln[-1])
            arena = d_arena[a0:a1].cpu().numpy()
            tr = Trace(arena, (off - np.uint64(a0)).astype(np.uint64), ln.copy(),
                       d_ts[lo:hi].cpu().numpy().view(np.uint64).copy())
            rec, fh, fi, _, _ = orc.parse(tr, ft=ft, record_base=lo)
            same = (len(rec) == hi - lo
                    and np.array_equal(d_rec[lo * 74: hi * 74].cpu().numpy().reshape(-1, 74), rec)
                    and np.array_equal(d_hash[lo:hi].cpu().numpy().view(np.uint32), fh)
                    and np.array_equal(d_id[lo:hi].cpu().numpy().view(np.uint32), fi))
            if not same and bad_at is None:
                bad_at = lo
            ok = ok and same
            if (lo // chunk) % 10 == 9:
                log(f"shard check: {hi}/{n} records ({time.perf_counter() - t0:.0f}s)")
        table = orc.flows(ft)
    finally:
        orc.free_flowtab(ft)
    table_ok = len(table) == len(gpu_flows) and np.array_equal(table, gpu_flows)
    out = {"full_bit_exact": bool(ok), "full_records": n, "flow_table_exact": bool(table_ok),
           "full_check_s": round(time.perf_counter() - t0, 1)}
    if bad_at is not None:
        out["first_bad_chunk"] = bad_at
    return out


def validate_shard_global(torch, dist, d_arena, d_off, d_len, d_ts, d_rec, d_hash, d_id, gidx,
                          n, nrec, merged_flows, chunk=2_000_000):
    """N>1 flow-hash shards, checked IN FULL on every rank (collective):
      1. every record and flow hash of this rank's shard vs the oracle run over the
         SAME frames (copied back from the device arena chunk by chunk, one oracle flow
         table carried across the chunks) — the oracle's shard-local ids are kept;
      2. the GLOBAL ids, against an independent host recomputation of the global
         first-seen order: each local flow's first global frame (the oracle table's
         first record -> gidx) is all-gathered over the ranks (padded to the largest
         rank's flow count), numpy sorts the union, and a flow's global id is its rank
         in that order; every device id of the shard must equal
         global_id[oracle local id]. No device exchange output is used;
      3. the merged global table (FlowHashExchange.merged_flows, identical on every
         rank): this rank's flows' rows — tuple, pkts, bytes, first_seen = global
         record index (every synthetic frame is accepted: = the first global frame) —
         against its oracle table, and the merged flow count against the union's.
    Host memory: 4 B per local record of oracle ids, kept between passes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import Oracle
    from tcbee_amd.trace import Trace
    orc = Oracle()
    ft = orc.new_flowtab(1 << 18)
    t0 = time.perf_counter()
    rec_ok = nrec == n
    bad_at = None
    fi_local = np.empty(n, dtype=np.uint32)
    g_host = gidx[:n].cpu().numpy().astype(np.int64)
    try:
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            off = d_off[lo:hi].cpu().numpy().view(np.uint64)
            ln = d_len[lo:hi].cpu().numpy().view(np.uint32)
            a0, a1 = int(off[0]), int(off[-1]) + int(ln[-1])
            arena = d_arena[a0:a1].cpu().numpy()
            tr = Trace(arena, (off - np.uint64(a0)).astype(np.uint64), ln.copy(),
                       d_ts[lo:hi].cpu().numpy().view(np.uint64).copy())
            rec, fh, fi, _, _ = orc.parse(tr, ft=ft, record_base=lo)
            same = (len(rec) == hi - lo
                    and np.array_equal(d_rec[lo * 74: hi * 74].cpu().numpy().reshape(-1, 74), rec)
                    and np.array_equal(d_hash[lo:hi].cpu().numpy().view(np.uint32), fh))
            if len(fi) == hi - lo:
                fi_local[lo:hi] = fi
            if not same and bad_at is None:
                bad_at = lo
            rec_ok = rec_ok and same
            if (lo // chunk) % 10 == 9:
                log(f"shard check: {hi}/{n} records ({time.perf_counter() - t0:.0f}s)")
        table = orc.flows(ft)
    finally:
        orc.free_flowtab(ft)
    # global first-seen order from the ranks' oracle tables (host recomputation)
    nloc = len(table)
    first_g = g_host[table["first_seen"].astype(np.int64)] if nloc else np.zeros(0, np.int64)
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    cnt = torch.tensor([nloc], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    cnts = [int(c.item()) for c in cnts]
    pad = max(max(cnts), 1)
    mine = torch.full((pad,), -1, dtype=torch.int64, device=dev)
    mine[:nloc] = torch.from_numpy(first_g)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    allf = np.concatenate([parts[r][:cnts[r]].cpu().numpy() for r in range(world)])
    order = np.argsort(allf, kind="stable")
    gid_all = np.empty(len(allf), dtype=np.int64)
    gid_all[order] = np.arange(len(allf))
    base = sum(cnts[:rank])
    gid = gid_all[base:base + nloc]
    distinct = len(np.unique(allf)) == len(allf)  # flows of disjoint shards: distinct frames
    ids_ok = rec_ok and distinct
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        want = gid[fi_local[lo:hi].astype(np.int64)].astype(np.uint32) if nloc else \
            np.zeros(hi - lo, np.uint32)
        ids_ok = ids_ok and np.array_equal(d_id[lo:hi].cpu().numpy().view(np.uint32), want)
    # this rank's rows of the merged global table
    mf = merged_flows
    table_ok = len(mf) == len(allf) and nloc > 0
    if table_ok:
        rows = mf[gid]
        table_ok = (np.array_equal(rows["tuple"], table["tuple"])
                    and np.array_equal(rows["pkts"], table["pkts"])
                    and np.array_equal(rows["bytes"], table["bytes"])
                    and np.array_equal(rows["first_seen"].astype(np.int64), first_g))
    out = {"full_bit_exact": bool(rec_ok and ids_ok), "full_records": n,
           "records_hashes_exact": bool(rec_ok), "global_ids_exact": bool(ids_ok),
           "merged_rows_exact": bool(table_ok), "flows_local": nloc,
           "flows_global_recomputed": len(allf), "full_check_s": round(time.perf_counter() - t0, 1)}
    if bad_at is not None:
        out["first_bad_chunk"] = bad_at
    return out


def validate_full(torch, d_rec, d_hash, d_id, n, sizes, kind, n_flows, seed, nrec, gpu_flows,
                  chunk=2_000_000, table_mult=1):
    """Every record, flow hash and flow id of the timed run vs the oracle streamed over
    the same trace in chunks (one flow table carried across them), and the whole
    flow table (untimed; config 3 at N=1). table_mult: the table saw the trace that
    many times (warm leg): same flows, ids and first_seen, pkts/bytes multiplied."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tcbee_amd
    from oracle_py import Oracle
    orc = Oracle()
    ft = orc.new_flowtab(1 << 15)
    t0 = time.perf_counter()
    ok = nrec == n
    bad_at = None
    try:
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            tr = tcbee_amd.synth_trace(hi - lo, sizes=sizes, kind=kind, n_flows=n_flows,
                                       seed=seed, first_index=lo)
            rec, fh, fi, _, _ = orc.parse(tr, ft=ft, record_base=lo)
            # synthetic frames are all accepted: record index == frame index
            same = (len(rec) == hi - lo
                    and np.array_equal(d_rec[lo * 74: hi * 74].cpu().numpy().reshape(-1, 74), rec)
                    and np.array_equal(d_hash[lo:hi].cpu().numpy().view(np.uint32), fh)
                    and np.array_equal(d_id[lo:hi].cpu().numpy().view(np.uint32), fi))
            if not same and bad_at is None:
                bad_at = lo
            ok = ok and same
            if (lo // chunk) % 10 == 9:
                log(f"full check: {hi}/{n} records ({time.perf_counter() - t0:.0f}s)")
        table = orc.flows(ft)
    finally:
        orc.free_flowtab(ft)
    if table_mult != 1:
        table = table.copy()
        table["pkts"] *= np.uint64(table_mult)
        table["bytes"] *= np.uint64(table_mult)
    table_ok = len(table) == len(gpu_flows) and np.array_equal(table, gpu_flows)
    out = {"full_bit_exact": bool(ok), "full_records": n, "flow_table_exact": bool(table_ok),
           "full_check_s": round(time.perf_counter() - t0, 1)}
    if bad_at is not None:
        out["first_bad_chunk"] = bad_at
    return out


def validate_sample(torch, d_rec, d_hash, n, sizes, kind, n_flows, seed, first, nrec,
                    sample=200_000):
    """Records [0, sample) and the last `sample` records vs the oracle on the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tcbee_amd
    from oracle_py import Oracle
    orc = Oracle()
    ok = True
    for lo in (0, max(0, n - sample)):
        hi = min(n, lo + sample)
        tr = tcbee_amd.synth_trace(hi - lo, sizes=sizes, kind=kind, n_flows=n_flows, seed=seed,
                                   first_index=first + lo)
        rec, fh, _, _, _ = orc.parse(tr)
        # synthetic frames are all accepted, so record index == frame index
        g = d_rec[lo * 74: hi * 74].cpu().numpy().reshape(-1, 74)
        gh = d_hash[lo:hi].cpu().numpy().view(np.uint32)
        ok = ok and len(rec) == hi - lo and np.array_equal(g, rec) and np.array_equal(gh, fh)
    return {"sample_bit_exact": bool(ok and nrec == n), "sample_frames": 2 * sample}


def cpu_baseline(sizes, kind, n_flows, seed, seconds, threads, sample_n=2_000_000):
    """The reference record path restated in C (oracle), timed on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tcbee_amd
    from oracle_py import Oracle
    orc = Oracle()
    tr = tcbee_amd.synth_trace(sample_n, sizes=sizes, kind=kind, n_flows=n_flows, seed=seed)
    out = {}
    for t in sorted({1, threads}):
        log(f"cpu baseline: {t} thread(s)")
        done, t0 = 0, time.perf_counter()
        while True:
            orc.baseline(tr, threads=t)
            done += tr.n
            el = time.perf_counter() - t0
            if el >= seconds / (2 if t == 1 and threads > 1 else 1):
                break
        out[t] = (done / el / 1e6, done, el)
    # CPU-1-file: one thread through the drain task's buffered file
    # path (orc_baseline_file), xdp.tcp on tmpfs; the file is removed between reps
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="tcbee_cpu_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        path = os.path.join(d, "xdp.tcp")
        done, el = 0, 0.0
        while el < seconds / 4:
            t0 = time.perf_counter()
            orc.baseline_file(tr, path)
            el += time.perf_counter() - t0
            done += tr.n
            os.unlink(path)
        out["file"] = (done / el / 1e6, done, el)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return out, tr.n


def _lib_identity() -> dict:
    from tcbee_amd import _lib
    return _lib.lib_identity()


def host_cores() -> int:
    """The host cores this job may use: what `nproc` prints (coreutils honours
    OMP_NUM_THREADS, which the GPU box sets to the job's CPU share, 16 per GPU;
    os.cpu_count() there is the whole machine's 256 logical CPUs, and 256
    threads on a 16-CPU share oversubscribe it)."""
    import subprocess
    try:
        return max(1, int(subprocess.run(["nproc"], capture_output=True, text=True,
                                         timeout=10).stdout.strip()))
    except (OSError, ValueError, subprocess.SubprocessError):
        try:
            return len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            return os.cpu_count() or 1


def cgroup_cpus():
    """CPU quota of this cgroup (cpu.max), None if unlimited/unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def host_e2e(sizes, kind, n_flows, seed, n=20_000_000, reps=9, threads=None):
    """End-to-end rates from host memory: frames in pageable host RAM -> records +
    flow ids back in pageable host RAM (H2D and D2H inside the timed region).
      pipe_window64: tcbee_pipe, header-window staging (frame bytes [12, 76): one
                     64-B line per frame shipped; pipe_window80: bytes [0, 80))
      pipe_whole:    tcbee_pipe, whole frames shipped
      parse_batch:   one synchronous tcbee_parse_batch call (no overlap), 4M frames"""
    import numpy as np

    import tcbee_amd
    from tcbee_amd.pipeline import Pipeline
    # 3/4 of the job's cores: on the 16-CPU share 12 threads (9 gather + 3 copy-out)
    # beat 16 in every paired run (521-556 vs 324-472 Mpkt/s, tools/e2e_cmp.py);
    # the gather is host-memory bound, not CPU bound (no cgroup throttling seen).
    # With registered outputs all of them gather: 12 and 16 equal (562 / 563 Mpkt/s,
    # profiles/r04_e2e_threads.log)
    threads = threads or max(4, host_cores() * 3 // 4)
    log(f"e2e: generating {n} frames on the host")
    tr = tcbee_amd.synth_trace(n, sizes=sizes, kind=kind, n_flows=n_flows, seed=seed)
    out = {"frames": n, "threads": threads, "arena_bytes": int(len(tr.arena))}
    # One output pair (records + ids) for every pipe (a pair per pipe kept
    # ~6 GB of page-locked and pageable outputs live next to the 7 GB trace):
    #   pipe_window64_registered  page-locks it (tcbee_pipe_register_output): each
    #                             chunk's records DMA straight into it;
    #   pipe_window64             the line's E2E number: the SAME pair, direct D2H or
    #                             staging chosen per box by a short calibration on the
    #                             first 4M frames before any timed run
    #                             (Pipeline.calibrate_output; round 4: direct won 515
    #                             to 343 on one box and lost 438 to 452 on another);
    #   pipe_window64_staged      pinned staging + a host copy-out into the pair;
    #   pipe_window80 / pipe_whole  direct D2H, wider windows / whole frames.
    # The variants are timed in interleaved rounds (median per variant): timed one
    # after the other, the first variant ran ~320 Mpkt/s in every bench line of rounds
    # 3-4 while the same box gave 520-560 in a process of its own — the seconds after
    # the 7 GB trace is generated are not the pipeline's steady state
    variants = (("pipe_window64_registered", 64, "registered"), ("pipe_window64", 64, "auto"),
                ("pipe_window64_staged", 64, "staged"), ("pipe_window80", 80, "registered"),
                ("pipe_whole", 0, "registered"))
    pipes, ts = {}, {}
    rec_out, id_out = np.empty((n, 74), np.uint8), np.empty(n, np.uint32)
    ref = None
    identical = True
    try:
        for name, window, mode in variants:
            log(f"e2e: {name} set-up")
            p = Pipeline(device=0, chunk_frames=1 << 20, window=window, depth=4, threads=threads,
                         chunk_bytes=(1 << 29), max_flows=max(4 * n_flows, 1 << 12))
            pipes[name] = p
            if mode != "staged":  # (the first registers the pair, the others borrow it)
                p.register_output(rec_out, id_out)
            for _ in range(2):  # warm-up: pinned staging, first touches
                p.run(tr, out_rec=rec_out, out_id=id_out)
            if ref is None:
                ref = (rec_out.copy(), id_out.copy())
            if mode == "auto":
                p.reset_flows()  # (calibrate_output refuses a pipe that holds flows)
                out["calibration"] = p.calibrate_output(tr, frames=4_000_000, reps=2)
            ts[name] = []
        log(f"e2e: {reps} interleaved rounds")
        last = {}
        for r in range(reps):
            for name, _, _ in variants:
                p = pipes[name]
                p.reset_flows()
                t0 = time.perf_counter()
                last[name] = p.run(tr, out_rec=rec_out, out_id=id_out)
                ts[name].append(time.perf_counter() - t0)
                if r == reps - 1:  # every variant's records and ids equal the first's
                    identical = (identical and np.array_equal(rec_out, ref[0])
                                 and np.array_equal(id_out, ref[1]))
    finally:
        for p in pipes.values():
            p.close()
    for name, window, mode in variants:
        el = float(np.median(ts[name]))
        h2d = n * (window + 12) + (64 if window == 64 else 0) if window else \
            int(len(tr.arena)) + 20 * n
        how = pipes[name].output_mode
        out[name] = {"mpkts": round(n / el / 1e6, 1), "s": round(el, 4), "records": last[name].n,
                     "h2d_bytes": h2d, "h2d_GBs": round(h2d / el / 1e9, 1),
                     "output": ("registered (direct D2H)" if how == "registered"
                                else "staged + copy-out")
                     + (" — chosen by calibration" if mode == "auto" else ""),
                     "best_mpkts": round(n / min(ts[name]) / 1e6, 1)}
    out["outputs_identical"] = bool(identical)
    del rec_out, id_out, ref
    m = 4_000_000
    sub = tr.slice(0, m)
    with tcbee_amd.PacketParser(max_frames=m, max_arena=len(sub.arena),
                                max_flows=max(n_flows, 1 << 12)) as p:
        p.parse(sub)
        t0 = time.perf_counter()
        for _ in range(3):
            p.reset_flows()
            r = p.parse(sub)
        el = (time.perf_counter() - t0) / 3
    out["parse_batch"] = {"mpkts": round(m / el / 1e6, 1), "frames": m}
    return out


def config5_replay(seed, n=1_000_000, n_flows=4, threads=None):
    """Config 5 of BASELINE.json: a trace file replayed end to end — classic pcap
    (tmpfs) -> tcbee_pipe (H2D, K1-K3, D2H) -> xdp.tcp -> the tcbee-process stage
    into SQLite (records pre-grouped by the GPU's flow ids) -> metrics.json. Each
    leg is run twice and the second (warm: library loads, device context) timed;
    it includes pipeline setup (pinned staging) and file creation, as a replay
    does. Checked: the .tcp bytes equal the oracle's records, the database holds
    n_flows flows."""
    import shutil
    import sqlite3
    import tempfile

    import tcbee_amd
    from tcbee_amd import host
    from tcbee_amd.pipeline import replay_pcap
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_py import Oracle
    log("config 5: pcap replay")
    tr = tcbee_amd.synth_trace(n, sizes="64", kind=1 if n_flows > 1 else 0, n_flows=n_flows,
                               seed=seed)
    d = tempfile.mkdtemp(prefix="tcbee_c5_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    # 3/4 of the job's cores: on the 16-CPU share 12 threads (9 gather + 3 copy-out)
    # beat 16 in every paired run (521-556 vs 324-472 Mpkt/s, tools/e2e_cmp.py);
    # the gather is host-memory bound, not CPU bound (no cgroup throttling seen)
    threads = threads or max(4, host_cores() * 3 // 4)
    out = {"frames": n, "flows": n_flows, "frame_bytes": 64, "threads": threads}
    try:
        pcap = os.path.join(d, "trace.pcap")
        host.write_pcap(pcap, tr)
        for name, with_db in (("pcap_to_tcp", False), ("pcap_to_sqlite", True)):
            for rep in range(2):
                prefix = os.path.join(d, f"{name}{rep}_")
                db = prefix + "tcbee.sqlite" if with_db else None
                t0 = time.perf_counter()
                r = replay_pcap(pcap, prefix, db_path=db, threads=threads)
                el = time.perf_counter() - t0
            out[name] = {"mpkts": round(n / el / 1e6, 3), "s": round(el, 3),
                         "records": r["records"]}
            if with_db:
                out[name]["sink"] = r.get("sink")
                con = sqlite3.connect(db)
                try:
                    out[name]["db_flows"] = int(con.execute("select count(*) from flows")
                                                .fetchone()[0])
                finally:
                    con.close()
        rec = Oracle().parse(tr)[0]
        tcp = np.fromfile(os.path.join(d, "pcap_to_tcp1_xdp.tcp"), dtype=np.uint8)
        out["check"] = {"tcp_bytes_exact": bool(tcp.size == rec.size
                                                and np.array_equal(tcp, rec.reshape(-1))),
                        "db_flows_ok": out["pcap_to_sqlite"].get("db_flows") == n_flows}
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return out


def pmc_traffic(args, k1_ms):
    """roofline.traffic: HBM bytes per k_parse launch from the committed rocprofv3 PMC
    passes of this same command (profiles/pmc_k_parse.json, written by
    tools/prof_summary.py: 2 x FETCH_SIZE + WRITE_SIZE). PMC counters cannot be
    read from inside the timed run, so they come from the separate --pmc runs;
    null when the committed profile is for another workload."""
    path = os.path.join(ROOT, "profiles", "pmc_k_parse.json")
    try:
        pmc = json.load(open(path))
    except (OSError, ValueError):
        return {"traffic": None}
    if (pmc.get("frames") != args.frames or pmc.get("sizes") != args.sizes
            or pmc.get("flows") != args.flows):
        return {"traffic": None}
    t = float(pmc["traffic_bytes_per_launch"])
    return {"traffic": round(t / 1e9, 3), "traffic_unit": "GB/launch (HBM, PMC)",
            "traffic_per_frame": round(t / args.frames, 1),
            "traffic_GBs": round(t / (k1_ms * 1e-3) / 1e9, 1)}


def max_over_ranks(torch, dist, x: float) -> float:
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=100_000_000, help="frames per GPU")
    ap.add_argument("--sizes", default="imix", choices=["imix", "64", "imix6"],
                    help="imix6: the IPv6/TCP trace (78/576/1500 B) as the main leg")
    ap.add_argument("--flows", type=int, default=10_000)
    ap.add_argument("--seed", type=int, default=0x7CBEE)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip config-2 and e2e legs")
    ap.add_argument("--e2e-frames", type=int, default=20_000_000)
    ap.add_argument("--shard", default=None, choices=["contig", "flowhash"],
                    help="partition of one global trace of frames x N: flow-hash shards "
                         "(the NIC-RSS view, north_star's partition; default for N > 1) or "
                         "contiguous frame ranges (every GPU sees every flow)")
    ap.add_argument("--config4", action="store_true",
                    help="config 4 of BASELINE.json: 125M IMIX frames per GPU, 1M flows, "
                         "flow-hash shards")
    ap.add_argument("--virtual-world", type=int, default=0,
                    help="N=1 with --shard flowhash: run rank 0's shard of a W-GPU job "
                         "(its frames and flows; no exchange) to measure one GPU's share")
    ap.add_argument("--sample-check", action="store_true",
                    help="N=1: check 2 x 200k records instead of every record + the table")
    ap.add_argument("--c4-frames", type=int, default=125_000_000,
                    help="N>1: frames per GPU of the config-4 leg (1M flows, flow-hash "
                         "shards, FlowHashExchange); 125M = BASELINE.json's 1B at N=8. "
                         "Smaller only to rehearse N ranks on one GPU")
    ap.add_argument("--c4-steps", type=int, default=5)
    args = ap.parse_args()
    if args.config4:
        args.frames, args.flows, args.sizes = 125_000_000, 1_000_000, "imix"
        args.shard = args.shard or "flowhash"

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.shard is None:
        # N = 1: one shard either way (the whole trace); the contiguous build keeps
        # the full bit-exact check of every record
        args.shard = "flowhash" if world > 1 or args.virtual_world > 1 else "contig"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    force_merge = os.environ.get("TCBEE_BENCH_FORCE_MERGE") == "1"
    if world > 1 or force_merge:
        import torch.distributed as dist
        # one process per GPU; TCBEE_DIST_BACKEND=gloo + fewer GPUs than ranks only for
        # rehearsing the N>1 path on a 1-GPU box (ranks then share a device)
        backend = os.environ.get("TCBEE_DIST_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    # One explicit stream for torch ops, RCCL and every tcbee call: the C ABI reads a
    # NULL stream as "the context's own (non-blocking) stream", so passing torch's
    # default-stream handle (0) would put the parse/merge on streams the collectives
    # and the remap do not wait for.
    torch.cuda.set_stream(torch.cuda.Stream())
    kind = 3 if args.sizes == "imix6" else (1 if args.flows > 1 else 0)

    elapsed, k1_ms, nrec, check, n_local = run_device(
        torch, dist, rank, world, args.frames, args.sizes, kind, args.flows, args.steps,
        args.warmup, args.seed, multi=world > 1 or force_merge,
        full_check=not args.sample_check, flowhash=args.shard == "flowhash",
        vworld=args.virtual_world)
    if world > 1:
        elapsed = max_over_ranks(torch, dist, elapsed)
    c4 = None
    if world > 1 and not args.no_extra and not args.config4:
        # north_star's config 4 at N GPUs (BASELINE.json configs[3]): 1M flows,
        # --c4-frames per GPU (1B frames in all at N=8), flow-hash shards, global ids
        # from the FlowHashExchange over RCCL, counters all-reduced; every rank checks
        # its shard against the oracle (collective, all ranks take part)
        log(f"rank {rank}: config-4 leg ({args.c4_frames} frames per GPU, 1M flows)")
        c_el, c_k1, c_n, c_chk, c_local = run_device(
            torch, dist, rank, world, args.c4_frames, "imix", 1, 1_000_000, args.c4_steps, 1,
            args.seed, multi=True, flowhash=True, full_check=not args.sample_check)
        c_el = max_over_ranks(torch, dist, c_el)
        c4 = {"workload": "config4: IMIX 64/576/1500 7:4:1 IPv4/TCP, 1000000 flows, "
                          "flow-hash shards, FlowHashExchange",
              "frames_global": args.c4_frames * world, "frames_per_gpu": args.c4_frames,
              "flows": 1_000_000, "steps": args.c4_steps,
              "mpkts": round(args.c4_frames * world * args.c4_steps / c_el / 1e6, 1),
              "ms_per_step": round(c_el / args.c4_steps * 1e3, 4),
              "k1_ms_rank0": round(c_k1, 4), "exchange_ms_rank0": c_chk.get("exchange_ms"),
              "check": c_chk}
    ms_per_step = elapsed / args.steps * 1e3
    total_frames = args.frames * world * args.steps
    value = total_frames / elapsed / 1e6

    out = None
    if rank == 0:
        # roofline of the dominant kernel (K1 k_parse), algorithmic bytes per launch
        hdr = 74 if args.sizes == "imix6" else V4_HDR_BYTES  # IPv6 / IPv4 TCP headers
        alg_bytes = n_local * (IDX_BYTES + hdr) + nrec * OUT_BYTES
        achieved = alg_bytes / (k1_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpkt/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": {
                "imix": ("config4: " if args.config4 else "config3: ")
                + f"IMIX 64/576/1500 7:4:1 IPv4/TCP, {args.flows} flows",
                "imix6": f"config3 over IPv6/TCP: IMIX 78/576/1500 7:4:1, {args.flows} flows",
                "64": f"64B IPv4/TCP, {args.flows} flow(s)"}[args.sizes],
                       "shard": args.shard + (f" (rank 0 of {args.virtual_world})"
                                              if args.virtual_world and world == 1 else ""),
                       "frames_per_gpu": args.frames, "flows": args.flows,
                       "parallelism": f"shard{world}" + ("+merge" if force_merge and world == 1
                                                         else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         **pmc_traffic(args, k1_ms), "kernel": "k_parse",
                         "k1_ms": round(k1_ms, 4),
                         "alg_bytes_per_frame": IDX_BYTES + hdr + OUT_BYTES},
            "check": check,
            # the binary measured: path + sha256 prefix of the libtcbee_amd.so this process
            # loaded (TCBEE_AB_LIB swaps it only with TCBEE_AB_OPTIN=1: then ab_lib is true)
            **_lib_identity(),
        }
        if dist is not None:
            out["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
        if c4 is not None:
            out["config4_flowhash"] = c4
        if not args.no_extra and world == 1 and not args.config4:
            # (a 0.07-ms step: 200 warm-up steps after the previous leg's idle validation
            #  and 200 timed ones, so that neither the clock ramp nor the timer brackets
            #  weigh in: 3 + 20 read ~3 % slower, tools/c2_warm.py)
            c2_steps = max(args.steps, 200)
            e_el, e_k1, e_n, e_chk, _ = run_device(torch, None, 0, 1, 1_000_000, "64", 0, 1,
                                                c2_steps, max(args.warmup, 200), args.seed,
                                                full_check=True)
            out["config2_1M_64B"] = {"mpkts": round(1_000_000 * c2_steps / e_el / 1e6, 1),
                                     "ms_per_step": round(e_el / c2_steps * 1e3, 4),
                                     "k1_ms": round(e_k1, 4), "check": e_chk}
            # config 3's second run: same frames, flows drawn Zipf(1.1)
            z_el, z_k1, z_n, z_chk, _ = run_device(torch, None, 0, 1, args.frames, args.sizes, 2,
                                                args.flows, args.steps, args.warmup, args.seed,
                                                full_check=not args.sample_check)
            out["config3_zipf"] = {"mpkts": round(args.frames * args.steps / z_el / 1e6, 1),
                                   "ms_per_step": round(z_el / args.steps * 1e3, 4),
                                   "k1_ms": round(z_k1, 4), "zipf_s": 1.1, "check": z_chk}
            # the IPv6 path at the same scale: 100M IPv6/TCP frames (78/576/1500 IMIX:
            # IPv6 needs 74 header bytes), 10k flows; K1 loads the IPv6 tail chunk
            v_el, v_k1, v_n, v_chk, _ = run_device(torch, None, 0, 1, args.frames, "imix6", 3,
                                                args.flows, args.steps, args.warmup, args.seed,
                                                full_check=not args.sample_check)
            v_alg = IDX_BYTES + 74 + OUT_BYTES
            out["config3_ipv6"] = {"mpkts": round(args.frames * args.steps / v_el / 1e6, 1),
                                   "ms_per_step": round(v_el / args.steps * 1e3, 4),
                                   "k1_ms": round(v_k1, 4), "alg_bytes_per_frame": v_alg,
                                   "k1_alg_GBs": round(args.frames * v_alg / v_k1 / 1e6, 1),
                                   "check": v_chk}
            # steady state of a recorder: the same frames with the table kept across
            # steps (every flow known: K1 hits only, K2 ranks nothing new)
            w_el, w_k1, w_n, w_chk, _ = run_device(torch, None, 0, 1, args.frames, args.sizes, 1,
                                                args.flows, args.steps, args.warmup, args.seed,
                                                full_check=not args.sample_check, warm=True)
            out["config3_warm_table"] = {"mpkts": round(args.frames * args.steps / w_el / 1e6, 1),
                                         "ms_per_step": round(w_el / args.steps * 1e3, 4),
                                         "k1_ms": round(w_k1, 4), "check": w_chk}
            # one GPU's shard of config 4 (1B frames / 8 GPUs, 1M flows): every flow
            # appears in every contiguous shard, so each GPU's table holds all 1M
            c4_n, c4_steps = 125_000_000, 5
            c_el, c_k1, c_n, c_chk, _ = run_device(torch, None, 0, 1, c4_n, "imix", 1, 1_000_000,
                                                c4_steps, 1, args.seed, full_check=True)
            out["config4_shard_1M_flows"] = {
                "frames": c4_n, "flows": 1_000_000, "mpkts": round(c4_n * c4_steps / c_el / 1e6, 1),
                "ms_per_step": round(c_el / c4_steps * 1e3, 4), "k1_ms": round(c_k1, 4),
                "check": c_chk}
            # one GPU's share of config 4 under north_star's flow-hash partition at N=8:
            # rank 0's shard of the 1B-frame trace (~125M frames, ~125k flows), no exchange
            v_el, v_k1, v_n, v_chk, v_local = run_device(
                torch, None, 0, 1, c4_n, "imix", 1, 1_000_000, c4_steps, 1, args.seed,
                flowhash=True, vworld=8, full_check=True)
            out["config4_flowhash_share_of_8"] = {
                "frames": v_local, "flows": v_chk.get("flows"),
                "mpkts": round(v_local * c4_steps / v_el / 1e6, 1),
                "ms_per_step": round(v_el / c4_steps * 1e3, 4), "k1_ms": round(v_k1, 4),
                "check": v_chk}
            out["e2e_host"] = host_e2e(args.sizes, kind, args.flows, args.seed,
                                       n=args.e2e_frames)
            out["config5_replay"] = config5_replay(args.seed)
        if not args.no_cpu and world == 1:
            # every core this process may run on (= nproc; on the GPU box the job's
            # CPU share, not the machine's logical CPU count)
            threads = host_cores()
            res, sample_n = cpu_baseline(args.sizes, kind, args.flows, args.seed,
                                         args.cpu_seconds, threads)
            v, done, el = res[threads]
            out["cpu_baseline"] = {
                "value": round(v, 2), "unit": "Mpkt/s", "cores": threads, "kind": "port",
                "nproc": threads, "machine_cpus": os.cpu_count(), "cgroup_cpus": cgroup_cpus(),
                "sample": (f"{sample_n} frames of the same workload, repeated {done // sample_n}x "
                           f"({el:.1f}s); oracle/tcbee_oracle.c orc_baseline_run = xdp_hook + "
                           "per-thread FLOWS(100) + bincode serialize"),
                "single_thread": round(res[1][0], 2),
                "single_thread_file": round(res["file"][0], 2),
                "file_sample": "1 thread, records appended to tmpfs xdp.tcp through a 720000-B "
                               "buffer (handlers/mod.rs:70-139)"}
        log("done")
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
