"""Worker for the world-size-2 gloo test of the multi-GPU choreography (CPU)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def run(rank, world, port, n, cap, result_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from merge_ref import entries_to_table, merge, table_to_entries
    from oracle_py import Oracle
    from tracegen import mixed_trace

    from tcbee_amd.dist import gather_tables, shard_range

    tr = mixed_trace(n, seed=404, n_flows=700)
    lo, hi = shard_range(tr.n, rank, world)
    orc = Oracle()
    rec, fh, fi, ctr, table = orc.parse(tr.slice(lo, hi))
    ent = torch.from_numpy(table_to_entries(table, cap))
    meta = torch.tensor([len(table), len(rec)], dtype=torch.int64)
    all_ent, all_meta = gather_tables(ent, meta)
    all_ent = all_ent.numpy().reshape(world, cap, 8)
    all_meta = all_meta.numpy().reshape(world, 2)
    tables = [entries_to_table(all_ent[r], int(all_meta[r, 0])) for r in range(world)]
    merged, maps = merge(tables, [int(all_meta[r, 1]) for r in range(world)])
    gids = maps[rank][fi] if len(fi) else fi
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), merged=merged.view(np.uint8),
             gids=gids, lo=lo, hi=hi, nrec=len(rec))
    dist.barrier()
    dist.destroy_process_group()


def run_owner(rank, world, port, n, cap, result_dir, filter_port=0):
    """CPU mirror of tcbee_amd.dist.OwnerExchange over gloo (contiguous shards): the
    oracle's shard table bucketed by owner (fold32 flow hash % world), the equal-split
    all-to-all, the owner's merge (merge_ref), global ids from the all-gathered
    owner first_seen arrays, and the ids sent back to the entries' senders."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from merge_ref import entries_to_table, merge, table_to_entries
    from oracle_py import Oracle
    from tracegen import mixed_trace

    from tcbee_amd.dist import all_gather_flat, all_to_all_flat, shard_range

    tr = mixed_trace(n, seed=404, n_flows=700)
    lo, hi = shard_range(tr.n, rank, world)
    rec, fh, fi, ctr, table = Oracle().parse(tr.slice(lo, hi), filter_port=filter_port)
    # owner of each local flow: the fold32 hash of (any) one of its records
    fhash = np.zeros(len(table), dtype=np.uint32)
    fhash[fi] = fh
    own = (fhash % world).astype(np.int64)
    send = np.zeros((world, cap, 8), dtype=np.int64)
    lid = np.zeros((world, cap), dtype=np.int64)
    meta = np.zeros(world + 1, dtype=np.int64)
    for o in range(world):
        sel = np.nonzero(own == o)[0]
        meta[o] = len(sel)
        send[o] = table_to_entries(table[sel], cap)
        lid[o, :len(sel)] = sel
    meta[world] = len(rec)
    all_meta = torch.zeros(world * (world + 1), dtype=torch.int64)
    all_gather_flat(all_meta, torch.from_numpy(meta))
    am = all_meta.numpy().reshape(world, world + 1)
    recv = torch.zeros(world * cap, 8, dtype=torch.int64)
    all_to_all_flat(recv, torch.from_numpy(send.reshape(-1, 8)))
    recv = recv.numpy().reshape(world, cap, 8)
    segs = [entries_to_table(recv[r], int(am[r, rank])) for r in range(world)]
    owned, maps = merge(segs, [int(am[r, world]) for r in range(world)])
    fs = np.zeros(cap + 1, dtype=np.int64)
    fs[:len(owned)] = owned["first_seen"].astype(np.int64)
    fs[cap] = len(owned)
    all_fs = torch.zeros(world * (cap + 1), dtype=torch.int64)
    all_gather_flat(all_fs, torch.from_numpy(fs))
    af = all_fs.numpy().reshape(world, cap + 1)
    gmap_o = np.arange(len(owned), dtype=np.int64)
    for r in range(world):
        if r != rank:
            gmap_o += np.searchsorted(af[r, :af[r, cap]], fs[:len(owned)])
    ret = np.zeros((world, cap), dtype=np.int64)
    for r in range(world):
        ret[r, :int(am[r, rank])] = gmap_o[maps[r]]
    back = torch.zeros(world * cap, dtype=torch.int64)
    all_to_all_flat(back, torch.from_numpy(ret.reshape(-1)))
    back = back.numpy().reshape(world, cap)
    gmap = np.zeros(len(table), dtype=np.int64)
    for o in range(world):
        gmap[lid[o, :meta[o]]] = back[o, :meta[o]]
    gids = gmap[fi] if len(fi) else fi
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), gids=gids, lo=lo, hi=hi)
    dist.barrier()
    dist.destroy_process_group()


def run_flowhash(rank, world, port, n, cap, result_dir, filter_port):
    """The flow-hash choreography on CPU (oracle tables, gloo collectives): host
    partition -> per-rank parse -> first_seen to global frame index through the
    record -> frame map -> all-gather + merge (no rebase) -> per-rank records
    before each merged flow's first frame, all-reduced -> global record index."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from merge_ref import entries_to_table, merge, table_to_entries
    from oracle_py import Oracle
    from tracegen import mixed_trace

    from tcbee_amd import host
    from tcbee_amd.dist import gather_tables

    tr = mixed_trace(n, seed=404, n_flows=700)
    sub, gidx = host.flowhash_shard(tr, world, rank)
    orc = Oracle()
    rec, fh, fi, ctr, table = orc.parse(sub, filter_port=filter_port)
    rec_frame = np.nonzero(orc.accept_mask(sub, filter_port=filter_port))[0]
    gframe = gidx[rec_frame]                      # ascending global frame of each record
    table = table.copy()
    table["first_seen"] = gframe[table["first_seen"].astype(np.int64)]
    ent = torch.from_numpy(table_to_entries(table, cap))
    meta = torch.tensor([len(table), 0], dtype=torch.int64)
    all_ent, all_meta = gather_tables(ent, meta)
    all_ent = all_ent.numpy().reshape(world, cap, 8)
    all_meta = all_meta.numpy().reshape(world, 2)
    tables = [entries_to_table(all_ent[r], int(all_meta[r, 0])) for r in range(world)]
    merged, maps = merge(tables, [0] * world)
    cnt = torch.from_numpy(np.searchsorted(gframe, merged["first_seen"].astype(np.int64))
                           .astype(np.int64))
    dist.all_reduce(cnt)
    merged["first_seen"] = cnt.numpy().astype(np.uint64)
    gids = maps[rank][fi] if len(fi) else fi
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), merged=merged.view(np.uint8),
             gids=gids, gidx=gidx, rec=rec)
    dist.barrier()
    dist.destroy_process_group()


def run_gpu(rank, world, port, n, cap, result_dir, mode, n_flows=3000, filter_port=0,
            backend="gloo", map_caps=None):
    """N>1 choreography on the GPU: ranks share device 0 over gloo. mode "step":
    FlowMerge.step on one stream; mode "overlap": OverlappedMerge over 3 steps of
    the same shard (fresh table each step, output slots rotating), as bench.py;
    mode "flowhash": the rank's flow-hash shard of a synthetic global trace of n
    frames, built by the device generator, exchanged with global first_seen;
    mode "flowhash_real": the rank's flow-hash shard (host partitioner, the NIC-RSS
    step) of a mixed trace with rejected and FILTER_PORT-filtered frames, placed
    through the parse's record -> frame map; mode "flowhash_noframe": the same
    without the map (must be refused: TCBEE_ESHARD). map_caps (mode "owner"): the
    id-map size of each rank (default `cap` on every rank)."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_stream(torch.cuda.Stream())
    import tcbee_amd
    from tcbee_amd import host
    from tcbee_amd.dist import FlowMerge, OverlappedMerge, shard_range
    from tracegen import mixed_trace

    fhx = mode.startswith("fhx")  # FlowHashExchange instead of FlowMerge
    if fhx:
        mode = "flowhash" + mode[3:]
    gidx = None
    if mode in ("flowhash", "flowhash_rss"):
        import bench
        s0 = torch.cuda.current_stream().cuda_stream
        # flowhash_rss: the bench's RSS table balanced on the bucket loads (same on
        # every rank) instead of fold32(hash) % world
        rss = bench.rss_for(torch, n, world, 1, n_flows, 0x7CBEE, s0)[0] if mode == "flowhash_rss" else None
        arena, alen, off, ln, ts, gidx, m = bench.build_shard_trace(
            torch, n, world, rank, "imix", 1, n_flows, 0x7CBEE, s0, rss=rss)
        if rss is not None:
            np.save(os.path.join(result_dir, f"rss{rank}.npy"), rss.cpu().numpy().view(np.uint16))
    else:
        tr = mixed_trace(n, seed=404, n_flows=n_flows)
        if mode.startswith("flowhash_"):
            sub, g = host.flowhash_shard(tr, world, rank)
            gidx = torch.from_numpy(g).cuda()
        else:
            lo, hi = shard_range(tr.n, rank, world)
            sub = tr.slice(lo, hi)
        m = sub.n
        alen = len(sub.arena)
        arena = torch.zeros(len(sub.arena) + 64, dtype=torch.uint8, device="cuda")
        arena[:len(sub.arena)] = torch.from_numpy(sub.arena).cuda()
        off = torch.from_numpy(sub.offset.view(np.int64)).cuda()
        ln = torch.from_numpy(sub.caplen.view(np.int32)).cuda()
        ts = torch.from_numpy(sub.ts_ns.view(np.int64)).cuda()
    with_frame = mode == "flowhash_real"  # (fhx_real too: the prefix was rewritten)
    nbuf = 2 if mode == "overlap" else 1
    slots = [{"rec": torch.empty(m * 74 + 64, dtype=torch.uint8, device="cuda"),
              "hash": torch.empty(m, dtype=torch.int32, device="cuda"),
              "id": torch.empty(m, dtype=torch.int32, device="cuda"),
              "frame": torch.empty(m, dtype=torch.int32, device="cuda") if with_frame else None,
              "n": torch.zeros(1, dtype=torch.int64, device="cuda"),
              "ctr": torch.zeros(4, dtype=torch.int64, device="cuda")} for _ in range(nbuf)]
    s = torch.cuda.current_stream().cuda_stream
    status = 0
    with tcbee_amd.PacketParser(max_frames=max(m, 1), max_flows=cap) as p, \
            tcbee_amd.PacketParser(max_frames=1024, max_flows=world * cap) as mg:
        if mode == "owner":
            from tcbee_amd.dist import OwnerExchange
            # per-owner segments: a rank holds at most `cap` flows, an owner about
            # 1/world of the global ones (generous here: tests cover small traces)
            ox = OwnerExchange(p, mg, seg_cap=cap, owner_cap=cap,
                               map_cap=map_caps[rank] if map_caps else cap,
                               max_total_records=n)
            for i in range(2):  # the second step re-uses every buffer of the first
                b = slots[0]
                b["ctr"].zero_()
                p.reset_flows(stream=s, sync=False)
                ox.step(arena, alen, off, ln, ts, m, b["rec"], m, b["hash"], b["id"], b["n"],
                        b["ctr"], s, filter_port=filter_port)
                dist.all_reduce(b["ctr"])
            torch.cuda.synchronize()
            status = p.status()
            merged = ox.merged_flows(mg, b["n"], m)
        elif fhx:
            from tcbee_amd.dist import FlowHashExchange
            fx = FlowHashExchange(p, cap, gidx if gidx is not None
                                  else torch.arange(m, dtype=torch.int64, device="cuda"))
            steps = 2  # the second step re-uses every buffer of the first
            for i in range(steps):
                b = slots[0]
                b["ctr"].zero_()
                p.reset_flows(stream=s, sync=False)
                fx.reset()
                fx.step(arena, alen, off, ln, ts, m, b["rec"], m, b["hash"], b["id"], b["n"],
                        b["ctr"], s, filter_port=filter_port, rec_frame=b["frame"])
                dist.all_reduce(b["ctr"])
            torch.cuda.synchronize()
            status = p.status()
            merged = fx.merged_flows(mg, b["n"], m, n, rec_frame=b["frame"])
            b = slots[0]
        else:
            fm = FlowMerge(p, mg, cap, n, nbuf=nbuf)
            fm.gidx = gidx
            om = OverlappedMerge(fm, nbuf=nbuf) if mode == "overlap" else None
            steps = 3 if om else 1
            for i in range(steps):
                k = i % nbuf
                b = slots[k]
                if om:
                    om.acquire(k)
                b["ctr"].zero_()
                p.reset_flows(stream=s, sync=False)
                p.parse_device(arena, alen, off, ln, ts, m, b["rec"], m, b["hash"], b["id"],
                               b["n"], b["ctr"], stream=s, filter_port=filter_port,
                               out_frame=b["frame"])
                if om:
                    om.submit(k, b["id"], b["n"], m, ctr=b["ctr"])
                else:
                    fm.step(b["id"], b["n"], m, stream=s, rec_frame=b["frame"])
                    dist.all_reduce(b["ctr"])
            torch.cuda.synchronize()
            status = p.status()
            merged = mg.flows()
            b = slots[(steps - 1) % nbuf]
        k = int(b["n"].item())
        np.savez(os.path.join(result_dir, f"rank{rank}.npz"),
                 gidx=(gidx.cpu().numpy() if gidx is not None else np.zeros(0, np.int64)),
                 rec=b["rec"][:k * 74].cpu().numpy().reshape(-1, 74),
                 gids=b["id"][:k].cpu().numpy().view(np.uint32),
                 ctr=b["ctr"].cpu().numpy(), merged=merged.view(np.uint8),
                 status=np.array([status]))
    dist.barrier()
    dist.destroy_process_group()


def run_gpu_windows(rank, world, port, n, n_flows, bounds, cap, map_cap, result_dir,
                    filter_port=0, default_stream=False):
    """FlowHashExchange over a STREAM of windows: global frames [bounds[w],
    bounds[w+1]) form window w; each rank parses its flow-hash shard's frames inside
    it as one batch, keeping its flow table and id map (no reset between windows).
    Saves the concatenated records / global ids / global frame indices, the summed
    counters and the local flow table with each flow's global id.
    default_stream: torch's DEFAULT stream throughout (no set_stream; the step is
    handed stream 0), the inputs of each window uploaded and the outputs read on it
    (the exchange must order its collectives itself)."""
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if not default_stream:
        torch.cuda.set_stream(torch.cuda.Stream())
    import tcbee_amd
    from tcbee_amd import host
    from tcbee_amd.dist import FlowHashExchange
    from tracegen import mixed_trace

    tr = mixed_trace(n, seed=404, n_flows=n_flows)
    mine = np.nonzero(host.flowhash_owner(tr, world) == rank)[0].astype(np.int64)
    arena = torch.zeros(len(tr.arena) + 64, dtype=torch.uint8, device="cuda")
    arena[:len(tr.arena)] = torch.from_numpy(tr.arena).cuda()
    wmax = max(int(((mine >= a) & (mine < b)).sum()) for a, b in zip(bounds, bounds[1:]))
    rec = torch.empty(max(wmax, 1) * 74 + 64, dtype=torch.uint8, device="cuda")
    hsh = torch.empty(max(wmax, 1), dtype=torch.int32, device="cuda")
    ids = torch.empty(max(wmax, 1), dtype=torch.int32, device="cuda")
    frame = torch.empty(max(wmax, 1), dtype=torch.int32, device="cuda")
    nrec = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert (s == 0) == default_stream
    out_rec, out_ids, out_g, tot = [], [], [], np.zeros(4, np.int64)
    with tcbee_amd.PacketParser(max_frames=max(wmax, 1), max_flows=map_cap) as p:
        fx = None
        for a, b in zip(bounds, bounds[1:]):
            g = mine[(mine >= a) & (mine < b)]
            sub = tr.select(g)
            off = torch.from_numpy(sub.offset.view(np.int64)).cuda()
            ln = torch.from_numpy(sub.caplen.view(np.int32)).cuda()
            ts = torch.from_numpy(sub.ts_ns.view(np.int64)).cuda()
            gidx = torch.from_numpy(g).cuda()
            if fx is None:
                fx = FlowHashExchange(p, cap, gidx, map_cap=map_cap)
            ctr.zero_()
            fx.step(arena, len(tr.arena), off, ln, ts, len(g), rec, len(g), hsh, ids, nrec, ctr,
                    s, filter_port=filter_port, rec_frame=frame, gidx=gidx)
            dist.all_reduce(ctr)
            torch.cuda.synchronize()
            k = int(nrec.item())
            out_rec.append(rec[:k * 74].cpu().numpy().reshape(-1, 74))
            out_ids.append(ids[:k].cpu().numpy().view(np.uint32))
            out_g.append(g[frame[:k].cpu().numpy().astype(np.int64)])
            tot += ctr.cpu().numpy()
        status = p.status()
        flows = p.flows()
        gmap = fx.gmap[:len(flows)].cpu().numpy().view(np.uint32)
        gtot = int(fx.gtot[fx.windows & 1].item())
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), rec=np.concatenate(out_rec),
             gids=np.concatenate(out_ids), gidx=np.concatenate(out_g), ctr=tot,
             flows=flows.view(np.uint8), gmap=gmap, gtot=np.array([gtot]),
             status=np.array([status]))
    dist.barrier()
    dist.destroy_process_group()


def run_replay(rank, world, port, pcap, prefix, db_path, filter_port, direction, result_dir):
    """replay_pcap_sharded on `world` gloo ranks sharing device 0."""
    import json

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tcbee_amd.dist import replay_pcap_sharded
    out = replay_pcap_sharded(pcap, prefix, direction=direction, filter_port=filter_port,
                              db_path=db_path, chunk_frames=4096, threads=2)
    with open(os.path.join(result_dir, f"rank{rank}.json"), "w") as f:
        json.dump({k: v for k, v in out.items() if k != "sink"}, f)
    dist.destroy_process_group()


def run_shard_check(rank, world, port, n, n_flows, result_dir, corrupt):
    """bench.validate_shard_global (the N>1 line's per-rank full check) on CPU tensors
    over gloo: each rank's flow-hash shard of a synthetic trace, its "device" outputs
    taken from the oracle run over the WHOLE trace (records, hashes, global ids) and
    the merged table = the oracle's global table. corrupt: "" (all exact), "id" (one
    global id changed on rank 1), "row" (one merged-table row's pkts changed) or
    "record" (one record byte on rank 0)."""
    import json

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import tcbee_amd
    from oracle_py import Oracle
    from tcbee_amd import host

    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=n_flows, seed=1234)
    rec, fh, fi, _, table = Oracle().parse(tr)
    g = np.nonzero(host.flowhash_owner(tr, world) == rank)[0].astype(np.int64)
    sub = tr.select(g)
    arena = torch.from_numpy(np.concatenate([sub.arena, np.zeros(64, np.uint8)]))
    d_rec = torch.from_numpy(rec[g].reshape(-1).copy())
    d_hash = torch.from_numpy(fh[g].view(np.int32).copy())
    d_id = torch.from_numpy(fi[g].view(np.int32).copy())
    merged = table.copy()
    if corrupt == "id" and rank == 1:
        d_id[len(g) // 2] += 1
    if corrupt == "row":
        merged["pkts"][len(merged) // 3] += 1
    if corrupt == "record" and rank == 0:
        d_rec[74 * 5 + 40] ^= 1
    out = bench.validate_shard_global(
        torch, dist, arena, torch.from_numpy(sub.offset.view(np.int64)),
        torch.from_numpy(sub.caplen.view(np.int32)), torch.from_numpy(sub.ts_ns.view(np.int64)),
        d_rec, d_hash, d_id, torch.from_numpy(g), len(g), len(g), merged, chunk=7000)
    with open(os.path.join(result_dir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
