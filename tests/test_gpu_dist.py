"""The N>1 path on the GPU (tcbee_amd.dist): world-size-2 gloo ranks sharing
device 0 run the device export -> all-gather -> tcbee_flow_merge_device ->
remap choreography, on one stream (FlowMerge.step) and overlapped with the
next step's parse on a side stream (OverlappedMerge, as bench.py). Records,
global flow ids, global counters and the merged table vs the oracle on the
unsharded trace."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


from ports import free_port  # noqa: E402


@pytest.mark.parametrize("mode", ["step", "overlap", "owner"])
def test_gpu_world2_merge(gpu, oracle, tmp_path, mode):
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, cap, world = 60_000, 2048, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), mode, 700),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert np.array_equal(np.concatenate([r["rec"] for r in res]), rec)
    assert np.array_equal(np.concatenate([r["gids"] for r in res]), fi)
    for r in res:
        assert np.array_equal(r["merged"].view(FLOW_DTYPE), table)
        assert int(r["ctr"][0]) == ctr["ingress"] and int(r["ctr"][2]) == ctr["handled"]


@pytest.mark.parametrize("mode", ["flowhash", "flowhash_rss", "fhx_rss"])
def test_gpu_world2_flowhash_shards(gpu, oracle, tmp_path, mode):
    """Flow-hash shards (config 4's NIC-RSS view): each rank's frames are the
    global frames whose flow hash % world is its rank (device shard generator) —
    or, with an RSS indirection table balanced on the bucket loads (the bench's
    N>1 placement), whose table entry is its rank; records, global flow ids and the
    merged table vs the oracle over the global trace, and the shards partition the
    trace."""
    import torch.multiprocessing as mp

    import dist_worker
    import tcbee_amd
    from tcbee_amd import host
    from tcbee_amd.parser import FLOW_DTYPE
    n, cap, world = 120_000, 4096, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), mode),
             nprocs=world, join=True)
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=3000)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    owner = fh % world
    if mode != "flowhash":
        import torch

        import bench
        rss = np.load(tmp_path / "rss0.npy")
        assert np.array_equal(rss, np.load(tmp_path / "rss1.npy"))  # one table on every rank
        # the table is the LPT balance of the device's bucket loads over the held-out
        # window after the trace (bench.rss_for; the device load equals the host
        # partitioner's: test_rss_load_range_matches_host); the host placement with
        # that table agrees frame by frame
        counts = torch.empty(len(rss), dtype=torch.int64, device="cuda")
        tcbee_amd.gen_rss_load_device(bench.RSS_WINDOW, 1, 3000, tcbee_amd.trace.DEFAULT_SEED,
                                      counts, first_frame=n)
        assert np.array_equal(rss, tcbee_amd.rss_table(counts.cpu().numpy(), world))
        owner = rss[fh % len(rss)]
        assert np.array_equal(host.flowhash_owner(tr, world, rss=rss), owner)
        per = np.bincount(owner, minlength=world)
        assert per.max() / per.mean() < 1.01  # balanced (modulo: 3000 flows spread ~2 %)
    all_g = np.concatenate([r["gidx"] for r in res])
    assert len(all_g) == n and np.array_equal(np.sort(all_g), np.arange(n))
    for r, x in enumerate(res):
        g = x["gidx"]
        assert np.array_equal(g, np.nonzero(owner == r)[0])
        assert np.array_equal(x["rec"], rec[g])
        assert np.array_equal(x["gids"], fi[g])
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"]


@pytest.mark.parametrize("exchange", ["flowhash", "fhx"])
def test_gpu_world2_flowhash_200k_flows(gpu, oracle, tmp_path, exchange):
    """the flow-hash partition at >= 200k flows (each rank's table
    ~125k flows, K3's bucketed large-table mode, the records-before first_seen
    fix-up over 600k global frames)."""
    import torch.multiprocessing as mp

    import dist_worker
    import tcbee_amd
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, world = 600_000, 250_000, 2
    cap = int(1.25 * flows / world) + 4096
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), exchange,
                                        flows), nprocs=world, join=True)
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=flows)
    ft = oracle.new_flowtab(1 << 19)
    try:
        rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
        table = oracle.flows(ft)
    finally:
        oracle.free_flowtab(ft)
    assert len(table) > 200_000
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    owner = fh % world
    for r, x in enumerate(res):
        g = x["gidx"]
        assert np.array_equal(g, np.nonzero(owner == r)[0])
        assert np.array_equal(x["rec"], rec[g])
        assert np.array_equal(x["gids"], fi[g])
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"] and int(x["status"][0]) == 0


@pytest.mark.parametrize("exchange", ["flowhash_real", "fhx_real"])
@pytest.mark.parametrize("filter_port", [0, 5201])
def test_gpu_world2_flowhash_real_trace(gpu, oracle, tmp_path, filter_port, exchange):
    """VERDICT r1 #2 / ADVICE r1: flow-hash shards of a REAL trace (non-TCP frames,
    runts, IPv6, v4-compatible collisions, FILTER_PORT) — record k of a rank is not
    its frame k. The host partitioner (the NIC-RSS step) splits the trace; each
    rank's parse writes its record -> frame map, the export places every flow at
    its global frame, and the merged first_seen is the global record index.
    Records, global ids, counters and the merged table vs the oracle over the
    whole trace."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, cap, world = 200_000, 5000, 8192, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path),
                                        exchange, flows, filter_port),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=filter_port)
    acc = oracle.accept_mask(tr, filter_port=filter_port)
    recidx = np.cumsum(acc) - 1
    assert acc.sum() == len(rec) and acc.sum() < n
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    got = np.concatenate([x["gidx"] for x in res])
    assert np.array_equal(np.sort(got), np.arange(n))  # the shards partition the trace
    for x in res:
        g = x["gidx"]
        ri = recidx[g[acc[g]]]
        assert np.array_equal(x["rec"], rec[ri])
        assert np.array_equal(x["gids"], fi[ri])
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"] and int(x["ctr"][2]) == ctr["handled"]
        assert int(x["status"][0]) == 0


def test_gpu_world2_flowhash_without_frame_map_is_refused(gpu, tmp_path):
    """A shard with rejected frames exported WITHOUT the record -> frame map cannot
    be placed in the global trace: the local context reports TCBEE_ESHARD instead
    of silently merging wrong first-seen order."""
    import torch.multiprocessing as mp

    import dist_worker
    from tcbee_amd import _lib
    n, flows, cap, world = 30_000, 500, 2048, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path),
                                        "flowhash_noframe", flows), nprocs=world, join=True)
    for r in range(world):
        assert int(np.load(tmp_path / f"rank{r}.npz")["status"][0]) == _lib.ESHARD


@pytest.mark.parametrize("mode", ["overlap", "flowhash_real", "fhx_real"])
def test_gpu_rccl_world1_exchange(gpu, oracle, tmp_path, mode):
    """The RCCL branch of the exchange (all_gather_into_tensor + all_reduce on the
    `nccl` backend, i.e. RCCL) on this one-GPU box: world 1, since RCCL refuses two
    ranks on one device ("Duplicate GPU detected"). Same checks as world 2."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, cap = 60_000, 700, 2048
    fp = 5201 if mode.endswith("_real") else 0
    mp.spawn(dist_worker.run_gpu, args=(1, free_port(), n, cap, str(tmp_path), mode, flows,
                                        fp, "nccl"),
             nprocs=1, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=fp)
    x = np.load(tmp_path / "rank0.npz")
    assert np.array_equal(x["rec"], rec) and np.array_equal(x["gids"], fi)
    assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
    assert int(x["ctr"][0]) == ctr["ingress"] and int(x["status"][0]) == 0


def test_gpu_world4_flowhash_exchange_real_trace(gpu, oracle, tmp_path):
    """Four gloo ranks on device 0: the flow-hash exchange's binary searches over
    three other ranks' first-frame arrays, a real mixed trace with FILTER_PORT."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, cap, world = 120_000, 3000, 4096, 4
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), "fhx_real",
                                        flows, 5201), nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=5201)
    acc = oracle.accept_mask(tr, filter_port=5201)
    recidx = np.cumsum(acc) - 1
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert np.array_equal(np.sort(np.concatenate([x["gidx"] for x in res])), np.arange(n))
    for x in res:
        g = x["gidx"]
        ri = recidx[g[acc[g]]]
        assert np.array_equal(x["rec"], rec[ri]) and np.array_equal(x["gids"], fi[ri])
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"] and int(x["status"][0]) == 0


@pytest.mark.parametrize("filter_port,stream", [(0, "own"), (5201, "own"), (0, "default"),
                                                (5201, "default")])
def test_gpu_world2_flowhash_exchange_windows(gpu, oracle, tmp_path, filter_port, stream):
    """A stream of windows through the flow-hash exchange (the tables are NOT reset
    between windows): flows keep their global ids across windows and new ones get
    the ids one parse of the whole trace gives. Ragged windows, one holding a single
    frame (so one rank parses an empty batch). Records, global ids, counters, and
    each rank's table rows (pkts/bytes/tuple at their global ids) vs the oracle.
    stream "default" (VERDICT r5 #1): no torch.cuda.set_stream, the step gets torch's
    default stream (handle 0) and every window's inputs, outputs and the counter
    all-reduce live on it — the exchange itself must put its device calls and its
    collectives on one stream (dist.rank_stream); each window's data differs, so a
    collective that read a buffer before its kernel wrote it would show."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, world = 150_000, 4000, 2
    bounds = [0, 3, 41_000, 41_001, 97_000, n]
    mp.spawn(dist_worker.run_gpu_windows, args=(world, free_port(), n, flows, bounds, 4096,
                                                8192, str(tmp_path), filter_port,
                                                stream == "default"),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=filter_port)
    acc = oracle.accept_mask(tr, filter_port=filter_port)
    recidx = np.cumsum(acc) - 1
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    seen = np.zeros(len(table), dtype=np.int64)
    for x in res:
        ri = recidx[x["gidx"]]
        assert np.array_equal(x["rec"], rec[ri]) and np.array_equal(x["gids"], fi[ri])
        assert int(x["ctr"][0]) == ctr["ingress"] and int(x["ctr"][2]) == ctr["handled"]
        assert int(x["status"][0]) == 0 and int(x["gtot"][0]) == len(table)
        loc = x["flows"].view(FLOW_DTYPE)
        gm = x["gmap"].astype(np.int64)
        assert np.array_equal(loc["tuple"], table["tuple"][gm])
        assert np.array_equal(loc["pkts"], table["pkts"][gm])
        assert np.array_equal(loc["bytes"], table["bytes"][gm])
        seen[gm] += 1
    assert (seen == 1).all()  # the ranks' tables partition the global one


def test_gpu_world2_flowhash_exchange_window_over_cap(gpu, tmp_path):
    """More new flows in one window than the exchange's per-rank capacity: every
    write stays inside its buffer and the context reports TCBEE_ESHARD."""
    import torch.multiprocessing as mp

    import dist_worker
    from tcbee_amd import _lib
    n, flows, world = 20_000, 1000, 2
    mp.spawn(dist_worker.run_gpu_windows, args=(world, free_port(), n, flows, [0, 5000, n], 64,
                                                4096, str(tmp_path), 0),
             nprocs=world, join=True)
    for r in range(world):
        assert int(np.load(tmp_path / f"rank{r}.npz")["status"][0]) == _lib.ESHARD


@pytest.mark.parametrize("world", [3, 4])
@pytest.mark.parametrize("filter_port", [0, 5201])
def test_gpu_owner_exchange_contiguous_real_trace(gpu, oracle, tmp_path, world, filter_port):
    """The owner exchange over contiguous shards of a real mixed trace (rejected and
    port-filtered frames, flows spanning every shard): records, global ids,
    counters and the merged table vs the oracle over the whole trace."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, flows, cap = 90_000, 3000, 8192
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), "owner",
                                        flows, filter_port), nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=filter_port)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert np.array_equal(np.concatenate([x["rec"] for x in res]), rec)
    assert np.array_equal(np.concatenate([x["gids"] for x in res]), fi)
    for x in res:
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"] and int(x["status"][0]) == 0


def test_gpu_owner_exchange_map_overflow_is_refused(gpu, tmp_path):
    """Ranks with more flows than their id maps hold (~5.5k local flows each, maps of
    4096): the flows past the map are not exchanged and every context reports
    TCBEE_ESHARD (no silent garbage ids)."""
    import torch.multiprocessing as mp

    import dist_worker
    from tcbee_amd import _lib
    n, flows, cap, world = 90_000, 3000, 8192, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), "owner",
                                        flows, 0, "gloo", [4096, 4096]), nprocs=world, join=True)
    for r in range(world):
        assert int(np.load(tmp_path / f"rank{r}.npz")["status"][0]) == _lib.ESHARD


def test_gpu_owner_exchange_one_rank_overflows(gpu, tmp_path):
    """Only rank 1's id map is too small: its dropped flows take no
    segment slot (no phantom flow reaches an owner), and rank 0 — whose own table
    fits — reports TCBEE_ESHARD too, since its global ids would be shifted."""
    import torch.multiprocessing as mp

    import dist_worker
    from tcbee_amd import _lib
    n, flows, cap, world = 90_000, 3000, 8192, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), "owner",
                                        flows, 0, "gloo", [cap, 1000]), nprocs=world, join=True)
    for r in range(world):
        assert int(np.load(tmp_path / f"rank{r}.npz")["status"][0]) == _lib.ESHARD, r


@pytest.mark.parametrize("world,filter_port,direction", [(2, 0, 0), (3, 5201, 1)])
def test_gpu_replay_pcap_sharded(gpu, oracle, tmp_path, world, filter_port, direction):
    """A pcap replayed over `world` ranks (contiguous shards, one pipeline each):
    the one .tcp file, the counters in metrics.json and the tcbee-process database
    equal the oracle path over the whole capture."""
    import json
    import os
    import sys

    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "oracle"))
    import process_ref  # test infrastructure only
    from tcbee_amd import host
    t = mixed_trace(40_000, seed=77, n_flows=60)
    pcap = str(tmp_path / "trace.pcap")
    host.write_pcap(pcap, t)
    prefix = str(tmp_path) + "/run_"
    db = str(tmp_path / "gpu.sqlite")
    mp.spawn(dist_worker.run_replay, args=(world, free_port(), pcap, prefix, db, filter_port,
                                           direction, str(tmp_path)), nprocs=world, join=True)
    rec, fh, fi, ctr, table = oracle.parse(t, filter_port=filter_port, direction=direction)
    name = "tc.tcp" if direction else "xdp.tcp"
    assert open(prefix + name, "rb").read() == rec.tobytes()
    out = json.load(open(tmp_path / "rank0.json"))
    assert out["records"] == len(rec) and out["counters"] == ctr and out["frames"] == t.n
    m = json.load(open(prefix + "metrics.json"))
    assert {k: m[k] for k in ("handled", "dropped", "ingress", "egress")} == ctr
    process_ref.process_records(rec.tobytes(), str(tmp_path / "orc.sqlite"))
    assert process_ref.dump_db(db) == process_ref.dump_db(str(tmp_path / "orc.sqlite"))


@pytest.mark.parametrize("first", [0, 120_000, 7_777_777])
def test_rss_load_range_matches_host(gpu, first):
    """tcbee_gen_rss_load_range_device over global frames [first, first + m) (the
    held-out window bench.rss_for balances on) == the host partitioner's bucket
    loads of the same frames generated on the host."""
    import torch

    import tcbee_amd
    from tcbee_amd import host
    m, nf = 150_000, 3000
    tr = tcbee_amd.synth_trace(m, sizes="imix", kind=1, n_flows=nf, first_index=first)
    counts = torch.empty(4096, dtype=torch.int64, device="cuda")
    tcbee_amd.gen_rss_load_device(m, 1, nf, tcbee_amd.trace.DEFAULT_SEED, counts,
                                  first_frame=first)
    assert np.array_equal(counts.cpu().numpy().astype(np.uint64), host.flowhash_load(tr, 4096))


def test_rss_table_refused_on_device(gpu):
    """an RSS table with an entry >= world reaching the C entry point
    directly (the Python wrapper refuses it earlier) gives the count
    TCBEE_RSS_INVALID (~0) instead of silently dropping that bucket's frames; the
    wrapper refuses tables that are not contiguous int16/uint16 device tensors."""
    import ctypes as C

    import torch

    import tcbee_amd
    from tcbee_amd import _lib
    n, world = 50_000, 2
    scratch = torch.empty(tcbee_amd.gen_shard_scratch_words(n), dtype=torch.int64, device="cuda")
    n_out = torch.zeros(1, dtype=torch.int64, device="cuda")
    for bad_at, want_bad in [(None, False), (4095, True), (0, True)]:
        rss = torch.zeros(4096, dtype=torch.int16, device="cuda")
        rss[1::2] = 1
        if bad_at is not None:
            rss[bad_at] = world
        _lib.check(_lib.lib().tcbee_gen_shard_index_rss_device(
            C.c_uint64(n), world, 0, 1, C.c_uint64(500), C.c_uint64(7), 1, rss.data_ptr(),
            C.c_uint32(4096), None, None, C.c_uint64(0), scratch.data_ptr(), n_out.data_ptr(),
            None))
        torch.cuda.synchronize()
        got = int(n_out.item())
        assert (got == -1) == want_bad and (want_bad or 0 < got < n)
    for t in (torch.zeros(64, dtype=torch.int32, device="cuda"),
              torch.zeros(64, dtype=torch.int16),
              torch.zeros(128, dtype=torch.int16, device="cuda")[::2]):
        with pytest.raises(ValueError):
            tcbee_amd.gen_shard_index_device(n, world, 0, 1, 500, 7, True, None, None, 0,
                                             scratch, n_out, rss=t)
