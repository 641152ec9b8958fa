"""Multi-rank path on CPU: world-size-2 gloo run of the shard + table-exchange
choreography (tcbee_amd.dist) against the oracle on the unsharded trace."""
import os

import numpy as np
import pytest


from ports import free_port  # noqa: E402


def test_shard_range_covers_everything():
    from tcbee_amd.dist import shard_range
    for n in (0, 1, 7, 1000, 12345):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))


def test_reference_merge_equals_unsharded(oracle):
    from merge_ref import merge
    from tracegen import mixed_trace
    tr = mixed_trace(30_000, seed=8, n_flows=900)
    full = oracle.parse(tr)
    tables, recs, ids = [], [], []
    cuts = [0, 7000, 7001, 19000, 30000]
    for lo, hi in zip(cuts, cuts[1:]):
        r = oracle.parse(tr.slice(lo, hi))
        tables.append(r[4])
        recs.append(len(r[0]))
        ids.append(r[2])
    merged, maps = merge(tables, recs)
    assert np.array_equal(merged, full[4])
    gids = np.concatenate([m[i] for m, i in zip(maps, ids)])
    assert np.array_equal(gids, full[2])


def test_gloo_world2_choreography(oracle, tmp_path):
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    n, cap, world = 40_000, 2048, 2
    mp.spawn(dist_worker.run, args=(world, free_port(), n, cap, str(tmp_path)), nprocs=world,
             join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    full = oracle.parse(tr)
    from tcbee_amd.parser import FLOW_DTYPE
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for r in res:
        assert np.array_equal(r["merged"].view(FLOW_DTYPE), full[4])
    gids = np.concatenate([r["gids"] for r in res])
    assert np.array_equal(gids, full[2])


@pytest.mark.parametrize("filter_port", [0, 5201])
def test_gloo_world2_flowhash_real_trace(oracle, tmp_path, filter_port):
    """Flow-hash partition of a trace with rejected and filtered frames: global
    ids and the merged table (first_seen = global record index) vs the oracle on
    the whole trace (the algorithm tcbee_amd.dist runs on the device)."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, cap, world = 40_000, 2048, 2
    mp.spawn(dist_worker.run_flowhash, args=(world, free_port(), n, cap, str(tmp_path),
                                             filter_port), nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    rec, fh, fi, ctr, table = oracle.parse(tr, filter_port=filter_port)
    acc = oracle.accept_mask(tr, filter_port=filter_port)
    recidx = np.cumsum(acc) - 1
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for x in res:
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        g = x["gidx"]
        ri = recidx[g[acc[g]]]
        assert np.array_equal(x["rec"], rec[ri]) and np.array_equal(x["gids"], fi[ri])


def test_flowhash_owner_matches_key_hash(oracle):
    """The host partitioner keys frames exactly as the hook does (fixed offsets,
    xdp.rs:37-127) and routes keyless frames round robin."""
    from tracegen import mixed_trace
    from tcbee_amd import host
    tr = mixed_trace(6000, seed=77, n_flows=300)
    for world in (1, 2, 3, 8):
        own = host.flowhash_owner(tr, world, threads=3)
        for i in range(tr.n):
            _, key = oracle.hook(tr.frame(i))
            if key is None:
                # runts and non-TCP frames: round robin (a runt with a keyable prefix
                # never reaches here: the hook and the partitioner share the bounds)
                assert own[i] == i % world
            else:
                h = oracle.flow_hash64(key)
                assert own[i] == ((h ^ (h >> 32)) & 0xFFFFFFFF) % world


def test_flowhash_owner_matches_device_shards():
    """On the synthetic trace the partitioner reproduces the device shard
    generator's placement (fold32(flow_hash64) % world: tcbee_gen_shard_index_device)."""
    import tcbee_amd
    from tcbee_amd import host
    tr = tcbee_amd.synth_trace(20_000, sizes="imix", kind=1, n_flows=3000)
    orc_hash = tcbee_amd.parser.flow_hash64
    own = host.flowhash_owner(tr, 4)
    for i in range(0, tr.n, 97):
        f = tr.frame(i)
        key = bytes(12) + f[26:30] + bytes(12) + f[30:34] + f[34:36][::-1] + f[36:38][::-1] \
            + bytes([6, 0, 0, 0])
        h = orc_hash(key)
        assert own[i] == ((h ^ (h >> 32)) & 0xFFFFFFFF) % 4


def test_rss_flows_per_rank_matches_the_trace(oracle):
    """bench.py sizes flow-hash shards from tcbee_amd.rss_flows_per_rank before any
    frame is parsed: every flow's fold32(flow_hash64(key)) computed from its flow
    number (synth_flow_folds) equals the oracle's hash of the key the hook builds
    from that flow's frames, and the per-rank counts equal the distinct flows of
    each host partitioner shard (modulo placement and an RSS table)."""
    import tcbee_amd
    from tcbee_amd import host
    n_flows = 3000
    tr = tcbee_amd.synth_trace(60_000, sizes="imix", kind=1, n_flows=n_flows)
    folds = set(tcbee_amd.synth_flow_folds(n_flows).tolist())
    keys = {}
    for i in range(0, tr.n, 7):
        _, key = oracle.hook(tr.frame(i))
        h = oracle.flow_hash64(key)
        keys[key] = (h ^ (h >> 32)) & 0xFFFFFFFF
    assert len(keys) > 2700 and set(keys.values()) <= folds
    rng = np.random.default_rng(5)
    table = rng.integers(0, 3, size=tcbee_amd.RSS_BUCKETS).astype(np.uint16)
    all_keys = [oracle.hook(tr.frame(i))[1] for i in range(tr.n)]
    for world, tab in ((4, None), (3, table)):
        per = tcbee_amd.rss_flows_per_rank(n_flows, world, table=tab)
        assert per.sum() == n_flows
        own = host.flowhash_owner(tr, world, threads=2, rss=tab)
        for r in range(world):
            # 60k frames of 3000 uniform flows: every flow appears
            assert len({k for k, o in zip(all_keys, own) if o == r}) == per[r]


def test_rss_table_lpt():
    """rss_table: every bucket mapped to a GPU < world, deterministic, and the
    per-GPU load within one bucket of the mean (longest-processing-time greedy)."""
    import tcbee_amd
    rng = np.random.default_rng(3)
    for world in (2, 3, 8):
        load = rng.poisson(rng.integers(0, 4, 4096) * 2000)
        t = tcbee_amd.rss_table(load, world)
        assert t.dtype == np.uint16 and len(t) == 4096 and int(t.max()) < world
        assert np.array_equal(t, tcbee_amd.rss_table(load, world))
        per = np.bincount(t, weights=load, minlength=world)
        assert per.max() - per.mean() <= load.max()
        assert per.max() / per.mean() < 1.001
    with pytest.raises(ValueError):
        tcbee_amd.rss_table([], 2)
    import torch
    bad = torch.from_numpy(np.array([0, 1, 2], dtype=np.uint16).view(np.int16))
    with pytest.raises(ValueError):  # an entry >= world would drop its bucket's frames
        tcbee_amd.gen_shard_index_device(10, 2, 0, 1, 5, 1, True, None, None, 0, None, None,
                                         rss=bad)


def test_flowhash_owner_rss_and_load(oracle):
    """The host partitioner with an RSS table: keyed frames go to
    table[fold32(hash) % len] (unkeyed round robin, as without a table); the bucket
    loads count the keyed frames per bucket; a table balanced on them evens out the
    GPUs' frame counts on a synthetic trace; bad tables are refused."""
    import tcbee_amd
    from tcbee_amd import host
    from tracegen import mixed_trace
    tr = mixed_trace(30_000, seed=11, n_flows=700)
    fold = np.full(tr.n, -1, dtype=np.int64)
    for i in range(tr.n):
        key = oracle.hook(tr.frame(i))[1]
        if key is not None:
            h = oracle.flow_hash64(key)
            fold[i] = (h ^ (h >> 32)) & 0xFFFFFFFF
    keyed = fold >= 0
    load = host.flowhash_load(tr, 512, threads=3)
    assert np.array_equal(load, np.bincount(fold[keyed] % 512, minlength=512))
    table = tcbee_amd.rss_table(load, 3)
    own = host.flowhash_owner(tr, 3, threads=4, rss=table)
    assert np.array_equal(own[keyed], table[fold[keyed] % 512])
    assert np.array_equal(own[~keyed], (np.arange(tr.n) % 3)[~keyed])
    syn = tcbee_amd.synth_trace(200_000, sizes="imix", kind=1, n_flows=2000)
    t8 = tcbee_amd.rss_table(host.flowhash_load(syn, 4096), 8)
    per = np.bincount(host.flowhash_owner(syn, 8, rss=t8), minlength=8)
    per_mod = np.bincount(host.flowhash_owner(syn, 8), minlength=8)
    assert per.max() / per.mean() < 1.002 < per_mod.max() / per_mod.mean()
    with pytest.raises(tcbee_amd.TcbeeError):
        host.flowhash_owner(tr, 2, rss=np.array([0, 1, 2], dtype=np.uint16))  # entry >= world
    with pytest.raises(tcbee_amd.TcbeeError):
        host.flowhash_load(tr, 4097)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_owner_exchange_mirror(oracle, tmp_path, world):
    """The owner exchange's algorithm (contiguous shards, flows merged at their hash
    owner, ids by the owners' first_seen arrays, returned by all-to-all) on CPU
    ranks over gloo: the global ids equal the unsharded oracle's."""
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    n, cap = 40_000, 2048
    mp.spawn(dist_worker.run_owner, args=(world, free_port(), n, cap, str(tmp_path), 5201),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    fi = oracle.parse(tr, filter_port=5201)[2]
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert np.array_equal(np.concatenate([x["gids"] for x in res]), fi)


@pytest.mark.parametrize("corrupt", ["", "id", "row", "record"])
def test_bench_shard_full_check_over_gloo(tmp_path, corrupt):
    """The N>1 bench line's per-rank full check (bench.validate_shard_global, VERDICT
    r5 #2) at world 2 over gloo on CPU tensors: exact inputs pass on every rank
    (records, hashes, global ids from the host recomputation of global first-seen
    order, the rank's rows of the merged table); one changed global id, merged-table
    row or record byte is caught on the rank that holds it."""
    import json

    import torch.multiprocessing as mp

    import dist_worker
    world = 2
    mp.spawn(dist_worker.run_shard_check, args=(world, free_port(), 30_000, 1500,
                                                str(tmp_path), corrupt),
             nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for r, x in enumerate(res):
        assert x["full_records"] > 10_000 and x["flows_global_recomputed"] == 1500
        bad_id = corrupt == "id" and r == 1
        bad_rec = corrupt == "record" and r == 0
        assert x["records_hashes_exact"] is (not bad_rec)
        assert x["global_ids_exact"] is (not (bad_id or bad_rec))
        assert x["full_bit_exact"] is (not (bad_id or bad_rec))
        assert x["merged_rows_exact"] is (corrupt != "row" or x["merged_rows_exact"])
    if corrupt == "row":  # the changed row belongs to exactly one rank
        assert sorted(x["merged_rows_exact"] for x in res) == [False, True]
    elif corrupt in ("", "id", "record"):
        assert all(x["merged_rows_exact"] for x in res)
