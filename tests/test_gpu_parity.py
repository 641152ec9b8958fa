"""HIP path vs the CPU oracle, through the C ABI. Integer/byte work: bit-exact.

Every comparison covers the 74-B records, the per-record flow hash and dense
flow id, the counters (counters.rs) and the exported flow table.
"""
import json
import os

import numpy as np
import pytest

import tcbee_amd
from tcbee_amd.trace import Trace

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat_vectors.json")))["vectors"]


def assert_same(gpu_res, orc_res, gpu_flows=None):
    rec, fh, fi, ctr, table = orc_res
    assert gpu_res.n == len(rec)
    if len(rec):
        bad = np.nonzero(np.any(gpu_res.records != rec, axis=1))[0]
        assert len(bad) == 0, f"{len(bad)} records differ, first at {bad[:5]}: " \
            f"gpu {gpu_res.records[bad[0]].tobytes().hex()} oracle {rec[bad[0]].tobytes().hex()}"
    if gpu_res.flow_hash is not None:
        assert np.array_equal(gpu_res.flow_hash, fh)
        assert np.array_equal(gpu_res.flow_id, fi)
    assert gpu_res.counters == ctr
    if gpu_flows is not None and table is not None:
        assert len(gpu_flows) == len(table)
        assert np.array_equal(gpu_flows["tuple"], table["tuple"])
        assert np.array_equal(gpu_flows["pkts"], table["pkts"])
        assert np.array_equal(gpu_flows["bytes"], table["bytes"])
        assert np.array_equal(gpu_flows["first_seen"], table["first_seen"])


def test_kat_vectors_single_batch(parser, oracle):
    for port in sorted({v["filter_port"] for v in KAT}):
        vs = [v for v in KAT if v["filter_port"] == port]
        tr = Trace.from_frames([bytes.fromhex(v["frame"]) for v in vs],
                               ts_ns=[v["ts"] for v in vs])
        parser.reset_flows()
        res = parser.parse(tr, filter_port=port)
        exp = [bytes.fromhex(v["expect"]) for v in vs if v["expect"]]
        assert [r.tobytes() for r in res.records] == exp
        assert_same(res, oracle.parse(tr, filter_port=port), parser.flows())


@pytest.mark.parametrize("n", [1, 2, 63, 64, 255, 256, 257, 511, 512, 513, 1023, 1025, 4099])
def test_mixed_sizes(parser, oracle, n):
    from tracegen import mixed_trace
    tr = mixed_trace(n, seed=n)
    parser.reset_flows()
    assert_same(parser.parse(tr), oracle.parse(tr), parser.flows())


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("port", [0, 5201, 80])
@pytest.mark.parametrize("direction", [0, 1])
def test_mixed_large(parser, oracle, seed, port, direction):
    from tracegen import mixed_trace
    tr = mixed_trace(200_000, seed=seed, n_flows=3000)
    parser.reset_flows()
    res = parser.parse(tr, filter_port=port, direction=direction)
    assert_same(res, oracle.parse(tr, filter_port=port, direction=direction), parser.flows())
    assert parser.status() == 0


def test_no_flows_flag(parser, oracle):
    from tracegen import mixed_trace
    tr = mixed_trace(50_000, seed=9)
    parser.reset_flows()
    res = parser.parse(tr, flows=False)
    rec, _, _, ctr, _ = oracle.parse(tr, flows=False)
    assert np.array_equal(res.records, rec) and res.counters == ctr
    assert parser.flow_count() == 0


@pytest.mark.parametrize("cap", [0, 1, 100, 777])
def test_out_cap_drops(parser, oracle, cap):
    from tracegen import mixed_trace
    tr = mixed_trace(20_000, seed=4)
    parser.reset_flows()
    res = parser.parse(tr, out_cap=cap)
    orc = oracle.parse(tr, out_cap=cap)
    assert_same(res, orc, parser.flows())


def test_multi_batch_flow_ids_continue(parser, oracle):
    from tracegen import mixed_trace
    tr = mixed_trace(60_000, seed=21, n_flows=500)
    parser.reset_flows()
    ft = oracle.new_flowtab()
    base = 0
    try:
        for lo, hi in [(0, 10_000), (10_000, 10_000), (10_000, 33_333), (33_333, 60_000)]:
            part = tr.slice(lo, hi)
            res = parser.parse(part)
            orc = oracle.parse(part, ft=ft, record_base=base)
            assert_same(res, orc)
            base += len(orc[0])
        gf = parser.flows()
        of = oracle.flows(ft)
        assert np.array_equal(gf, of)
    finally:
        oracle.free_flowtab(ft)


def test_empty_batch(parser, oracle):
    parser.reset_flows()
    tr = Trace(np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
               np.zeros(0, np.uint64))
    res = parser.parse(tr)
    assert res.n == 0 and res.counters == {"ingress": 0, "egress": 0, "handled": 0,
                                           "dropped": 0}


def test_config2_1M_bit_exact(parser, oracle):
    tr = tcbee_amd.synth_trace(1_000_000, sizes="64")
    parser.reset_flows()
    res = parser.parse(tr)
    orc = oracle.parse(tr)
    assert_same(res, orc, parser.flows())
    fl = parser.flows()
    assert len(fl) == 1 and int(fl["pkts"][0]) == 1_000_000 and int(fl["first_seen"][0]) == 0


def test_k1_profiling_events(parser, oracle):
    """tcbee_ctx_profile (bench.py's live K1 timing): one event pair per
    K1 launch, timing-only events (no system-scope fence) whose durations are positive
    and fit inside the wall time of the synchronized calls; profiling changes no output,
    and a profile(False) context records nothing."""
    import time
    import torch
    tr = tcbee_amd.synth_trace(500_000, sizes="imix", kind=1, n_flows=2000)
    orc = oracle.parse(tr)
    parser.profile(False)
    assert parser.profile_read() == (0.0, 0)
    parser.profile(True)
    walls = []
    for _ in range(3):
        parser.reset_flows()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = parser.parse(tr)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        assert_same(res, orc, parser.flows())
    ms, k = parser.profile_read()
    parser.profile(False)
    assert k == 3
    assert 0.0 < ms <= sum(walls) * 1e3


def test_config3_imix_multiflow(parser, oracle):
    tr = tcbee_amd.synth_trace(300_000, sizes="imix", kind=1, n_flows=10_000)
    parser.reset_flows()
    assert_same(parser.parse(tr), oracle.parse(tr), parser.flows())


def test_config3_ipv6_multiflow(parser, oracle):
    """IPv6/TCP IMIX (kind 3): K1's IPv6 tail loads over a whole batch."""
    tr = tcbee_amd.synth_trace(300_000, sizes="imix6", kind=3, n_flows=10_000)
    parser.reset_flows()
    assert_same(parser.parse(tr), oracle.parse(tr), parser.flows())


def test_config3_zipf(parser, oracle):
    """Config 3's second run (Zipf s=1.1 flow mix): a hot head flow (~10 % of the
    records) and a long tail through the same kernels."""
    tr = tcbee_amd.synth_trace(300_000, sizes="imix", kind=2, n_flows=10_000)
    parser.reset_flows()
    assert_same(parser.parse(tr), oracle.parse(tr), parser.flows())


def test_device_generator_matches_host(gpu):
    import torch
    for sizes, kind, nf in [("64", 0, 1), ("imix", 1, 777), ("imix", 2, 10_000), ("64", 2, 1),
                            ("imix6", 3, 5000)]:
        n = 100_000
        off, ln, ts, alen = tcbee_amd.synth_index(n, sizes=sizes)
        host = tcbee_amd.synth_trace(n, sizes=sizes, kind=kind, n_flows=nf)
        d_arena = torch.zeros(alen + 16, dtype=torch.uint8, device="cuda")
        d_off = torch.from_numpy(off.view(np.int64)).cuda()
        d_len = torch.from_numpy(ln.view(np.int32)).cuda()
        tcbee_amd.gen_frames_device(d_arena, d_off, d_len, n, kind, nf, tcbee_amd.trace.DEFAULT_SEED)
        torch.cuda.synchronize()
        assert np.array_equal(d_arena[:alen].cpu().numpy(), host.arena)


def test_device_path_matches_host_path(parser, oracle):
    """parse_device on torch-allocated HBM buffers == host path == oracle."""
    import torch
    from tracegen import mixed_trace
    tr = mixed_trace(100_000, seed=33)
    n = tr.n
    d_arena = torch.from_numpy(tr.arena).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    d_rec = torch.empty(n * 74 + 16, dtype=torch.uint8, device="cuda")
    d_hash = torch.empty(n, dtype=torch.int32, device="cuda")
    d_id = torch.empty(n, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    parser.reset_flows()
    parser.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, d_rec, n, d_hash, d_id,
                        d_n, d_ctr)
    parser.sync()
    k = int(d_n.item())
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert k == len(rec)
    assert np.array_equal(d_rec[: k * 74].cpu().numpy().reshape(k, 74), rec)
    assert np.array_equal(d_hash[:k].cpu().numpy().view(np.uint32), fh)
    assert np.array_equal(d_id[:k].cpu().numpy().view(np.uint32), fi)
    c = d_ctr.cpu().numpy()
    assert dict(zip(["ingress", "egress", "handled", "dropped"], map(int, c))) == ctr


def test_arena_beyond_4GiB(parser, oracle):
    """Frames straddling and beyond the 4 GiB offset of a 4.3 GB device arena, the
    last frame ending exactly at arena_len: 64-bit offsets all the way through."""
    import torch
    from tracegen import mixed_trace
    tr = mixed_trace(40_000, seed=44, n_flows=700)
    base = (1 << 32) - 777  # the trace crosses the 4 GiB line
    alen = base + len(tr.arena)
    n = tr.n
    d_arena = torch.zeros(alen + 64, dtype=torch.uint8, device="cuda")
    d_arena[base:alen] = torch.from_numpy(tr.arena).cuda()
    d_off = torch.from_numpy((tr.offset + np.uint64(base)).view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    d_rec = torch.empty(n * 74 + 16, dtype=torch.uint8, device="cuda")
    d_hash = torch.empty(n, dtype=torch.int32, device="cuda")
    d_id = torch.empty(n, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    parser.reset_flows()
    parser.parse_device(d_arena, alen, d_off, d_len, d_ts, n, d_rec, n, d_hash, d_id, d_n, d_ctr)
    parser.sync()
    k = int(d_n.item())
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert k == len(rec)
    assert np.array_equal(d_rec[: k * 74].cpu().numpy().reshape(k, 74), rec)
    assert np.array_equal(d_hash[:k].cpu().numpy().view(np.uint32), fh)
    assert np.array_equal(d_id[:k].cpu().numpy().view(np.uint32), fi)
    assert np.array_equal(parser.flows(), table)
    del d_arena
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fpl", ["1", "2", "4"])
def test_tile_shape_determinism(gpu, oracle, fpl, monkeypatch):
    """Same trace, different frames-per-lane tilings -> identical outputs."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_FPL", fpl)
    tr = mixed_trace(150_000, seed=77, n_flows=2000)
    with tcbee_amd.PacketParser(max_frames=1 << 18, max_arena=1 << 26, max_flows=1 << 14,
                                variants=True) as p:
        assert_same(p.parse(tr), oracle.parse(tr), p.flows())


@pytest.mark.parametrize("every,fpl", [("1", "2"), ("3", "2"), ("64", "2"), ("3", "4")])
def test_lookback_recount_fallback(gpu, oracle, every, fpl, monkeypatch):
    """Tiles that never publish force successors to recount them from the input:
    results stay exact (the look-back assumes no dispatch order)."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_TEST_WITHHOLD", every)
    monkeypatch.setenv("TCBEE_FPL", fpl)
    tr = mixed_trace(20_000 if every == "1" else 60_000, seed=91, n_flows=300)
    with tcbee_amd.PacketParser(max_frames=1 << 17, max_arena=1 << 25, max_flows=1 << 12,
                                variants=True) as p:
        assert_same(p.parse(tr), oracle.parse(tr), p.flows())
        assert p.status() == 0


@pytest.mark.parametrize("mode", ["range", "bucket", "atomic"])
@pytest.mark.parametrize("n,flows", [(300_000, 30_000), (200_000, 13_000), (120_000, 100_000)])
def test_k3_large_table_modes(gpu, oracle, mode, n, flows, monkeypatch):
    """More flows than K3's LDS bins (12288): mode 3 (claim ranges, one LDS map +
    bins per range, where the grid has the XCD columns for it; else mode 1), mode 1
    (claims bucketed per block, per-bucket LDS histograms; TCBEE_TEST_K3_NORANGE)
    and mode 2 (device atomics, + TCBEE_TEST_K3_NOBUCKET) all exact, over two
    batches (claims of batch 1 looked up again in batch 2)."""
    from tracegen import mixed_trace
    if mode in ("bucket", "atomic"):
        monkeypatch.setenv("TCBEE_TEST_K3_NORANGE", "1")
    if mode == "atomic":
        monkeypatch.setenv("TCBEE_TEST_K3_NOBUCKET", "1")
    tr = mixed_trace(n, seed=97, n_flows=flows)
    cut = n // 3
    with tcbee_amd.PacketParser(max_frames=1 << 19, max_arena=1 << 28, max_flows=1 << 18,
                                variants=mode != "range") as p:
        r1 = p.parse(tr.slice(0, cut))
        r2 = p.parse(tr.slice(cut, n))
        rec, fh, fi, ctr, table = oracle.parse(tr)
        assert np.array_equal(np.concatenate([r1.records, r2.records]), rec)
        assert np.array_equal(np.concatenate([r1.flow_id, r2.flow_id]), fi)
        fl = p.flows()
        assert len(fl) == len(table) and np.array_equal(fl, table)
        assert p.status() == 0
        if mode != "range":
            assert p.count_mode() == (1 if mode == "bucket" else 2)


@pytest.mark.parametrize("nopack", ["0", "1"])
@pytest.mark.parametrize("flows", [1, 40, 5000, 20_000])
def test_k3_big_caplen_and_hot_flow(gpu, oracle, flows, nopack, monkeypatch):
    """caplen >= 64 KiB (counted by device atomics, outside the 40-bit LDS byte
    field) mixed with ordinary frames, and one hot flow (the wave-uniform add);
    K1->K3 scratch packed (claim + 14-bit caplen, escapes stored beside) or not."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_TEST_NOPACK", nopack)
    tr = mixed_trace(150_000, seed=101, n_flows=flows)
    rng = np.random.default_rng(5)
    big = rng.choice(tr.n, size=300, replace=False)
    pad = 2_600_000
    arena = np.concatenate([tr.arena, np.zeros(pad, np.uint8)])
    ln = tr.caplen.copy()
    # 16383+ overflows the packed K1->K3 caplen field; 65536+ leaves the LDS bins;
    # 2^20-1+ leaves the 20-bit caplen of a K3 mode-1 region entry (flows=20000)
    ln[big] = rng.integers(16_000, pad, size=len(big)).astype(np.uint32)
    tr2 = Trace(arena, tr.offset, ln, tr.ts_ns)
    with tcbee_amd.PacketParser(max_frames=1 << 18, max_arena=1 << 27, max_flows=1 << 16,
                                variants=nopack == "1") as p:
        assert_same(p.parse(tr2), oracle.parse(tr2), p.flows())
        assert p.status() == 0


@pytest.mark.parametrize("nopack", ["0", "1"])
def test_k3_mode1_long_caplens(gpu, oracle, nopack, monkeypatch):
    """K3 mode 1 (k_count_chunk2) with caplens around every field boundary: < 2047 (the
    region entry), 2047..16383 (round 6: the chunk sends their bytes to the flow's
    counter by a device atomic), 16383+ (past the packed K1 -> K3 field), 65536+ and
    2^20+; asserted to run in mode 1; records, ids and the table (pkts, bytes) exact."""
    monkeypatch.setenv("TCBEE_TEST_NOPACK", nopack)
    tr = tcbee_amd.synth_trace(400_000, sizes="imix", kind=1, n_flows=60_000, seed=2047)
    rng = np.random.default_rng(11)
    pad = 1_200_000
    arena = np.concatenate([tr.arena, np.zeros(pad, np.uint8)])
    ln = tr.caplen.copy()
    for lo, hi, k in ((2040, 2060, 400), (2047, 16_400, 800), (16_380, 70_000, 300),
                      ((1 << 20) - 8, (1 << 20) + 100_000, 40)):
        idx = rng.choice(tr.n, size=k, replace=False)
        ln[idx] = rng.integers(lo, hi, size=k).astype(np.uint32)
    tr2 = Trace(arena, tr.offset, ln, tr.ts_ns)
    with tcbee_amd.PacketParser(max_frames=1 << 19, max_arena=len(arena) + 64,
                                max_flows=62_000, variants=nopack == "1") as p:
        assert_same(p.parse(tr2), oracle.parse(tr2), p.flows())
        assert p.count_mode() == 1 and p.status() == 0


@pytest.mark.parametrize("cuts", [[0, 30_000], [0, 9_000, 9_001, 21_000, 30_000],
                                  [0, 3_000, 6_000, 9_000, 12_000, 15_000, 18_000, 21_000, 30_000]])
def test_device_merge_matches_unsharded(gpu, oracle, cuts):
    """Per-shard contexts -> device export -> concatenation (what the RCCL all-gather
    delivers) -> tcbee_flow_merge_device -> remap == the oracle on the whole trace."""
    import torch
    from tracegen import mixed_trace
    tr = mixed_trace(30_000, seed=12, n_flows=900)
    full = oracle.parse(tr)
    cap, world = 2048, len(cuts) - 1
    ents, metas, ids = [], [], []
    for lo, hi in zip(cuts, cuts[1:]):
        # (~1.7k distinct keys: a mixed trace draws ~1.9 keys per pool flow)
        with tcbee_amd.PacketParser(max_frames=1 << 16, max_arena=1 << 24, max_flows=cap) as p:
            res = p.parse(tr.slice(lo, hi))
            ent = torch.zeros((cap, 8), dtype=torch.int64, device="cuda")
            meta = torch.zeros(2, dtype=torch.int64, device="cuda")
            p.export_device(ent, cap, meta)
            p.sync()
            ents.append(ent)
            metas.append(meta)
            ids.append(res.flow_id)
    with tcbee_amd.PacketParser(max_frames=1 << 10, max_flows=1 << 12) as m:
        out_ids = torch.empty(world * cap, dtype=torch.int32, device="cuda")
        m.merge_device(torch.cat(ents), world, cap, torch.cat(metas), tr.n, out_ids)
        m.sync()
        assert np.array_equal(m.flows(), full[4])
        gids = []
        for r, x in enumerate(ids):
            d = torch.from_numpy(x.view(np.int32).copy()).cuda()
            tcbee_amd.parser.remap_ids_device(d, len(x), None, out_ids[r * cap:(r + 1) * cap], cap)
            torch.cuda.synchronize()
            gids.append(d.cpu().numpy().view(np.uint32))
        assert np.array_equal(np.concatenate(gids), full[2])
        # merging again replaces the table (idempotent)
        m.merge_device(torch.cat(ents), world, cap, torch.cat(metas), tr.n, out_ids)
        m.sync()
        assert np.array_equal(m.flows(), full[4])


@pytest.mark.parametrize("map_len,big", [(1, False), (5000, False), (16384, True),
                                         (40_000, True)])
def test_remap_ids_paths(gpu, map_len, big):
    """ids[p] = map[ids[p]]: map entries staged in LDS (u16, first 16384), global ids
    >= 0xFFFF and ids past the LDS part looked up in HBM, ids >= map_len -> ~0;
    unaligned start, ragged tail, and the count taken from the device word."""
    import torch
    rng = np.random.default_rng(map_len)
    hi = (1 << 31) if big else 60_000
    mp = rng.integers(0, hi, size=map_len, dtype=np.int64).astype(np.uint32)
    if big:
        mp[::7] = np.uint32(0xFFFF)  # the LDS sentinel value itself is a valid id
    n = 1_000_003
    ids = rng.integers(0, map_len + 3, size=n + 5, dtype=np.int64).astype(np.uint32)
    d = torch.from_numpy(ids.view(np.int32).copy()).cuda()
    d_map = torch.from_numpy(mp.view(np.int32).copy()).cuda()
    n_dev = torch.tensor([n - 2], dtype=torch.int64, device="cuda")
    sub = d[1:]  # 4-B offset: the scalar head before the 16-B vectors
    tcbee_amd.parser.remap_ids_device(sub, n, n_dev, d_map, map_len)
    torch.cuda.synchronize()
    got = sub.cpu().numpy().view(np.uint32)
    src = ids[1:]
    k = n - 2
    want = np.where(src[:k] < map_len, mp[np.minimum(src[:k], map_len - 1)], np.uint32(0xFFFFFFFF))
    assert np.array_equal(got[:k], want)
    assert np.array_equal(got[k:], src[k:])  # past *n_dev: untouched


def test_flow_table_full_reports(gpu):
    from tracegen import mixed_trace
    tr = mixed_trace(50_000, seed=5, n_flows=5000)
    with tcbee_amd.PacketParser(max_frames=1 << 17, max_arena=1 << 25, max_flows=16) as p:
        res = p.parse(tr)
        assert res.n > 0
        assert p.status() == tcbee_amd._lib.EFLOWFULL


@pytest.mark.parametrize("short", [0, 7])
def test_flow_table_exact_capacity(gpu, oracle, short):
    """max_flows bounds the claims exactly (round 3's compact table): a mixed trace
    (IPv4-form keys in the 16-B compact slots, IPv6 keys in the 64-B wide slots)
    with max_flows = its distinct flows is bit-exact with status OK; `short` flows
    fewer refuse exactly that many flows (dead slots: their frames stay
    unclassified, id ~0), records unchanged, TCBEE_EFLOWFULL; a second batch with
    the table full finds the dead slots again (no new claims, no duplicates)."""
    from tracegen import mixed_trace
    tr = mixed_trace(60_000, seed=77, n_flows=2500)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    cap = len(table) - short
    with tcbee_amd.PacketParser(max_frames=1 << 17, max_arena=1 << 25, max_flows=cap) as p:
        r1 = p.parse(tr.slice(0, 40_000))
        r2 = p.parse(tr.slice(40_000, tr.n))
        assert np.array_equal(np.concatenate([r1.records, r2.records]), rec)
        ids = np.concatenate([r1.flow_id, r2.flow_id])
        fl = p.flows()
        if short == 0:
            assert p.status() == 0
            assert np.array_equal(ids, fi) and np.array_equal(fl, table)
        else:
            assert p.status() == tcbee_amd._lib.EFLOWFULL
            assert len(fl) == cap
            refused = ids == 0xFFFFFFFF
            assert 0 < refused.sum() < len(ids)
            # every record of a claimed flow carries an id < cap, and a flow's
            # records are all claimed or all refused
            assert ids[~refused].max() < cap
            keys = np.unique(fi[refused])
            assert not np.isin(fi[~refused], keys).any()
            assert len(keys) == short


def test_batch_over_1M_frames_multibatch(gpu, oracle):
    """Batches above 1M frames take the 4-kernel rank scan (bounded by the highest
    first-seen word, bitmap cleared again by K3); three batches, the second one
    adding flows to a table that already has some."""
    tr = tcbee_amd.synth_trace(2_600_000, sizes="imix", kind=1, n_flows=6000)
    cuts = [0, 1_200_000, 2_400_000, 2_600_000]
    with tcbee_amd.PacketParser(max_frames=1_300_000, max_arena=1 << 30, max_flows=1 << 14) as p:
        rs = [p.parse(tr.slice(lo, hi)) for lo, hi in zip(cuts, cuts[1:])]
        rec, fh, fi, ctr, table = oracle.parse(tr)
        assert np.array_equal(np.concatenate([r.records for r in rs]), rec)
        assert np.array_equal(np.concatenate([r.flow_id for r in rs]), fi)
        assert np.array_equal(p.flows(), table)


def test_k3_mode_switch_across_batches(gpu, oracle):
    """A table that grows past K3's LDS bins between batches: batch 1 is counted in
    mode 0 (<= 12288 flows), batch 2 in mode 1 (bucketed); ids and counts continue."""
    from tracegen import mixed_trace
    a = mixed_trace(40_000, seed=31, n_flows=3000)
    b = mixed_trace(160_000, seed=32, n_flows=40_000)
    frames = [a.frame(i) for i in range(a.n)] + [b.frame(i) for i in range(b.n)]
    tr = Trace.from_frames(frames)
    with tcbee_amd.PacketParser(max_frames=1 << 18, max_arena=1 << 26, max_flows=1 << 17) as p:
        r1 = p.parse(tr.slice(0, a.n))
        n1 = p.flow_count()
        r2 = p.parse(tr.slice(a.n, tr.n))
        rec, fh, fi, ctr, table = oracle.parse(tr)
        assert n1 <= 12288 < len(table)
        assert np.array_equal(np.concatenate([r1.flow_id, r2.flow_id]), fi)
        assert np.array_equal(p.flows(), table)


def test_config4_scale_over_1M_flows_mixed(gpu, oracle):
    """Config 4's table size: > 1M distinct flows from a mixed trace
    (rejects, runts, IPv6, v4-compatible collisions), two batches of 2.5M frames
    through K1's large-table probe path, K2's multi-kernel rank scan and K3's
    bucketed mode; records, ids and the whole table vs the oracle."""
    from tracegen import mixed_trace
    tr = mixed_trace(5_000_000, seed=4004, n_flows=1_700_000)
    cut = 2_500_000
    a, b = tr.slice(0, cut), tr.slice(cut, tr.n)
    # (1.88M distinct keys: a mixed trace draws ~1.1 keys per pool flow at this size)
    with tcbee_amd.PacketParser(max_frames=cut, max_arena=max(len(a.arena), len(b.arena)),
                                max_flows=2_000_000) as p:
        r1 = p.parse(a)
        r2 = p.parse(b)
        ft = oracle.new_flowtab(1 << 22)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        assert len(table) > 1_000_000
        assert np.array_equal(np.concatenate([r1.records, r2.records]), rec)
        assert np.array_equal(np.concatenate([r1.flow_hash, r2.flow_hash]), fh)
        assert np.array_equal(np.concatenate([r1.flow_id, r2.flow_id]), fi)
        fl = p.flows()
        assert len(fl) == len(table) and np.array_equal(fl, table)
        assert p.status() == 0


@pytest.mark.parametrize("cap_mult", [1, 4])
def test_config4_1M_flows_device_right_sized(gpu, oracle, cap_mult):
    """1M synthetic IMIX flows, device-resident path; the table sized exactly for 1M
    flows (max_flows = flows: every claim used, slot load 1/8, 176 MB of slot lines)
    and 4x that (load 1/32)."""
    import torch
    n, flows = 3_500_000, 1_000_000
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=flows)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fh_d = torch.empty(n, dtype=torch.int32, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=cap_mult * flows) as p:
        s = torch.cuda.current_stream().cuda_stream
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, fh_d, fi_d, n_d,
                       ctr_d, stream=s)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 21)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        assert int(n_d.item()) == len(rec) == n
        assert np.array_equal(rec_d[:n * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(fh_d.cpu().numpy().view(np.uint32), fh)
        assert np.array_equal(fi_d.cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(p.flows(), table)
        assert p.status() == 0


@pytest.mark.parametrize("pool,n,k3v", [(10_500, 1_500_000, ""), (17_000, 2_000_000, ""),
                                        (75_000, 2_500_000, ""), (170_000, 3_000_000, ""),
                                        (10_500, 1_500_000, "16"), (17_000, 2_000_000, "16")])
def test_k3_range_mode_large_batches(gpu, oracle, pool, n, k3v, monkeypatch):
    """Large-table K3 on one batch, device-resident: mode 3 at 2 and 3 claim ranges,
    mode 1 beyond (143k flows: 36 buckets, lane-scattered; ~290k flows: 71 buckets,
    the LDS-staged scatter); a mixed trace with hot, rejected and > 64 KiB frames;
    ids, the whole table and counters vs the oracle. k3v "16": the variants build
    with 16 records per lane and iteration (what the product runs on batches of
    >= 16M frames), mode 3 here."""
    import torch
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_TEST_K3_WIDE", "1" if k3v else "0")
    tr = mixed_trace(n, seed=pool, n_flows=pool)  # ~1.9 distinct keys per pool flow
    ln = tr.caplen.copy()
    rng = np.random.default_rng(7)
    big = rng.choice(tr.n - 1, size=50, replace=False)
    pad = 200_000
    arena = np.concatenate([tr.arena, np.zeros(pad, np.uint8)])
    ln[big] = np.uint32(70_000)  # caplen past the LDS bins' 64 KiB: device atomics
    tr = Trace(arena, tr.offset, ln, tr.ts_ns)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=4 * pool, variants=bool(k3v)) as p:
        s = torch.cuda.current_stream().cuda_stream
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d, n_d,
                       ctr_d, stream=s)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 20)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        k = int(n_d.item())
        assert k == len(rec) and 12288 < len(table)
        assert np.array_equal(fi_d[:k].cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(p.flows(), table)
        assert ctr_d.cpu().numpy().tolist() == [ctr["ingress"], ctr["egress"], ctr["handled"],
                                                 ctr["dropped"]]
        assert p.status() == 0
        assert p.count_mode() == (3 if len(table) <= 3 * 12288 else 1)


@pytest.mark.parametrize("flows", [130_560, 130_561, 261_120, 261_121])
def test_k3_chunk_sub_bin_boundaries(gpu, oracle, flows):
    """Mode 1's chunk sort bins claims by claim >> sh, sh the smallest shift >= 8
    that keeps a chunk's bins under 511 (tcbee_kernels.hip k_count_chunk2): 130560
    flows = 510 bins of 256 (sh 8, every bin used), 130561 the first count at sh 9,
    261120 / 261121 the same edge of sh 9 -> 10. Every flow appears (16 frames per
    flow of the per-frame draw; checked: the table has exactly
    `flows` entries); ids, records and the table vs the oracle."""
    import torch
    n = 16 * flows
    tr = tcbee_amd.synth_trace(n, sizes="64", kind=1, n_flows=flows, seed=flows)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16) as p:
        s = torch.cuda.current_stream().cuda_stream
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d, n_d,
                       ctr_d, stream=s)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 20)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        assert len(table) == flows
        k = int(n_d.item())
        assert k == len(rec) == n
        assert np.array_equal(fi_d[:k].cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(p.flows(), table)
        assert p.status() == 0 and p.count_mode() == 1


def test_null_stream_after_default_stream_work(gpu, oracle):
    """A context created and used right behind work still queued on HIP's legacy
    default stream (a framework's fills of the outputs, a busy default stream): with
    a NULL stream the parse waits for that work (tcbee_amd.h), and the context's own
    initialisation is complete when create returns. Outputs pre-filled with a
    sentinel on the default stream; ids, records, counters and the table vs the
    oracle. (A contract test: the round-5 failure this ordering fixed — every id 0,
    about one parity-file run in five — was intermittent and this test alone passed
    on the library before the fix too)"""
    import torch
    n, flows = 2_000_000, 150_000
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=flows, seed=77)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    torch.cuda.synchronize()
    busy = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for v in range(8):  # a few ms of default-stream work ahead of everything below
        busy.fill_(v)
    rec_d = torch.full((n * 74 + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    fi_d = torch.full((n,), -2, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16) as p:
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d, n_d,
                       ctr_d, stream=None)
        p.sync()
        torch.cuda.synchronize()
        k = int(n_d.item())
        assert k == len(rec)
        assert np.array_equal(fi_d[:k].cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert ctr_d.cpu().numpy().tolist() == [ctr["ingress"], ctr["egress"], ctr["handled"],
                                                 ctr["dropped"]]
        assert np.array_equal(p.flows(), table)
    del busy


def test_null_stream_parse_with_another_device_current(gpu, oracle):
    """a NULL-stream call records the legacy default stream of the CURRENT
    device; ctx_stream now makes the context's device current first, so a thread whose
    current device is another GPU still orders the parse after the right device's
    default-stream work. Needs two GPUs (skipped on a one-GPU box)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two HIP devices")
    tr = tcbee_amd.synth_trace(300_000, sizes="imix", kind=1, n_flows=5000, seed=88)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    n = tr.n
    with torch.cuda.device(1):
        d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
        d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
        d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
        d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
        rec_d = torch.full((n * 74 + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        fi_d = torch.full((n,), -2, dtype=torch.int32, device="cuda")
        n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize(1)
    with tcbee_amd.PacketParser(device=1, max_frames=n, max_flows=8192) as p:
        torch.cuda.set_device(0)
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d, n_d,
                       ctr_d, stream=None)
        p.sync()
        torch.cuda.synchronize(1)
        k = int(n_d.item())
        assert k == len(rec)
        assert np.array_equal(fi_d[:k].cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(p.flows(), table)


@pytest.mark.parametrize("lib", ["legacy_init_hook", "product"])
def test_legacy_init_race_pinned(gpu, oracle, lib, monkeypatch):
    """round 5's intermittent all-zero flow ids, made deterministic.

    Pre-fix, tcbee_ctx_create zero-filled the first-seen bitmap (and the look-back
    status, the wide slots) with hipMemset on HIP's legacy default stream, and a
    NULL-stream parse ran on the context's non-blocking stream without waiting for
    that stream. A fill still queued behind a framework's default-stream work could
    therefore land between K2's k_mark (which sets each new flow's first-frame bit)
    and k_scan_words (which counts them): every new flow then ranks 0, and every
    record's id is 0 while the record count stays right — the failure of
    test_zipf_many_flows[1M] in gpurun_out/prod_t1.log. Here the interleaving is
    pinned by host-released waits (variants-build test entry points):
      1. a wait kernel on the legacy default stream (the "long default-stream
         kernel"), released by host flag A;
      2. the context is created behind it (the legacy-init hook: its fills queue
         behind the wait, and create returns at once — hipMemset does not block);
      3. the NULL-stream parse: with the hook K1 + k_mark run, then K2 holds its
         stream on host flag B (tcbee_test_k2_hold);
      4. flag A: the wait ends and the fills run (the test waits for them by an event
         on the default stream); 5. flag B: K2 scans the zeroed bitmap.
    The hook must give ids all 0 (count and records right); the product, through the
    same steps 1-2-4 (no hold exists there), must be bit-exact: its fills are on the
    context's stream before create returns, and its NULL-stream parse waits for the
    legacy stream's queued work (ctx_stream)."""
    import ctypes as C
    import time as _t

    import torch
    hook = lib == "legacy_init_hook"
    if hook:
        monkeypatch.setenv("TCBEE_TEST_LEGACY_INIT", "1")
    n, flows = 4_000_000, 10_000  # > 1M frames: the four-kernel K2 (k_mark ... k_assign)
    tr = tcbee_amd.synth_trace(n, sizes="64", kind=1, n_flows=flows, seed=606)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fi_d = torch.full((n,), -2, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    states = torch.zeros(2, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    Lv = tcbee_amd._lib.lib(variants=True)
    fa, fb = C.c_void_p(), C.c_void_p()
    tcbee_amd._lib.check(Lv.tcbee_test_flag_create(C.byref(fa)), "flag")
    tcbee_amd._lib.check(Lv.tcbee_test_flag_create(C.byref(fb)), "flag")
    flag_a = C.c_uint64.from_address(fa.value)
    flag_b = C.c_uint64.from_address(fb.value)
    p = None
    try:
        # 1. the default-stream wait (10 s at most), queued first
        tcbee_amd._lib.check(Lv.tcbee_test_wait_host_device(
            fa, 1, 10_000_000, C.c_void_p(states.data_ptr()), None), "wait A")
        # 2. the context, created behind it
        t0 = _t.perf_counter()
        p = tcbee_amd.PacketParser(max_frames=n, max_flows=flows + 1024, max_wide_flows=16,
                                   variants=hook)
        create_s = _t.perf_counter() - t0
        if hook:
            tcbee_amd._lib.check(Lv.tcbee_test_k2_hold(
                p._h, fb, C.c_void_p(states.data_ptr() + 8)), "k2 hold")
        # 3. the NULL-stream parse
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d,
                       n_d, ctr_d, stream=None)
        _t.sleep(0.2)  # (the hook: K1 + k_mark are done well before this)
        # 4. release the default stream; wait until its queued work (the hook's fills)
        #    has completed, without waiting on any other stream
        flag_a.value = 1
        ev = torch.cuda.Event()
        ev.record(torch.cuda.default_stream())
        t1 = _t.perf_counter()
        while not ev.query():
            assert _t.perf_counter() - t1 < 15, "the default stream did not drain"
            _t.sleep(0.001)
        # 5. release K2 (hook)
        flag_b.value = 1
        p.sync()
        torch.cuda.synchronize()
        st = states.cpu().tolist()
        k = int(n_d.item())
        ids = fi_d[:k].cpu().numpy().view(np.uint32)
        assert st[0] == 3, f"the default-stream wait timed out ({st}): create blocked"
        assert create_s < 5, create_s
        assert k == len(rec) == n
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        if hook:
            assert st[1] == 3, st
            # the round-5 failure, reproduced: every record's flow id 0
            assert not ids.any(), f"{int((ids != 0).sum())} non-zero ids"
            assert len(np.unique(fi)) == flows
        else:
            assert np.array_equal(ids, fi)
            assert ctr_d.cpu().numpy().tolist() == [ctr["ingress"], ctr["egress"],
                                                     ctr["handled"], ctr["dropped"]]
            assert np.array_equal(p.flows(), table) and p.status() == 0
    finally:
        flag_a.value = 1
        flag_b.value = 1
        torch.cuda.synchronize()
        if p is not None:
            p.close()
        Lv.tcbee_test_flag_destroy(fa)
        Lv.tcbee_test_flag_destroy(fb)


@pytest.mark.parametrize("flows", [200_000, 1_000_000])
def test_zipf_many_flows(gpu, oracle, flows):
    """Zipf(1.1) over many flows: a head flow holding ~12 % of the records beside a
    long tail, through K3 mode 1 — a chunk's hot sub-bin takes hundreds of records
    (the ranking's one-add-per-wave path) while most sub-bins hold one or two; ids,
    records and the table (only the flows that appeared) vs the oracle."""
    import torch
    n = 4_000_000
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=2, n_flows=flows, seed=flows + 2)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16) as p:
        s = torch.cuda.current_stream().cuda_stream
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d, n_d,
                       ctr_d, stream=s)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 21)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        k = int(n_d.item())
        assert k == len(rec) == n and len(table) > 12_288
        assert int(table["pkts"].max()) > n // 20  # the head flow
        assert np.array_equal(fi_d[:k].cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(p.flows(), table)
        assert p.status() == 0 and p.count_mode() == (3 if len(table) <= 3 * 12288 else 1)


@pytest.mark.parametrize("flows", [60_000, 250_000])
def test_ipv6_many_flows(gpu, oracle, flows):
    """IPv6/TCP IMIX (kind 3) with many flows: every key lives in the wide slots
    (64-B tag/key slots, not the compact IPv4 ones), K3 in mode 1 (60k flows: 15
    buckets; 250k: 62, chunk sub-bins of 512 claims); every flow appears (16 frames
    per flow); records, hashes, ids and the whole table vs the oracle."""
    import torch
    n = 16 * flows
    tr = tcbee_amd.synth_trace(n, sizes="imix6", kind=3, n_flows=flows, seed=flows + 6)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fh_d = torch.empty(n, dtype=torch.int32, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    with tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16) as p:
        s = torch.cuda.current_stream().cuda_stream
        p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, fh_d, fi_d, n_d,
                       ctr_d, stream=s)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 20)
        try:
            rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        assert len(table) == flows
        k = int(n_d.item())
        assert k == len(rec) == n
        assert np.array_equal(rec_d[:k * 74].cpu().numpy().reshape(-1, 74), rec)
        assert np.array_equal(fh_d.cpu().numpy().view(np.uint32), fh)
        assert np.array_equal(fi_d.cpu().numpy().view(np.uint32), fi)
        assert np.array_equal(p.flows(), table)
        assert ctr_d.cpu().numpy().tolist() == [ctr["ingress"], ctr["egress"], ctr["handled"],
                                                 ctr["dropped"]]
        assert p.status() == 0 and p.count_mode() == 1


@pytest.mark.parametrize("reset", [False, True])
@pytest.mark.parametrize("flows", [300, 40_000])
def test_async_ids_stream_batches(gpu, oracle, reset, flows):
    """TCBEE_EX_ASYNC_IDS: each batch's K3 (ids, pkts/bytes, counters, out_n) runs on
    a side stream while the next batch parses (two alternating slots inside the
    context; the next K2 waits for it). Four back-to-back batches, flow ids carried
    across them or the table reset before each (the bench's cold table); every
    record, id, counter and the final table vs the oracle."""
    import torch
    from tracegen import mixed_trace
    nb, per = 4, 150_000
    tr = mixed_trace(nb * per, seed=flows + 3, n_flows=flows)
    parts = [tr.slice(i * per, (i + 1) * per) for i in range(nb)]
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream().cuda_stream
    dev = []
    for t in parts:
        d = {"arena": torch.from_numpy(np.concatenate([t.arena, np.zeros(64, np.uint8)])).cuda(),
             "off": torch.from_numpy(t.offset.view(np.int64)).cuda(),
             "len": torch.from_numpy(t.caplen.view(np.int32)).cuda(),
             "ts": torch.from_numpy(t.ts_ns.view(np.int64)).cuda(),
             "rec": torch.empty(per * 74 + 64, dtype=torch.uint8, device="cuda"),
             "id": torch.empty(per, dtype=torch.int32, device="cuda"),
             "n": torch.zeros(1, dtype=torch.int64, device="cuda"),
             "ctr": torch.zeros(4, dtype=torch.int64, device="cuda")}
        dev.append(d)
    torch.cuda.synchronize()
    with tcbee_amd.PacketParser(max_frames=per, max_flows=4 * flows + 4096) as p:
        for d, t in zip(dev, parts):
            if reset:
                p.reset_flows(stream=main, sync=False)
            p.parse_device(d["arena"], len(t.arena), d["off"], d["len"], d["ts"], t.n, d["rec"],
                           t.n, None, d["id"], d["n"], d["ctr"], stream=main,
                           ids_stream=side.cuda_stream)
        torch.cuda.synchronize()
        ft = oracle.new_flowtab(1 << 17)
        try:
            for i, (d, t) in enumerate(zip(dev, parts)):
                if reset:
                    oracle.free_flowtab(ft)
                    ft = oracle.new_flowtab(1 << 17)
                base = 0 if reset else int(sum(int(x["n"].item()) for x in dev[:i]))
                rec, fh, fi, ctr, _ = oracle.parse(t, ft=ft, record_base=base)
                k = int(d["n"].item())
                assert k == len(rec)
                assert np.array_equal(d["rec"][:k * 74].cpu().numpy().reshape(-1, 74), rec)
                assert np.array_equal(d["id"][:k].cpu().numpy().view(np.uint32), fi)
                assert d["ctr"].cpu().numpy().tolist() == [ctr["ingress"], 0, ctr["handled"], 0]
            table = oracle.flows(ft)
        finally:
            oracle.free_flowtab(ft)
        assert np.array_equal(p.flows(), table)
        assert p.status() == 0


def _concat(a, b):
    """Trace a followed by trace b (b's offsets rebased past a's arena)."""
    return Trace(np.concatenate([a.arena, b.arena]),
                 np.concatenate([a.offset, b.offset + np.uint64(len(a.arena))]),
                 np.concatenate([a.caplen, b.caplen]), np.concatenate([a.ts_ns, b.ts_ns]))


@pytest.mark.parametrize("variant", ["0", "0n", "twopass"])
@pytest.mark.parametrize("flows", [40_000, 150_000])
def test_k3_chunked_scatter(gpu, oracle, variant, flows, monkeypatch):
    """K3 mode 1's single-pass chunked scatter (k_count_chunk2: chunks of 12288
    records in 76 KiB of LDS, two workgroups per CU — "0n": unpacked K1 -> K3
    words — bucket-sorted in LDS, ids gathered bucket by bucket, region runs per
    chunk) and the two-pass scatter the product keeps for tables of more than 510
    buckets ("twopass": TCBEE_TEST_K3_TWOPASS forces it here), bit-exact vs the
    oracle: a ragged last chunk, caplens past the 20-bit region field and the
    packed K1 -> K3 field, a single-flow stretch (every wave on one bucket), two
    batches (claims of batch 1 looked up again in batch 2)."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_TEST_K3_NORANGE", "1")
    monkeypatch.setenv("TCBEE_TEST_K3_TWOPASS", "1" if variant == "twopass" else "0")
    if variant.endswith("n"):
        monkeypatch.setenv("TCBEE_TEST_NOPACK", "1")
    mt = mixed_trace(350_001, seed=123, n_flows=flows)
    rng = np.random.default_rng(9)
    big = rng.choice(mt.n, size=200, replace=False)
    pad = 2_600_000
    ln = mt.caplen.copy()
    ln[big] = rng.integers(16_000, pad, size=len(big)).astype(np.uint32)
    mt = Trace(np.concatenate([mt.arena, np.zeros(pad, np.uint8)]), mt.offset, ln, mt.ts_ns)
    tr = _concat(mt, tcbee_amd.synth_trace(70_000, sizes="64", kind=0, n_flows=1))
    cut = 150_000
    with tcbee_amd.PacketParser(max_frames=1 << 19, max_arena=1 << 28, max_flows=1 << 18,
                                variants=True) as p:
        r1 = p.parse(tr.slice(0, cut))
        assert p.count_mode() == 1
        r2 = p.parse(tr.slice(cut, tr.n))
        assert p.count_mode() == 1
        rec, fh, fi, ctr, table = oracle.parse(tr)
        assert np.array_equal(np.concatenate([r1.records, r2.records]), rec)
        assert np.array_equal(np.concatenate([r1.flow_id, r2.flow_id]), fi)
        fl = p.flows()
        assert len(fl) == len(table) and np.array_equal(fl, table)
        assert p.status() == 0


@pytest.mark.parametrize("fuse", [True, False])
def test_small_context_fused_rank(gpu, oracle, monkeypatch, fuse):
    """Contexts of <= 256 flows rank each batch's new flows inside K3 (no rank
    launch, tcbee_capi fuse): batches of a mixed trace (both hooks' frame classes,
    hot flows, an empty batch, a 1M-frame single-flow batch after a reset) give the
    oracle's records, ids and table; TCBEE_NO_FUSE_RANK=1 (the separate rank
    kernel) gives the same."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_NO_FUSE_RANK", "0" if fuse else "1")
    tr = mixed_trace(80_000, seed=909, n_flows=60)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert 0 < len(table) <= 256
    with tcbee_amd.PacketParser(max_frames=1 << 20, max_arena=1 << 27, max_flows=256,
                                variants=not fuse) as p:
        ft = oracle.new_flowtab()
        base = 0
        try:
            for lo, hi in [(0, 1), (1, 5_000), (5_000, 5_000), (5_000, 41_111), (41_111, 80_000)]:
                part = tr.slice(lo, hi)
                res = p.parse(part)
                orc = oracle.parse(part, ft=ft, record_base=base)
                assert_same(res, orc)
                base += len(orc[0])
            assert np.array_equal(p.flows(), oracle.flows(ft))
            assert p.status() == 0
        finally:
            oracle.free_flowtab(ft)
        one = tcbee_amd.synth_trace(1_000_000, sizes="64", kind=0, n_flows=1)
        for _ in range(2):  # config 2, the table reset before each batch (as bench.py)
            p.reset_flows()
            res = p.parse(one)
            assert_same(res, oracle.parse(one), p.flows())


@pytest.mark.parametrize("fuse", [True, False])
def test_small_context_big_frames_over_k3_blocks(gpu, oracle, monkeypatch, fuse):
    """a small context's fused rank (<= 256 flows) with frames of
    >= 64 KiB caplen — counted by device atomics, by local id — spread over many K3
    blocks, in flows that are new in the batch: every block must resolve a new flow's
    local id itself and its counters must be zero before any block adds (k_prep
    zeroes the ids not yet handed out); loopback-sized 70 000-B frames, three
    batches (the second one after a reset), records, ids and table vs the oracle."""
    monkeypatch.setenv("TCBEE_NO_FUSE_RANK", "0" if fuse else "1")
    tr = tcbee_amd.synth_trace(400_000, sizes="imix", kind=1, n_flows=200)
    rng = np.random.default_rng(17)
    big = rng.choice(tr.n, size=3000, replace=False)
    pad = 80_000
    ln = tr.caplen.copy()
    ln[big] = rng.integers(65_536, 70_001, size=len(big)).astype(np.uint32)
    tr = Trace(np.concatenate([tr.arena, np.zeros(pad, np.uint8)]), tr.offset, ln, tr.ts_ns)
    with tcbee_amd.PacketParser(max_frames=1 << 19, max_arena=1 << 28, max_flows=256,
                                variants=not fuse) as p:
        for lo, hi, reset in [(0, 250_000, True), (250_000, 400_000, True),
                              (0, 400_000, False)]:
            if reset:
                p.reset_flows()
            part = tr.slice(lo, hi)
            if reset:
                assert_same(p.parse(part), oracle.parse(part), p.flows())
            else:
                # the table holds batch 2's flows, the record base its records
                ft = oracle.new_flowtab()
                try:
                    prev = oracle.parse(tr.slice(250_000, 400_000), ft=ft)
                    orc = oracle.parse(part, ft=ft, record_base=len(prev[0]))
                    assert_same(p.parse(part), orc)
                    assert np.array_equal(p.flows(), oracle.flows(ft))
                finally:
                    oracle.free_flowtab(ft)
            assert p.status() == 0


def test_product_library_ignores_variant_env(gpu, oracle, monkeypatch):
    """the product library reads no environment variable. With every
    test-hook variable of the variants build set (NORANGE/TWOPASS/NOBUCKET select
    other K3 modes, NOPACK/WITHHOLD/NO_FUSE_RANK/WIDE/FPL/WALK other K1-K3 paths), a
    product context keeps its own paths (K3 mode 3 on a ~19k-flow trace) and matches
    the oracle bit-exact, while a context of the variants build does follow them (it
    reports K3 mode 2: the setting took) and matches the oracle too."""
    from tracegen import mixed_trace
    for k, v in {"TCBEE_TEST_NOPACK": "1", "TCBEE_TEST_WITHHOLD": "3",
                 "TCBEE_NO_FUSE_RANK": "1", "TCBEE_FPL": "4", "TCBEE_TEST_K3_NORANGE": "1",
                 "TCBEE_TEST_K3_NOBUCKET": "1", "TCBEE_TEST_K3_TWOPASS": "1",
                 "TCBEE_TEST_K3_WIDE": "1", "TCBEE_WALK": "0"}.items():
        monkeypatch.setenv(k, v)
    tr = mixed_trace(300_000, seed=808, n_flows=10_000)
    orc = oracle.parse(tr)
    assert 12_288 < len(orc[4]) < 36_000
    for variants, mode in ((False, 3), (True, 2)):
        with tcbee_amd.PacketParser(max_frames=1 << 19, max_arena=1 << 28, max_flows=1 << 16,
                                    variants=variants) as p:
            assert_same(p.parse(tr), orc, p.flows())
            assert p.status() == 0
            assert p.count_mode() == mode, (variants, p.count_mode())


@pytest.mark.parametrize("short", [0, 9])
def test_max_wide_flows_exact_bound(gpu, oracle, short):
    """tcbee_ctx_create_ex sizes the 64-B wide slots for
    max_wide_flows non-IPv4-form keys instead of max_flows. With max_wide_flows = the
    trace's IPv6 keys the context is bit-exact; `short` fewer refuse exactly that many
    IPv6 keys (TCBEE_EFLOWFULL, frames unclassified, no claim taken: every IPv4 key
    and the other IPv6 keys keep dense ids), records unchanged."""
    from tracegen import mixed_trace
    tr = mixed_trace(60_000, seed=78, n_flows=2500)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    t = table["tuple"]
    wide = (t[:, 0:12].any(axis=1)) | (t[:, 16:28].any(axis=1))
    nwide = int(wide.sum())
    assert nwide > 100 and (~wide).sum() > 100
    with tcbee_amd.PacketParser(max_frames=1 << 17, max_arena=1 << 25, max_flows=len(table),
                                max_wide_flows=nwide - short) as p:
        res = p.parse(tr)
        assert np.array_equal(res.records, rec)
        fl = p.flows()
        if short == 0:
            assert p.status() == 0
            assert_same(res, (rec, fh, fi, ctr, table), fl)
            return
        assert p.status() == tcbee_amd._lib.EFLOWFULL
        assert len(fl) == len(table) - short
        ft = fl["tuple"]
        assert int(((ft[:, 0:12].any(axis=1)) | (ft[:, 16:28].any(axis=1))).sum()) == nwide - short
        refused = res.flow_id == 0xFFFFFFFF
        keys = np.unique(fi[refused])
        assert len(keys) == short and wide[keys].all()
        assert res.flow_id[~refused].max() < len(table) - short
        assert not np.isin(fi[~refused], keys).any()


@pytest.mark.parametrize("flows", [1, 40, 5000])
def test_k3_wide_iteration_variant(gpu, oracle, flows, monkeypatch):
    """K3 mode 0 with 16 records per lane and iteration (the product's form for
    batches of >= 16M frames, forced here by TCBEE_TEST_K3_WIDE): a ragged tail,
    saturated packed caplens (the side array), > 64 KiB frames (device atomics), a
    hot flow (the wave-uniform add) — bit-exact vs the oracle."""
    from tracegen import mixed_trace
    monkeypatch.setenv("TCBEE_TEST_K3_WIDE", "1")
    tr = mixed_trace(150_001, seed=303, n_flows=flows)
    rng = np.random.default_rng(8)
    big = rng.choice(tr.n, size=300, replace=False)
    pad = 2_600_000
    ln = tr.caplen.copy()
    ln[big] = rng.integers(16_000, pad, size=len(big)).astype(np.uint32)
    tr2 = Trace(np.concatenate([tr.arena, np.zeros(pad, np.uint8)]), tr.offset, ln, tr.ts_ns)
    # (a mixed trace draws ~1.9 keys per pool flow: 5000 -> ~9.5k flows, mode 0)
    with tcbee_amd.PacketParser(max_frames=1 << 18, max_arena=1 << 27, max_flows=12_000,
                                variants=True) as p:
        assert_same(p.parse(tr2), oracle.parse(tr2), p.flows())
        assert p.status() == 0 and p.count_mode() == 0


def test_small_context_generations_and_prep_free_batches(gpu, oracle):
    """Round 4: a small context (<= 256 flows) keeps two table generations; a fused
    batch's K3 prepares the next batch (tile words, state slot) and empties the
    inactive generation, so the next batch has no k_prep launch and a reset is a
    switch of generation. A sequence mixing resets, kept tables, IPv6 keys (wide
    slots), frames of >= 64 KiB, table reads between batches, an empty batch, a
    no-flows batch, a sync reset and batches of different tile counts, each checked
    against the oracle (records, hashes, ids, counters, the table)."""
    from tracegen import mixed_trace
    tr = mixed_trace(60_000, seed=1212, n_flows=24)
    rng = np.random.default_rng(3)
    ln = tr.caplen.copy()
    big = rng.choice(tr.n, size=200, replace=False)
    ln[big] = rng.integers(65_536, 70_001, size=len(big)).astype(np.uint32)
    tr = Trace(np.concatenate([tr.arena, np.zeros(80_000, np.uint8)]), tr.offset, ln, tr.ts_ns)
    assert len(oracle.parse(tr)[4]) <= 256
    cuts = [(0, 20_000), (20_000, 21_000), (21_000, 60_000), (5_000, 5_000), (100, 7_000),
            (7_000, 59_999), (0, 60_000), (33, 34), (1_000, 45_000)]
    # per step: reset before? ('dev' = tcbee_flow_reset_device, 'sync', None), flows on?
    plan = [("dev", True), ("dev", True), (None, True), ("dev", True), (None, True),
            ("sync", True), ("dev", False), ("dev", True), (None, True)]
    with tcbee_amd.PacketParser(max_frames=1 << 17, max_arena=1 << 27, max_flows=256) as p:
        ft = oracle.new_flowtab()
        base = 0
        try:
            for (lo, hi), (reset, flows) in zip(cuts, plan):
                if reset:
                    p.reset_flows(sync=reset == "sync")
                    oracle.free_flowtab(ft)
                    ft = oracle.new_flowtab()
                    base = 0
                part = tr.slice(lo, hi)
                res = p.parse(part, flows=flows)
                orc = oracle.parse(part, ft=ft if flows else None, record_base=base, flows=flows)
                if flows:
                    assert_same(res, orc)
                    base += len(orc[0])
                    assert np.array_equal(p.flows(), oracle.flows(ft))
                else:
                    assert np.array_equal(res.records, orc[0]) and res.counters == orc[3]
                assert p.status() == 0
        finally:
            oracle.free_flowtab(ft)


def test_k3_wide_iteration_large_batch(gpu, oracle):
    """Batches of >= 16M frames run K3 with 16 records per lane and iteration
    (CountArgs::wide_iter, the product's config-3 form): 16.8M 64-B frames over 3000
    flows, a ragged last block — records, hashes, ids, counters and the table vs the
    oracle, count mode 0."""
    n = (16 << 20) + 12_345
    tr = tcbee_amd.synth_trace(n, sizes="64", kind=1, n_flows=3000)
    with tcbee_amd.PacketParser(max_frames=n, max_arena=len(tr.arena), max_flows=4096) as p:
        assert_same(p.parse(tr), oracle.parse(tr), p.flows())
        assert p.status() == 0 and p.count_mode() == 0


def _fuzz_trace(seed: int, n: int, pool: int, port: int) -> Trace:
    """Random frames in a random-byte arena: caplens around every accept boundary
    (< 14, 53/54, 73/74) and up to 70 000 B (such a frame runs over the next ones),
    ethertype IPv4 / IPv6 / other, protocol TCP or not; with `pool` > 0 the addresses
    and ports come from `pool` keys (one of them carrying `port`), else they stay
    random. Frame starts are >= 64 B apart (no frame's header bytes are another's)."""
    rng = np.random.default_rng(seed)
    edge = np.array([0, 1, 13, 14, 15, 33, 53, 54, 55, 72, 73, 74, 75, 76, 96, 70_000])
    ln = np.where(rng.random(n) < 0.3, edge[rng.integers(0, len(edge), n)],
                  rng.integers(0, 400, n))
    stride = np.maximum(np.minimum(ln, 400), 64) + rng.integers(0, 16, n)
    off = np.concatenate([[0], np.cumsum(stride[:-1])]).astype(np.int64)
    arena = rng.integers(0, 256, size=int(off[-1]) + 70_000 + 64, dtype=np.uint8)
    et = rng.choice([0x0800, 0x86DD, 0x8100, 0x0806], size=n, p=[0.45, 0.4, 0.1, 0.05])
    arena[off + 12] = et >> 8
    arena[off + 13] = et & 0xFF
    v4 = et == 0x0800
    tcp = rng.random(n) < 0.85
    arena[np.where(v4, off + 23, off + 20)] = np.where(tcp, 6, rng.integers(0, 256, n))
    if pool:
        # key bytes: 32 address bytes (v4 uses the first 8) + sport, dport
        key = rng.integers(0, 256, size=(pool, 36), dtype=np.uint8)
        key[0, 34:36] = [port >> 8, port & 0xFF]
        k = rng.integers(0, pool, n)
        i4, i6 = np.nonzero(v4)[0], np.nonzero(~v4)[0]
        for j in range(8):  # v4: saddr, daddr at 26..33, ports at 34..37
            arena[off[i4] + 26 + j] = key[k[i4], j]
        for j in range(32):  # v6: saddr, daddr at 22..53, ports at 54..57
            arena[off[i6] + 22 + j] = key[k[i6], j]
        for j in range(4):
            arena[off[i4] + 34 + j] = key[k[i4], 32 + j]
            arena[off[i6] + 54 + j] = key[k[i6], 32 + j]
    ts = rng.integers(0, 2**63, size=n, dtype=np.int64).astype(np.uint64)
    return Trace(arena, off.astype(np.uint64), ln.astype(np.uint32), ts)


@pytest.mark.parametrize("seed,pool,port", [(1, 0, 0), (2, 40, 0), (3, 40, 4242), (4, 3000, 0)])
def test_random_frames_fuzz(gpu, oracle, seed, pool, port):
    """Random frames (_fuzz_trace) through one batch and through three batches of a
    kept table: records, hashes, ids, counters and the table bit-exact vs the oracle
    (pool 40: a small context — two table generations, the fused rank; pool 0: a
    distinct key per accepted frame)."""
    n = 300_000
    tr = _fuzz_trace(seed, n, pool, port)
    orc = oracle.parse(tr, filter_port=port)
    nf = max(len(orc[4]), 16)
    cap = 256 if pool == 40 else nf + 64
    with tcbee_amd.PacketParser(max_frames=n, max_arena=len(tr.arena), max_flows=cap) as p:
        assert_same(p.parse(tr, filter_port=port), orc, p.flows())
        assert p.status() == 0
        p.reset_flows()
        ft = oracle.new_flowtab(1 << 20)
        base = 0
        try:
            for lo, hi in [(0, 1000), (1000, 123_457), (123_457, n)]:
                part = tr.select(np.arange(lo, hi))
                o = oracle.parse(part, ft=ft, record_base=base, filter_port=port)
                assert_same(p.parse(part, filter_port=port), o)
                base += len(o[0])
            assert np.array_equal(p.flows(), oracle.flows(ft))
        finally:
            oracle.free_flowtab(ft)
        assert p.status() == 0
