"""Host-side callers of the record path (libtcbee_host.so, include/tcbee_host.h):
pcap ingest, .tcp files, the tcbee-process stage + SQLite sink, metrics.json.

CPU only. The sink is checked against oracle/process_ref.py (a statement-level
restatement of tcbee-process + ts-storage issuing the reference's own SQL) by
comparing whole database dumps; the SQL semantics themselves are pinned by the
reference's committed ts-storage/db.sqlite (tests/golden/ts_storage_db.json).
"""
from __future__ import annotations

import json
import os
import struct
import sys

import numpy as np
import pytest

import tcbee_amd
from tcbee_amd import host
from tcbee_amd.trace import Trace
from tracegen import mixed_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import process_ref  # noqa: E402  (test infrastructure only)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REC = struct.Struct("<QII16s16sHHIIH6BH4s")
FF = b"\xff\xff\xff\xff"


def rec(time=1, saddr=0x0A000001, daddr=0x0A000002, s6=bytes(16), d6=bytes(16), sport=1234,
        dport=5201, seq=1, ack=1, window=1, flags=(0, 0, 0, 0, 0, 0), check=1, div=FF) -> bytes:
    return REC.pack(time, saddr, daddr, s6, d6, sport, dport, seq, ack, window, *flags, check, div)


def oracle_records(oracle, n=4000, seed=3, n_flows=48):
    t = mixed_trace(n, seed=seed, n_flows=n_flows)
    r, fh, fi, ctr, table = oracle.parse(t)
    return r.reshape(-1).tobytes(), fi


def key_ids(records: bytes) -> np.ndarray:
    """Dense ids by first appearance of the record's address/port bytes — the ids a
    GPU flow table assigns (one id per eBPF IpTuple key)."""
    keys: dict = {}
    n = len(records) // 74
    ids = np.zeros(n, np.uint32)
    for i in range(n):
        ids[i] = keys.setdefault(bytes(records[74 * i + 8:74 * i + 52]), len(keys))
    return ids


def sink_dump(tmp_path, name, feed, durable=False):
    path = str(tmp_path / f"{name}.sqlite")
    s = host.Sink(path, durable=durable)
    err = None
    try:
        feed(s)
    except tcbee_amd.TcbeeError as e:
        err = e.code
    st = s.close()
    return process_ref.dump_db(path), st, err


def oracle_dump(tmp_path, name, records):
    path = str(tmp_path / f"{name}.sqlite")
    try:
        st = process_ref.process_records(records, path)
        err = None
    except process_ref.MarkerPanic:
        st, err = None, tcbee_amd._lib.EFORMAT
    return process_ref.dump_db(path), st, err


# ---- library -------------------------------------------------------------------
def test_host_library_exports_every_symbol():
    L = host.hlib()
    for name in host.HOST_EXPORTED:
        assert hasattr(L, name), name
    assert L.tcbee_host_abi_version() == 2
    hdr = open(os.path.join(ROOT, "include", "tcbee_host.h")).read()
    for name in host.HOST_EXPORTED:
        assert name + "(" in hdr, name


# ---- .tcp decode -----------------------------------------------------------------
def test_decode_matches_oracle(oracle):
    records, _ = oracle_records(oracle, 3000, seed=5)
    pk, nd = host.decode_records(records)
    assert nd == 0 and len(pk) == len(records) // 74
    for i in range(0, len(pk), 7):
        r = records[74 * i:74 * i + 74]
        o = oracle.decode(r)
        p = process_ref.decode(r)
        assert o["decoded"] and o["marker_ok"]
        assert int(pk[i]["time"]) == o["time"] == p["time"]
        assert int(pk[i]["seq"]) == p["seq"] and int(pk[i]["checksum"]) == p["checksum"]
        assert host.packet_tuple(pk[i]) == process_ref.get_ip_tuple(p)
        assert o["tuple"][2:] == host.packet_tuple(pk[i])[2:]


def test_decode_invalid_bool_falls_back_to_default():
    good = rec(seq=7)
    bad = rec(flags=(0, 2, 0, 0, 0, 0))
    pk, nd = host.decode_records(good + bad + good)
    assert nd == 1
    assert int(pk[1]["time"]) == 0 and bytes(pk[1]["div"]) == bytes(4)
    assert int(pk[2]["seq"]) == 7
    assert host.check_records(good + bad + good) == 1
    assert host.check_records(good + good) == 2
    assert host.check_records(good + rec(div=b"\xff\xff\xff\xfe")) == 1


@pytest.mark.parametrize("addr,text", [
    ("::", "::"), ("::1", "::1"), ("2001:db8::1", "2001:db8::1"),
    ("2001:db8:0:0:1:0:0:1", "2001:db8::1:0:0:1"),        # first longest run wins
    ("2001:0:0:1:0:0:0:1", "2001:0:0:1::1"),              # the longer run wins
    ("1:0:1:0:1:0:1:0", "1:0:1:0:1:0:1:0"),               # single zeros stay
    ("::ffff:10.0.0.1", "::ffff:10.0.0.1"),               # v4-mapped, dotted
    ("::10.0.0.1", "::a00:1"),                            # v4-compatible: plain hex
    ("fe80::abcd:0:0:1", "fe80::abcd:0:0:1"), ("1::", "1::"),
])
def test_ipv6_display_like_rust(addr, text):
    import ipaddress
    b = ipaddress.IPv6Address(addr).packed
    pk, _ = host.decode_records(rec(saddr=0, s6=b, d6=b))
    src, dst, *_ = host.packet_tuple(pk[0])
    assert src == dst == text == process_ref.rust_ipv6(b)


def test_zero_v4_address_is_keyed_as_ipv6():
    pk, _ = host.decode_records(rec(saddr=0, daddr=0x0A000002))
    assert host.packet_tuple(pk[0]) == ("::", "::", 1234, 5201, 6)
    pk, _ = host.decode_records(rec(saddr=0x0A000001, daddr=0x0A000002))
    assert host.packet_tuple(pk[0]) == ("10.0.0.1", "10.0.0.2", 1234, 5201, 6)


# ---- pcap -------------------------------------------------------------------------
@pytest.mark.parametrize("ns", [True, False])
def test_pcap_round_trip(tmp_path, ns):
    t = mixed_trace(3000, seed=11)
    if not ns:
        t.ts_ns[:] = t.ts_ns // 1000 * 1000
    p = str(tmp_path / "a.pcap")
    host.write_pcap(p, t, nanosecond=ns)
    with host.Pcap(p) as pc:
        assert pc.info["n"] == t.n and pc.info["nanosecond"] == int(ns)
        assert pc.info["truncated"] == 0 and pc.info["linktype"] == 1
        v = pc.trace()
        assert np.array_equal(v.caplen, t.caplen) and np.array_equal(v.ts_ns, t.ts_ns)
        for i in range(t.n):
            assert v.frame(i) == t.frame(i)


def _pcap_bytes(frames, big_endian=False, ns=False, linktype=1):
    e = ">" if big_endian else "<"
    out = struct.pack(e + "IHHiIII", 0xA1B23C4D if ns else 0xA1B2C3D4, 2, 4, 0, 0, 65535,
                      linktype)
    for i, f in enumerate(frames):
        out += struct.pack(e + "IIII", 100 + i, 500 * i, len(f), len(f)) + f
    return out


def test_pcap_swapped_truncated_and_rejects(tmp_path):
    frames = [bytes(range(i % 200, i % 200 + 60)) for i in range(5)]
    p = tmp_path / "be.pcap"
    p.write_bytes(_pcap_bytes(frames, big_endian=True))
    with host.Pcap(str(p)) as pc:
        assert pc.info["swapped"] == 1 and pc.n == 5
        v = pc.trace()
        assert [v.frame(i) for i in range(5)] == frames
        assert list(v.ts_ns) == [(100 + i) * 10**9 + 500 * i * 1000 for i in range(5)]
    p.write_bytes(_pcap_bytes(frames)[:-7])                     # cut into the last frame
    with host.Pcap(str(p)) as pc:
        assert pc.n == 4 and pc.info["truncated"] == 1
    p.write_bytes(_pcap_bytes([]))
    with host.Pcap(str(p)) as pc:
        assert pc.n == 0
    p.write_bytes(_pcap_bytes(frames, linktype=113))            # Linux SLL: not Ethernet
    with pytest.raises(tcbee_amd.TcbeeError) as e:
        host.Pcap(str(p))
    assert e.value.code == tcbee_amd._lib.EFORMAT
    p.write_bytes(b"\x0a\x0d\x0d\x0a" + bytes(40))              # pcapng
    with pytest.raises(tcbee_amd.TcbeeError):
        host.Pcap(str(p))


def test_pcap_feeds_oracle_identically(tmp_path, oracle):
    t = mixed_trace(2000, seed=12)
    p = str(tmp_path / "m.pcap")
    host.write_pcap(p, t)
    with host.Pcap(p) as pc:
        a = oracle.parse(pc.trace())[0]
    b = oracle.parse(t)[0]
    assert np.array_equal(a, b)


# ---- .tcp writer ---------------------------------------------------------------------
def test_tcpfile_append_and_buffering(tmp_path, oracle):
    records, _ = oracle_records(oracle, 2000, seed=6)
    path = str(tmp_path / "xdp.tcp")
    with open(path, "wb") as f:
        f.write(b"PRE")                                          # append, never truncate
    with host.TcpFile(path, buffer_bytes=74 * 5 + 3) as w:       # odd buffer: every path
        pos = 0
        for k in (1, 3, 7, 0, 20, 2):
            w.append(records[pos:pos + 74 * k])
            pos += 74 * k
        w.append(records[pos:])
    assert open(path, "rb").read() == b"PRE" + records


# ---- metrics.json ------------------------------------------------------------------
def test_metrics_json(tmp_path):
    prefix = str(tmp_path) + "/run_"
    p = host.write_metrics(prefix, {"ingress": 5, "egress": (1 << 32) + 3, "handled": 8,
                                    "dropped": 0})
    assert open(p).read() == ('{"handled":8,"dropped":0,"ingress":5,"egress":3,'
                              '"ingress_calls":0,"egress_calls":0}')
    assert json.load(open(p))["egress"] == 3


# ---- sink vs oracle ------------------------------------------------------------------
def test_sink_matches_oracle_mixed(tmp_path, oracle):
    records, ids = oracle_records(oracle, 6000, seed=21)
    o, ost, _ = oracle_dump(tmp_path, "o", records)
    a, ast, err = sink_dump(tmp_path, "a", lambda s: s.packets(records))
    assert err is None and a == o
    assert ast == ost
    assert len(o["flows"]) > 10 and len(o["time_series_data"]) > 1000
    # grouped path with the oracle's dense flow ids (what the GPU produces)
    g, gst, err = sink_dump(tmp_path, "g", lambda s: s.packets_grouped(records, ids))
    assert err is None and g == o and gst == ost
    # per-statement commits: same content
    d, _, err = sink_dump(tmp_path, "d", lambda s: s.packets(records), durable=True)
    assert err is None and d == o


def _wedge_records():
    """Two flows; flow A has a repeated timestamp inside its 2nd 1001-point batch
    (rejected -> SEQ wedged: later events lose ACK/WINDOW/CHECKSUM too, except
    events with seq 0), flow B a repeat inside its last (flush) batch. Plus flag
    records, zero-address v4 records and a v6 flow."""
    out = []
    for i in range(4200):
        t = 1000 + i
        if i == 1500:
            t = 1000 + 1200                                      # duplicate in batch 2
        seq = 0 if i % 97 == 0 else i + 1
        out.append(rec(time=t, seq=seq, ack=i % 5, window=(i * 7) % 3, check=i & 0xFFFF,
                       sport=1111))
        if i % 3 == 0:
            tb = 50_000 + i
            if i == 4197:
                tb = 50_000 + 4194
            out.append(rec(time=tb, saddr=0x0B000001, sport=2222, seq=i, ack=i + 1,
                           flags=(i % 2, 1, 0, 0, i % 5 == 0, 0)))
        if i % 11 == 0:
            out.append(rec(time=90_000 + i, saddr=0, daddr=0x0A000002, sport=3333))
            out.append(rec(time=90_000 + i, saddr=0x0A000001, daddr=0, sport=3333))
        if i % 13 == 0:
            out.append(rec(time=70_000 + i, saddr=0, daddr=0, s6=bytes(15) + b"\x01",
                           d6=b"\x20\x01\x0d\xb8" + bytes(11) + b"\x02", sport=4444, seq=i))
    return b"".join(out)


def test_sink_wedge_and_flags_match_oracle(tmp_path):
    records = _wedge_records()
    o, ost, _ = oracle_dump(tmp_path, "o", records)
    assert ost["failed_batches"] >= 2 and ost["failed_records"] > 0
    a, ast, err = sink_dump(tmp_path, "a", lambda s: s.packets(records))
    assert err is None and a == o and ast == ost
    ids = key_ids(records)
    g, gst, err = sink_dump(tmp_path, "g", lambda s: s.packets_grouped(records, ids))
    assert err is None and g == o and gst == ost
    # (a rejected full batch is one multi-row statement rolled back whole; per-statement
    #  commits too)
    d, dst, err = sink_dump(tmp_path, "d", lambda s: s.packets(records), durable=True)
    assert err is None and d == o and dst == ost
    flagged = [r for r in o["time_series_data"] if r[2] == 1]
    assert flagged, "FLAG_* points land in value_boolean"


def test_sink_marker_failure_matches_oracle_panic(tmp_path):
    good = _wedge_records()[:74 * 3000]
    records = good + rec(div=bytes(4)) + good[:74 * 10]
    o, _, oerr = oracle_dump(tmp_path, "o", records)
    assert oerr == tcbee_amd._lib.EFORMAT
    a, _, err = sink_dump(tmp_path, "a", lambda s: s.packets(records))
    assert err == tcbee_amd._lib.EFORMAT and a == o
    g, _, err = sink_dump(tmp_path, "g", lambda s: s.packets_grouped(records, key_ids(records)))
    assert err == tcbee_amd._lib.EFORMAT and g == o


def test_sink_split_calls_equal_one_call(tmp_path, oracle):
    records, ids = oracle_records(oracle, 5000, seed=22)
    o, _, _ = oracle_dump(tmp_path, "o", records)
    cut = 74 * 2345

    def feed(s):
        s.packets_grouped(records[:cut], ids[:cut // 74], int(ids.max()) + 1)
        s.packets(records[cut:])
    a, _, err = sink_dump(tmp_path, "a", feed)
    assert err is None and a == o


def test_process_files_matches_oracle(tmp_path, oracle):
    r1, _ = oracle_records(oracle, 3000, seed=31)
    r2, _ = oracle_records(oracle, 2000, seed=32)
    src = str(tmp_path) + "/rec_"
    open(src + "xdp.tcp", "wb").write(r1 + b"\xff\xff")          # partial tail entry ignored
    open(src + "tc.tcp", "wb").write(r2)
    st = host.process_files(src, str(tmp_path / "a.sqlite"))
    ost = process_ref.process_files(src, str(tmp_path / "o.sqlite"))
    assert st == ost
    assert process_ref.dump_db(str(tmp_path / "a.sqlite")) == \
        process_ref.dump_db(str(tmp_path / "o.sqlite"))


def test_process_files_missing_inputs(tmp_path):
    st = host.process_files(str(tmp_path) + "/none_", str(tmp_path / "e.sqlite"))
    assert st["records"] == 0
    d = process_ref.dump_db(str(tmp_path / "e.sqlite"))
    assert d["flows"] == [] and d["time_series"] == []


# ---- ts-storage fixture --------------------------------------------------------------
def test_ts_storage_fixture_replay(tmp_path):
    """Replays ts-storage/tests/sqlite.rs.rs `all_func` through the sink's ts-storage
    primitives; the result must equal the reference's committed db.sqlite."""
    fx = json.load(open(os.path.join(GOLDEN, "ts_storage_db.json")))
    path = str(tmp_path / "db.sqlite")
    s = host.Sink(path)
    tup = ("10.0.0.1", "10.0.0.2", 100, 200, 16)
    f1 = s.create_flow(*tup)
    s.delete_flow(*tup)
    f2 = s.create_flow(*tup)
    s.add_attribute(f2, "TEST", host.T_TEXT, "TEST")
    s.set_attribute(f2, "TEST", host.T_INT, 100)
    s.add_attribute(f2, "TEST2", host.T_TEXT, "TEST")
    s.delete_attribute(f2, "TEST")
    s.delete_attribute(f2, "TEST2")
    s.delete_flow(*tup)
    f3 = s.create_flow(*tup)
    assert (f1, f2, f3) == (1, 2, 3)
    ts1 = s.create_series(f3, "TestTS", host.T_INT)
    assert s.insert_points(ts1, host.T_INT, [0.0], [10])            # insert_data_point
    assert s.insert_points(ts1, host.T_INT, [0.5, 1.0, 2.0, 3.0], [10, 11, 12, 13])
    assert not s.insert_points(ts1, host.T_INT, [99.0, 99.0], [1, 2])  # rejected whole
    assert s.insert_points(ts1, host.T_INT, [99.0, 100.0], [3, 4])
    s.close()
    got = process_ref.dump_db(path)
    want = {k: [list(r) for r in v] for k, v in fx["rows"].items()}
    assert got == want
    # schema: same columns / defaults / keys / unique sets / foreign keys
    sys.path.insert(0, GOLDEN)
    import sqlite3

    import make_tsdb_fixture
    c = sqlite3.connect(path)
    assert json.loads(json.dumps(make_tsdb_fixture.schema(c))) == fx["schema"]
    c.close()


def test_oracle_replays_fixture_too(tmp_path):
    """The Python restatement issues the reference SQL; it must land on the same DB."""
    fx = json.load(open(os.path.join(GOLDEN, "ts_storage_db.json")))
    path = str(tmp_path / "db.sqlite")
    db = process_ref.RefTSDB(path)
    tup = ("10.0.0.1", "10.0.0.2", 100, 200, 16)
    db.create_flow(tup)
    db.delete_flow(tup)
    f2 = db.create_flow(tup)
    db.add_flow_attribute(f2, "TEST", 3, "TEST")
    db.set_flow_attribute(f2, "TEST", 0, 100)
    db.add_flow_attribute(f2, "TEST2", 3, "TEST")
    db.delete_flow_attribute(f2, "TEST")
    db.delete_flow_attribute(f2, "TEST2")
    db.delete_flow(tup)
    f3 = db.create_flow(tup)
    ts1 = db.create_time_series(f3, "TestTS", 0)
    db.insert_data_point(ts1, 0, 0.0, 10)
    db.insert_multiple_points(ts1, 0, [(0.5, 10), (1.0, 11), (2.0, 12), (3.0, 13)])
    import sqlite3
    with pytest.raises(sqlite3.IntegrityError):
        db.insert_multiple_points(ts1, 0, [(99.0, 1), (99.0, 2)])
    db.insert_multiple_points(ts1, 0, [(99.0, 3), (100.0, 4)])
    db.close()
    assert process_ref.dump_db(path) == {k: [list(r) for r in v] for k, v in fx["rows"].items()}


def test_config1_loopback_trace_through_sink(oracle, tmp_path):
    """Config 1's shape on the CPU side: the loopback iperf3 capture's oracle records
    (both hooks; flags always 0 despite SYN/FIN) through the tcbee-process stage
    (xdp.tcp then tc.tcp) equal process_ref's database: two flows, no flag series."""
    import numpy as np

    from tracegen import iperf3_loopback_trace
    from tcbee_amd.trace import Trace
    t = iperf3_loopback_trace(4000)
    t2 = Trace(t.arena, t.offset, t.caplen, t.ts_ns - np.uint64(1500))
    rx, rt = oracle.parse(t), oracle.parse(t2, direction=1)
    assert len(rx[0]) == len(rt[0]) == t.n and len(rx[4]) == 2
    assert not rx[0][:, 62:68].any()
    prefix = str(tmp_path) + "/lo_"
    open(prefix + "xdp.tcp", "wb").write(rx[0].tobytes())
    open(prefix + "tc.tcp", "wb").write(rt[0].tobytes())
    host.process_files(prefix, str(tmp_path / "g.sqlite"))
    process_ref.process_records(rx[0].tobytes() + rt[0].tobytes(), str(tmp_path / "o.sqlite"))
    got = process_ref.dump_db(str(tmp_path / "g.sqlite"))
    assert got == process_ref.dump_db(str(tmp_path / "o.sqlite"))
    assert [r[1:] for r in got["flows"]][0][3:] == [5201, 6]
    names = {r[2] for r in got["time_series"]}
    assert not any(n.startswith("FLAG_") for n in names)


def test_compiled_c_host_builds_and_refuses_without_gpu(tmp_path):
    """tcbee-record-gpu (tcbee_amd/host/tcbee_record_gpu.c) links against the two C
    ABIs only; usage errors exit 2, and without a GPU the pipe creation fails loudly
    (exit 1, the ABI's error text) instead of falling back to anything."""
    import subprocess
    exe = os.path.join(ROOT, "tcbee_amd", "bin", "tcbee-record-gpu")
    assert os.access(exe, os.X_OK)
    assert subprocess.run([exe], capture_output=True).returncode == 2
    if tcbee_amd.device_count() > 0:
        pytest.skip("GPU present (tests/test_gpu_pipeline.py runs it)")
    tr = tcbee_amd.synth_trace(100, sizes="64")
    pcap = str(tmp_path / "t.pcap")
    host.write_pcap(pcap, tr)
    r = subprocess.run([exe, pcap, str(tmp_path) + "/x_"], capture_output=True, text=True)
    assert r.returncode == 1 and "pipe_create" in r.stderr
