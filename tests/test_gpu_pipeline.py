"""GPU: the host-frames ingest pipeline (tcbee_pipe) and the end-to-end pcap
replay. Every output is compared with the CPU oracle fed the same frames."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

import tcbee_amd
from tcbee_amd import host
from tcbee_amd.pipeline import Pipeline, replay_pcap
from tracegen import mixed_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import process_ref  # noqa: E402  (test infrastructure only)

pytestmark = pytest.mark.gpu


def check_same(res, orc, flows_gpu=None):
    rec, fh, fi, ctr, table = orc
    assert res.n == len(rec)
    assert np.array_equal(res.records, rec)
    if res.flow_id is not None:
        assert np.array_equal(res.flow_id, fi)
    assert res.counters == ctr
    if flows_gpu is not None:
        assert np.array_equal(flows_gpu, table)


@pytest.mark.parametrize("nt", ["1", "0"])
@pytest.mark.parametrize("window,chunk,depth,threads", [
    (80, 4096, 3, 8), (80, 1000, 4, 1), (0, 4096, 3, 8), (96, 65536, 5, 3), (0, 777, 3, 2),
    (64, 4096, 3, 8), (64, 1000, 4, 1),
])
def test_pipeline_matches_oracle(gpu, oracle, window, chunk, depth, threads, nt, monkeypatch):
    """The product pipe (TCBEE_PIPE_NT=1 behaviour): the header-window gather copies
    whole windows with streaming stores, so the staged bytes past a frame's caplen are
    the NEXT frame's (mixed_trace's arena is random bytes everywhere); the variants
    build with TCBEE_PIPE_NT=0: memcpy of caplen bytes."""
    monkeypatch.setenv("TCBEE_PIPE_NT", nt)
    t = mixed_trace(60_000, seed=100 + chunk, n_flows=300)
    with Pipeline(device=0, chunk_frames=chunk, window=window, depth=depth,
                  threads=threads, max_flows=1 << 12, variants=nt == "0") as p:
        res = p.run(t)
        check_same(res, oracle.parse(t), p.flows())
        st = p.stats()
        assert st["frames"] == t.n and st["chunks"] >= t.n // chunk


@pytest.mark.parametrize("window", [80, 64])
@pytest.mark.parametrize("nt", ["1", "0"])
def test_pipeline_windows_at_arena_end(gpu, oracle, nt, window, monkeypatch):
    """Runts and short frames packed back to back at the very end of the arena: their
    windows run past arena_len, so the gather falls back to a bounded copy (zero
    fill past the arena) for exactly those frames; window 64 starts 12
    bytes into each frame."""
    from tcbee_amd.trace import Trace
    monkeypatch.setenv("TCBEE_PIPE_NT", nt)
    t = mixed_trace(5000, seed=21, n_flows=40)
    rng = np.random.default_rng(3)
    tail = [t.frame(i)[:int(rng.integers(10, 90))] for i in range(200)]
    frames = [t.frame(i) for i in range(t.n)] + tail
    t2 = Trace.from_frames(frames)
    assert int(t2.offset[-1] + t2.caplen[-1]) == len(t2.arena)
    with Pipeline(device=0, chunk_frames=1024, window=window, depth=3, threads=4,
                  max_flows=1 << 12, variants=nt == "0") as p:
        check_same(p.run(t2), oracle.parse(t2), p.flows())


def test_pipeline_whole_frames_byte_budget(gpu, oracle):
    """window 0 with a tiny chunk_bytes: chunks are cut by bytes, not frames."""
    t = mixed_trace(20_000, seed=7)
    with Pipeline(device=0, chunk_frames=1 << 16, window=0, chunk_bytes=64 * 1024) as p:
        res = p.run(t)
        check_same(res, oracle.parse(t), p.flows())
        assert p.stats()["chunks"] > 20


def test_pipeline_filter_egress_noflows(gpu, oracle):
    t = mixed_trace(30_000, seed=8)
    with Pipeline(device=0, chunk_frames=5000) as p:
        res = p.run(t, filter_port=5201, direction=tcbee_amd.DIR_EGRESS)
        check_same(res, oracle.parse(t, filter_port=5201, direction=1))
        res2 = p.run(t, flows=False)
        rec, _, _, ctr, _ = oracle.parse(t, flows=False)
        assert np.array_equal(res2.records, rec) and res2.counters == ctr
        assert res2.flow_id is None


def test_pipeline_calls_continue_flow_ids(gpu, oracle):
    """Two runs on one pipe = one trace: ids continue, like tcbee_parse_batch."""
    t = mixed_trace(40_000, seed=9, n_flows=500)
    a, b = t.slice(0, 17_000), t.slice(17_000, t.n)
    with Pipeline(device=0, chunk_frames=4096) as p:
        ra = p.run(a)
        rb = p.run(b)
        ft = oracle.new_flowtab(4096)
        oa = oracle.parse(a, ft=ft)
        ob = oracle.parse(b, ft=ft, record_base=len(oa[0]))
        table = oracle.flows(ft)
        oracle.free_flowtab(ft)
        assert np.array_equal(ra.flow_id, oa[2]) and np.array_equal(rb.flow_id, ob[2])
        assert np.array_equal(p.flows(), table)


def test_pipeline_sink_callback_and_out_cap(gpu, oracle):
    t = mixed_trace(25_000, seed=10)
    rec, fh, fi, ctr, _ = oracle.parse(t)
    got, ids, firsts = [], [], []
    with Pipeline(device=0, chunk_frames=3000) as p:
        res = p.run(t, collect=False,
                    sink=lambda r, i, first: (got.append(r.copy()), ids.append(i.copy()),
                                              firsts.append(first)))
        assert res.n == len(rec) and res.records is None
        assert np.array_equal(np.concatenate(got), rec)
        assert np.array_equal(np.concatenate(ids), fi)
        assert firsts == list(np.cumsum([0] + [len(g) for g in got[:-1]]))
        small = np.empty((100, 74), np.uint8)
        p.reset_flows()
        with pytest.raises(tcbee_amd.TcbeeError) as e:
            p.run(t, out_rec=small, out_id=np.empty(100, np.uint32))
        assert e.value.code == tcbee_amd._lib.ECAPACITY
        assert np.array_equal(small, rec[:100])


@pytest.mark.parametrize("window", [64, 0])
def test_pipeline_registered_output(gpu, oracle, window):
    """the caller's arrays registered once (tcbee_pipe_register_output):
    chunks DMA straight into them. Records / ids / counters equal the oracle; the
    sink sees the same records (pointers into the caller's arrays); flow ids continue
    across runs; a registered array with a smaller out_cap than the records sends the
    chunk past it through staging (ECAPACITY, the first out_cap written); ids not
    registered (records only) and unregistering fall back to staging, same bytes."""
    t = mixed_trace(50_000, seed=61, n_flows=400)
    rec, fh, fi, ctr, table = oracle.parse(t)
    n = len(rec)
    out = np.zeros((n + 50, 74), np.uint8)
    ids = np.zeros(n + 50, np.uint32)
    with Pipeline(device=0, chunk_frames=4096, window=window, depth=3, threads=4,
                  max_flows=1 << 12) as p:
        p.register_output(out, ids)
        seen = []
        res = p.run(t, out_rec=out, out_id=ids,
                    sink=lambda r, i, first: seen.append((first, r.copy(), i.copy())))
        check_same(res, (rec, fh, fi, ctr, table), p.flows())
        assert not out[n:].any() and not ids[n:].any()
        assert np.array_equal(np.concatenate([r for _, r, _ in seen]), rec)
        assert np.array_equal(np.concatenate([i for _, _, i in seen]), fi)
        # a second run continues the ids; reset: the same bytes again
        p.reset_flows()
        out[:] = 0
        check_same(p.run(t, out_rec=out, out_id=ids), (rec, fh, fi, ctr, table))
        # out_cap below the records: the overflowing chunk goes through staging
        p.reset_flows()
        out[:] = 0
        with pytest.raises(tcbee_amd.TcbeeError) as e:
            p.run(t, out_rec=out[:n - 5000], out_id=ids)
        assert e.value.code == tcbee_amd._lib.ECAPACITY
        assert np.array_equal(out[:n - 5000], rec[:n - 5000]) and not out[n - 5000:].any()
        # records-only registration, then none at all: staging, identical results
        for reg in ((out, None), (None, None)):
            p.register_output(*reg)
            p.reset_flows()
            out[:] = 0
            ids[:] = 0
            check_same(p.run(t, out_rec=out[:n], out_id=ids[:n]), (rec, fh, fi, ctr, table))
        with pytest.raises(ValueError):
            p.register_output(np.zeros((10, 70), np.uint8))


def test_pipeline_shared_registration_and_calibration(gpu, oracle):
    """Round 5: two pipes share ONE registered output pair
    (the second borrows the first's page-locking, and releasing the borrower leaves it
    registered for the owner); calibrate_output times direct D2H against staging on
    a prefix and keeps the faster; whichever it keeps, records / ids / counters / the
    table equal the oracle, and forcing the other mode gives the same bytes."""
    t = mixed_trace(60_000, seed=62, n_flows=500)
    want = oracle.parse(t)
    n = len(want[0])
    out = np.zeros((n, 74), np.uint8)
    ids = np.zeros(n, np.uint32)
    with Pipeline(device=0, chunk_frames=4096, window=64, depth=3, threads=4,
                  max_flows=1 << 12) as owner:
        owner.register_output(out, ids)
        with Pipeline(device=0, chunk_frames=4096, window=64, depth=3, threads=4,
                      max_flows=1 << 12) as b:
            b.register_output(out, ids)  # already page-locked: borrowed
            check_same(b.run(t, out_rec=out, out_id=ids), want, b.flows())
            with pytest.raises(ValueError, match="holds flows"):  # not silently
                b.calibrate_output(t, frames=20_000, reps=1)
            b.reset_flows()
            cal = b.calibrate_output(t, frames=20_000, reps=1)
            assert cal["chosen"] in ("registered", "staged") and cal["frames"] == 20_000
            assert b.output_mode == cal["chosen"]
            assert cal["registered_mpkts"] > 0 and cal["staged_mpkts"] > 0
            out[:] = 0
            ids[:] = 0
            check_same(b.run(t, out_rec=out, out_id=ids), want, b.flows())
            # the other mode, forced: same bytes
            if b.output_mode == "registered":
                b.register_output(None)
            else:
                b.register_output(out, ids)
            b.reset_flows()
            out[:] = 0
            check_same(b.run(t, out_rec=out, out_id=ids), want, b.flows())
        # the borrower is gone: the owner's registration still holds (direct D2H)
        out[:] = 0
        ids[:] = 0
        check_same(owner.run(t, out_rec=out, out_id=ids), want, owner.flows())


def _hip_host_registered(arr: np.ndarray, byte: int = 0) -> bool:
    """hipHostGetFlags on arr's byte `byte` (a variants-build test entry point: the
    query register_output makes, in the HIP runtime the pipes share)."""
    import ctypes as C
    r = C.c_int(0)
    Lv = tcbee_amd._lib.lib(variants=True)
    tcbee_amd._lib.check(Lv.tcbee_test_host_registered(C.c_void_p(arr.ctypes.data + byte),
                                                       C.byref(r)), "host_registered")
    return bool(r.value)


def test_pipeline_registration_refcounted(gpu, oracle):
    """output registrations are process-wide and refcounted. (1) The pipe
    that page-locked a pair is released FIRST: the pair stays page-locked while the
    borrower holds it (its direct D2H runs keep exact outputs) and is unregistered
    when the borrower releases it. (2) A borrower asking for more than the owner
    locked (a larger cap over the same arrays) is refused, not sent past the pinned
    range. (3) A caller's own hipHostRegister is borrowed and never unregistered."""
    t = mixed_trace(40_000, seed=63, n_flows=300)
    want = oracle.parse(t)
    n = len(want[0])
    out = np.zeros((n, 74), np.uint8)
    ids = np.zeros(n, np.uint32)
    kw = dict(device=0, chunk_frames=4096, window=64, depth=3, threads=2, max_flows=1 << 12)
    assert not _hip_host_registered(out)
    owner = Pipeline(**kw)
    owner.register_output(out, ids)
    assert _hip_host_registered(out) and _hip_host_registered(ids)
    with Pipeline(**kw) as b:
        b.register_output(out, ids)
        owner.close()  # the owner goes first
        assert _hip_host_registered(out) and _hip_host_registered(ids)
        check_same(b.run(t, out_rec=out, out_id=ids), want, b.flows())
    assert not _hip_host_registered(out) and not _hip_host_registered(ids)

    half = n // 2
    with Pipeline(**kw) as small, Pipeline(**kw) as big:
        small.register_output(out[:half], ids[:half])
        with pytest.raises(tcbee_amd.TcbeeError) as ei:
            big.register_output(out, ids)  # covers more than the owner page-locked
        assert ei.value.code == tcbee_amd._lib.EINVAL
        big.register_output(out[:half // 2], ids[:half // 2])  # inside it: borrowed
        small.register_output(None)
        assert _hip_host_registered(out)  # big still holds it
    assert not _hip_host_registered(out)

    import torch
    cr = torch.cuda.cudart()
    assert int(cr.cudaHostRegister(out.ctypes.data, out.nbytes, 0)) == 0
    try:
        with Pipeline(**kw) as p:
            p.register_output(out, None)  # the caller's registration: used as is
            check_same(p.run(t, out_rec=out), want)
        assert _hip_host_registered(out)  # and left to the caller
    finally:
        assert int(cr.cudaHostUnregister(out.ctypes.data)) == 0


def test_pipeline_empty_and_tiny(gpu, oracle):
    with Pipeline(device=0, chunk_frames=1024) as p:
        t0 = mixed_trace(0, seed=1)
        r0 = p.run(t0)
        assert r0.n == 0
        t1 = mixed_trace(5, seed=1)
        check_same(p.run(t1), oracle.parse(t1))


def test_replay_pcap_end_to_end(gpu, oracle, tmp_path):
    """pcap -> GPU -> xdp.tcp + SQLite + metrics.json, each equal to the oracle path."""
    t = mixed_trace(30_000, seed=77, n_flows=40)
    # unique timestamps per flow keep the database out of the duplicate-timestamp wedge
    pcap = str(tmp_path / "trace.pcap")
    host.write_pcap(pcap, t)
    prefix = str(tmp_path) + "/run_"
    out = replay_pcap(pcap, prefix, db_path=str(tmp_path / "gpu.sqlite"), chunk_frames=4096)
    rec, fh, fi, ctr, table = oracle.parse(t)
    assert out["records"] == len(rec) and out["counters"] == ctr and out["flows"] == len(table)
    data = open(prefix + "xdp.tcp", "rb").read()
    assert data == rec.tobytes()
    process_ref.process_records(rec.tobytes(), str(tmp_path / "orc.sqlite"))
    assert process_ref.dump_db(str(tmp_path / "gpu.sqlite")) == \
        process_ref.dump_db(str(tmp_path / "orc.sqlite"))
    m = json.load(open(prefix + "metrics.json"))
    assert m == {"handled": ctr["handled"], "dropped": ctr["dropped"],
                 "ingress": ctr["ingress"], "egress": ctr["egress"],
                 "ingress_calls": 0, "egress_calls": 0}
    # the tcbee-process stage over the written file gives the same database again
    host.process_files(prefix, str(tmp_path / "proc.sqlite"))
    assert process_ref.dump_db(str(tmp_path / "proc.sqlite")) == \
        process_ref.dump_db(str(tmp_path / "orc.sqlite"))


def test_config1_loopback_iperf3_replay(gpu, oracle, tmp_path):
    """Config 1 of BASELINE.json (tcbee-record -h on `lo` while iperf3 runs,
    tcbee-record/run.sh:2), replayed: a loopback iperf3 capture — zero MACs, one
    connection = two IpTuples, SYN / SYN-ACK / FIN flags, option-bearing TCP
    headers, 10k frames captured to 96 B — through pcap -> tcbee_pipe -> xdp.tcp
    (XDP ingress) and tc.tcp (TC egress: on lo every packet passes both hooks; the
    egress copy is stamped 1.5 us earlier, as TC egress runs before XDP ingress
    there) -> the tcbee-process stage -> SQLite, each equal to the oracle path.
    The live cross-check against tcbee-record itself needs root, an XDP/TC attach
    and a Rust toolchain: not run."""
    from tracegen import iperf3_loopback_trace
    from tcbee_amd.trace import Trace
    t_in = iperf3_loopback_trace(10_000)
    t_out = Trace(t_in.arena, t_in.offset, t_in.caplen, t_in.ts_ns - np.uint64(1500))
    pin, pout = str(tmp_path / "lo_in.pcap"), str(tmp_path / "lo_out.pcap")
    host.write_pcap(pin, t_in, snaplen=96)
    host.write_pcap(pout, t_out, snaplen=96)
    prefix = str(tmp_path) + "/lo_"
    a = replay_pcap(pin, prefix, direction=tcbee_amd.DIR_INGRESS, chunk_frames=4096)
    b = replay_pcap(pout, prefix, direction=tcbee_amd.DIR_EGRESS, chunk_frames=4096)
    rx = oracle.parse(t_in)
    rt = oracle.parse(t_out, direction=1)
    assert a["records"] == b["records"] == t_in.n
    assert a["counters"] == rx[3] and b["counters"] == rt[3]
    assert a["flows"] == b["flows"] == 2 == len(rx[4])
    assert open(prefix + "xdp.tcp", "rb").read() == rx[0].tobytes()
    assert open(prefix + "tc.tcp", "rb").read() == rt[0].tobytes()
    # the flags quirk: SYN/FIN/PSH/ACK frames all carry six zero flag bytes
    assert not rx[0][:, 62:68].any()
    host.process_files(prefix, str(tmp_path / "gpu.sqlite"))
    process_ref.process_records(rx[0].tobytes() + rt[0].tobytes(), str(tmp_path / "orc.sqlite"))
    got = process_ref.dump_db(str(tmp_path / "gpu.sqlite"))
    assert got == process_ref.dump_db(str(tmp_path / "orc.sqlite"))
    assert len(got["flows"]) == 2 and got["flows"][0][1:] == ["127.0.0.1", "127.0.0.1",
                                                              got["flows"][0][3], 5201, 6]
    m = json.load(open(prefix + "metrics.json"))
    assert m["egress"] == t_in.n and m["handled"] == t_in.n


@pytest.mark.parametrize("egress,port", [(False, 0), (True, 5201)])
def test_compiled_c_host_replay(gpu, oracle, tmp_path, egress, port):
    """tcbee-record-gpu: a compiled C program over the two C ABIs only (no Python in
    the process) — pcap -> tcbee_pipe -> <prefix>xdp.tcp / tc.tcp through the
    buffered .tcp writer -> metrics.json -> the tcbee-process stage into SQLite; the
    bytes, the counters and the database equal the oracle path's (both hooks,
    FILTER_PORT)."""
    import subprocess
    exe = os.path.join(ROOT, "tcbee_amd", "bin", "tcbee-record-gpu")
    t = mixed_trace(40_000, seed=88, n_flows=60)
    pcap = str(tmp_path / "trace.pcap")
    host.write_pcap(pcap, t)
    prefix = str(tmp_path) + "/c_"
    db = str(tmp_path / "c.sqlite")
    args = [exe, "--port", str(port), "--db", db, "--threads", "4"] + (["--tc"] if egress else [])
    r = subprocess.run(args + [pcap, prefix], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    rec, fh, fi, ctr, table = oracle.parse(t, filter_port=port, direction=int(egress))
    assert out["frames"] == t.n and out["records"] == len(rec) and out["flows"] == len(table)
    assert {k: out[k] for k in ("ingress", "egress", "handled", "dropped")} == ctr
    name = "tc.tcp" if egress else "xdp.tcp"
    assert open(prefix + name, "rb").read() == rec.tobytes()
    m = json.load(open(prefix + "metrics.json"))
    assert m == {"handled": ctr["handled"], "dropped": ctr["dropped"], "ingress": ctr["ingress"],
                 "egress": ctr["egress"], "ingress_calls": 0, "egress_calls": 0}
    process_ref.process_records(rec.tobytes(), str(tmp_path / "orc.sqlite"))
    assert process_ref.dump_db(db) == process_ref.dump_db(str(tmp_path / "orc.sqlite"))
