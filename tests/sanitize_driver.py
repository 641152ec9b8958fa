"""Runs inside a child process with the sanitizer runtime preloaded (see
tests/test_sanitize.py): drives the ASan/UBSan builds of libtcbee_host and of the
oracle over valid, truncated and malformed inputs. Any sanitizer report aborts
the process; a clean run prints SANITIZE_OK."""
import os
import struct
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
os.environ.setdefault("TCBEE_NO_TORCH", "1")

from oracle_py import Oracle  # noqa: E402
from tracegen import iperf3_loopback_trace, mixed_trace  # noqa: E402

from tcbee_amd import host  # noqa: E402
from tcbee_amd._lib import TcbeeError  # noqa: E402
from tcbee_amd.trace import Trace  # noqa: E402


def expect_error(fn, *a):
    try:
        fn(*a)
    except (TcbeeError, OSError, ValueError):
        return
    # some malformed inputs are legal (e.g. a truncated tail is counted, not refused)


def pcap_cases(d, rng):
    tr = mixed_trace(3000, seed=11, n_flows=50)
    good = os.path.join(d, "good.pcap")
    host.write_pcap(good, tr)
    raw = open(good, "rb").read()
    paths = []
    # every cut inside the global header and the first records, then random cuts
    cuts = list(range(0, 120)) + sorted(rng.integers(120, len(raw), size=60).tolist())
    for k, c in enumerate(cuts):
        p = os.path.join(d, f"cut{k}.pcap")
        open(p, "wb").write(raw[:c])
        paths.append(p)
    # record headers with absurd caplen / garbage bodies
    for k in range(40):
        b = bytearray(raw[:24 + 16 * 3 + 200])
        pos = 24 + int(rng.integers(0, 64))
        b[pos:pos + 4] = struct.pack("<I", int(rng.integers(0, 2**32)))
        p = os.path.join(d, f"bad{k}.pcap")
        open(p, "wb").write(bytes(b))
        paths.append(p)
    for name, data in (("empty.pcap", b""), ("pcapng.pcap", b"\x0a\x0d\x0d\x0a" + bytes(60)),
                       ("noise.pcap", rng.integers(0, 256, size=4096, dtype=np.uint8).tobytes())):
        p = os.path.join(d, name)
        open(p, "wb").write(data)
        paths.append(p)
    for p in paths:
        try:
            with host.Pcap(p) as pc:
                t = pc.trace()
                if t.n:
                    host.flowhash_owner(t, 3, threads=2)
                    # every frame the index exposes lies inside the mapping
                    assert int((t.offset + t.caplen).max()) <= len(t.arena)
        except TcbeeError:
            pass


def tcp_cases(d, rng, orc):
    tr = mixed_trace(5000, seed=12, n_flows=80)
    rec = orc.parse(tr)[0]
    noise = rng.integers(0, 256, size=(500, 74), dtype=np.uint8)
    flips = rec[:500].copy()
    flips[np.arange(500), rng.integers(0, 74, size=500)] ^= np.uint8(0xFF)
    for blob in (rec, noise, flips, rec[:0]):
        host.decode_records(blob)
        host.check_records(blob)
    # append writer, then the tcbee-process stage over whole, truncated and corrupt files
    prefix = os.path.join(d, "t_")
    with host.TcpFile(prefix + "xdp.tcp") as f:
        f.append(rec)
    open(prefix + "tc.tcp", "wb").write(rec[:100].tobytes()[:-13])  # ragged tail
    host.process_files(prefix, os.path.join(d, "a.sqlite"))
    bad = os.path.join(d, "b_")
    open(bad + "xdp.tcp", "wb").write(np.concatenate([rec[:50], flips[:50]]).tobytes())
    expect_error(host.process_files, bad, os.path.join(d, "b.sqlite"))
    with host.Sink(os.path.join(d, "s.sqlite")) as s:
        s.packets(rec[:1000])
        ids = rng.integers(0, 7, size=1000).astype(np.uint32)
        s.packets_grouped(rec[1000:2000], ids, 7)
        expect_error(s.packets, noise[:10])
    lo = iperf3_loopback_trace(500)
    host.write_metrics(os.path.join(d, "m_"), {"ingress": 2**33, "egress": 1, "handled": 5,
                                                 "dropped": 0})
    host.flowhash_owner(lo, 8, threads=4)


def partition_edges(rng):
    # frames running past the arena end and offsets beyond it: clamped, never read
    tr = mixed_trace(2000, seed=13, n_flows=30)
    off = tr.offset.copy()
    ln = tr.caplen.copy()
    off[::50] = np.uint64(len(tr.arena) + 100)
    ln[1::50] = np.uint32(1 << 20)
    host.flowhash_owner(Trace(tr.arena, off, ln, tr.ts_ns), 5, threads=3)
    edge = Trace(tr.arena, off, ln, tr.ts_ns)
    load = host.flowhash_load(edge, 97, threads=3)  # RSS bucket loads, table routing
    table = (np.arange(97) % 5).astype(np.uint16)
    host.flowhash_owner(edge, 5, threads=3, rss=table)
    assert int(load.sum()) <= edge.n


def oracle_cases(rng, orc):
    for seed in range(3):
        tr = mixed_trace(20000, seed=100 + seed, n_flows=300)
        for fp in (0, 5201):
            for direction in (0, 1):
                orc.parse(tr, filter_port=fp, direction=direction)
                orc.accept_mask(tr, filter_port=fp, direction=direction)
        orc.baseline(tr, threads=4)
        orc.ref_flows(tr)
    ft = orc.new_flowtab(4)  # grows from a tiny capacity
    try:
        orc.parse(mixed_trace(30000, seed=9, n_flows=5000), ft=ft)
    finally:
        orc.free_flowtab(ft)
    for r in rng.integers(0, 256, size=(300, 74), dtype=np.uint8):
        orc.decode(r.tobytes())


def main():
    rng = np.random.default_rng(2025)
    orc = Oracle(os.environ["TCBEE_ORACLE_LIB"])
    with tempfile.TemporaryDirectory() as d:
        pcap_cases(d, rng)
        tcp_cases(d, rng, orc)
    partition_edges(rng)
    oracle_cases(rng, orc)
    maps = open("/proc/self/maps").read()
    loaded = sorted({ln.split()[-1] for ln in maps.splitlines()
                     if "_asan.so" in ln or "libasan" in ln})
    print("LOADED", " ".join(loaded), flush=True)
    print("SANITIZE_OK", flush=True)


if __name__ == "__main__":
    main()
