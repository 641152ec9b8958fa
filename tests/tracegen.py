"""Adversarial mixed traces for parity tests (seeded, vectorised numpy).

Frames of every class the hook distinguishes, at arbitrary byte alignments:
IPv4/TCP (IHL 5 and 6..15), IPv6/TCP, IPv6 with a hop-by-hop header, IPv4/UDP,
ARP, VLAN-tagged, unknown ethertypes, and runts around every length check
(13/14/23/24/33/34/53/54/73/74 B). Flows are drawn from a small pool so the
flow table sees repeats, and a slice of IPv6 frames carries v4-compatible
addresses that collide with IPv4 keys on purpose.
"""
from __future__ import annotations

import numpy as np

from tcbee_amd.trace import TS_BASE_NS, TS_STEP_NS, Trace

CLASSES = ["v4tcp", "v4tcp_opts", "v6tcp", "v6hop", "v4udp", "arp", "vlan", "other", "runt"]
PROBS = [0.40, 0.07, 0.18, 0.04, 0.09, 0.04, 0.04, 0.04, 0.10]
RUNT_LENS = np.array([0, 1, 12, 13, 14, 15, 20, 21, 23, 24, 33, 34, 53, 54, 55, 73, 74, 75],
                     dtype=np.int64)


def mixed_trace(n: int, seed: int = 1, n_flows: int = 64, max_gap: int = 3,
                filter_hits: int = 5201) -> Trace:
    rng = np.random.default_rng(seed)
    cls = rng.choice(len(CLASSES), size=n, p=PROBS)
    # lengths
    ln = rng.integers(54, 220, size=n)
    is_v6 = (cls == 2) | (cls == 3)
    ln[is_v6] = rng.integers(74, 240, size=int(is_v6.sum()))
    runt = cls == 8
    ln[runt] = RUNT_LENS[rng.integers(0, len(RUNT_LENS), size=int(runt.sum()))]
    ln[cls == 1] = rng.integers(58, 230, size=int((cls == 1).sum()))
    # a few exact-boundary v4/v6 frames that ARE TCP (runts carry valid headers)
    gap = rng.integers(0, max_gap + 1, size=n)
    off = np.zeros(n, dtype=np.int64)
    if n:
        off[1:] = np.cumsum(ln[:-1] + gap[:-1])
    total = int(off[-1] + ln[-1]) if n else 0
    arena = rng.integers(0, 256, size=total + 256, dtype=np.uint8)

    def put(idx, rel, val):
        """arena[off[idx] + rel] = val (uint8), only where the byte is inside the frame
        is irrelevant: headers are written regardless (frames are zero-copy views)."""
        if len(idx) == 0:
            return
        arena[off[idx] + rel] = np.asarray(val, dtype=np.int64).astype(np.uint8)

    def put16(idx, rel, val):
        val = np.asarray(val, dtype=np.int64)
        put(idx, rel, (val >> 8) & 0xFF)
        put(idx, rel + 1, val & 0xFF)

    def put32(idx, rel, val):
        val = np.asarray(val, dtype=np.int64)
        for k in range(4):
            put(idx, rel + k, (val >> (24 - 8 * k)) & 0xFF)

    # flow pool
    f = rng.integers(0, n_flows, size=n)
    fsa = rng.integers(0, 2**32, size=n_flows, dtype=np.int64)
    fsa[: max(1, n_flows // 16)] = 0  # some saddr 0.0.0.0 (KAT-7 class)
    fda = rng.integers(1, 2**32, size=n_flows, dtype=np.int64)
    fsp = rng.integers(0, 65536, size=n_flows)
    fdp = rng.integers(0, 65536, size=n_flows)
    fdp[: n_flows // 4] = filter_hits
    fsp[n_flows // 4: n_flows // 3] = filter_hits
    fv6 = rng.integers(0, 256, size=(n_flows, 32), dtype=np.int64)
    fv6[: n_flows // 8, :12] = 0       # v4-compatible addresses (collide with v4 keys)
    fv6[: n_flows // 8, 16:28] = 0
    fv6[: n_flows // 8, 12:16] = np.stack([(fsa[: n_flows // 8] >> s) & 0xFF
                                           for s in (24, 16, 8, 0)], 1)
    fv6[: n_flows // 8, 28:32] = np.stack([(fda[: n_flows // 8] >> s) & 0xFF
                                           for s in (24, 16, 8, 0)], 1)

    idx_all = np.arange(n)
    # ethertypes
    v4 = idx_all[(cls == 0) | (cls == 1) | (cls == 4) | (runt & (rng.random(n) < 0.6))]
    v6 = idx_all[is_v6 | (runt & ~np.isin(idx_all, v4))]
    put16(v4, 12, 0x0800)
    put16(v6, 12, 0x86DD)
    put16(idx_all[cls == 5], 12, 0x0806)
    put16(idx_all[cls == 6], 12, 0x8100)
    put16(idx_all[cls == 7], 12, rng.choice([0x88CC, 0x0801, 0x86DC, 0x0000, 0xFFFF],
                                             size=int((cls == 7).sum())))
    # IPv4 headers (frame byte 14..33)
    ihl = np.full(n, 5)
    ihl[cls == 1] = rng.integers(6, 16, size=int((cls == 1).sum()))
    put(v4, 14, 0x40 | ihl[v4])
    put(v4, 23, np.where(cls[v4] == 4, 17, 6))
    put32(v4, 26, fsa[f[v4]])
    put32(v4, 30, fda[f[v4]])
    # IPv6 headers
    put(v6, 14, 0x60)
    put(v6, 20, np.where(cls[v6] == 3, 0, 6))
    for k in range(32):
        put(v6, 22 + k, fv6[f[v6], k])
    # TCP ports at 34 (v4) / 54 (v6) from the flow
    put16(v4, 34, fsp[f[v4]])
    put16(v4, 36, fdp[f[v4]])
    put16(v6, 54, fsp[f[v6]])
    put16(v6, 56, fdp[f[v6]])

    ts = np.uint64(TS_BASE_NS) + np.uint64(TS_STEP_NS) * np.arange(n, dtype=np.uint64)
    return Trace(arena[:total], off.astype(np.uint64), ln.astype(np.uint32), ts)


def iperf3_loopback_trace(n: int = 10_000, seed: int = 5201, snaplen: int = 96,
                          ts0: int = 5_000_000_000_000, gap_ns: int = 800) -> Trace:
    """A loopback iperf3 TCP transfer as `tcpdump -i lo -s <snaplen>` would capture
    it (config 1 of BASELINE.json: tcbee-record/run.sh:2 records `lo` while iperf3
    runs): all-zero MACs, 127.0.0.1 both ends, ONE connection (two IpTuples,
    client->server data and server->client ACKs): SYN / SYN-ACK / ACK with
    option-bearing headers (doff 10 / 8), PSH-ACK data segments of lo's 65483-B
    MSS (captured to `snaplen`), an ACK every second segment, FIN-ACK / FIN-ACK /
    ACK at the end. Timestamps are ktime-like (ns since boot)."""
    rng = np.random.default_rng(seed)
    cport, sport = 40_000 + int(rng.integers(0, 20_000)), 5201
    isn_c, isn_s = (int(x) for x in rng.integers(0, 2**32, size=2))
    mss = 65483 - 12
    frames = []  # (dir 0 = client->server, flags, seq, ack, tcp_hdr_len, payload)
    frames.append((0, 0x02, isn_c, 0, 40, 0))
    frames.append((1, 0x12, isn_s, (isn_c + 1) % 2**32, 40, 0))
    frames.append((0, 0x10, isn_c + 1, isn_s + 1, 32, 0))
    seq_c, seq_s = isn_c + 1, isn_s + 1
    k = 0
    while len(frames) < n - 3:
        frames.append((0, 0x18, seq_c % 2**32, seq_s % 2**32, 32, mss))
        seq_c += mss
        k += 1
        if k % 2 == 0 and len(frames) < n - 3:
            frames.append((1, 0x10, seq_s % 2**32, seq_c % 2**32, 32, 0))
    frames.append((0, 0x11, seq_c % 2**32, seq_s % 2**32, 32, 0))
    frames.append((1, 0x11, seq_s % 2**32, (seq_c + 1) % 2**32, 32, 0))
    frames.append((0, 0x10, (seq_c + 1) % 2**32, (seq_s + 1) % 2**32, 32, 0))
    out = []
    ip_id = [int(rng.integers(0, 65536)), int(rng.integers(0, 65536))]
    for d, flags, seq, ack, th, pay in frames:
        flen = 14 + 20 + th + pay
        tot = 20 + th + pay
        b = bytearray(min(flen, snaplen))
        hdr = bytearray(14 + 20 + th)
        hdr[12:14] = b"\x08\x00"                       # MACs stay zero on lo
        ip = bytearray(20)
        ip[0], ip[1] = 0x45, 0
        ip[2:4] = tot.to_bytes(2, "big") if tot < 65536 else b"\xff\xff"
        ip[4:6] = (ip_id[d] & 0xFFFF).to_bytes(2, "big")
        ip_id[d] += 1
        ip[6:8] = b"\x40\x00"                          # DF
        ip[8], ip[9] = 64, 6
        ip[12:16] = bytes([127, 0, 0, 1])
        ip[16:20] = bytes([127, 0, 0, 1])
        s = sum(int.from_bytes(ip[j:j + 2], "big") for j in range(0, 20, 2))
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        ip[10:12] = (~s & 0xFFFF).to_bytes(2, "big")
        hdr[14:34] = ip
        t = bytearray(th)
        t[0:2] = (cport if d == 0 else sport).to_bytes(2, "big")
        t[2:4] = (sport if d == 0 else cport).to_bytes(2, "big")
        t[4:8] = seq.to_bytes(4, "big")
        t[8:12] = ack.to_bytes(4, "big")
        t[12] = (th // 4) << 4
        t[13] = flags
        t[14:16] = (65495 if flags & 0x02 else 512).to_bytes(2, "big")
        t[16:18] = int(rng.integers(0, 65536)).to_bytes(2, "big")  # lo: partial checksum
        if th > 20:
            t[20:22] = b"\x01\x01"                     # NOP NOP
            t[22:24] = b"\x08\x0a"                     # timestamps option
            t[24:28] = int(rng.integers(0, 2**32)).to_bytes(4, "big")
        hdr[34:34 + th] = t
        m = min(len(hdr), len(b))
        b[:m] = hdr[:m]
        out.append(bytes(b))
    ts = np.uint64(ts0) + np.uint64(gap_ns) * np.arange(len(out), dtype=np.uint64)
    return Trace.from_frames(out, ts_ns=ts)
