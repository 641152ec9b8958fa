"""Generates tests/golden/kat_vectors.json — known-answer vectors for the
packet-record path, HAND-DERIVED from the reference source (SURVEY.md
Appendix B), not computed by the oracle or by the GPU path.

The reference repository holds no fixtures for this path and cannot be run here
(Rust + eBPF, no toolchain): these vectors are the only anchor of the oracle
("parity unpinned" beyond them). Each expected record below is written out
byte by byte from reading:
  - tcbee-ebpf/src/probes/xdp.rs:27-223, tc.rs:28-183 (accept logic, offsets,
    `.to_be()` byte order, the flag quirk at xdp.rs:105-110)
  - tcbee-common/src/bindings/tcp_header.rs:551-572 (field order)
  - tcbee/src/handlers/mod.rs:126,139 (bincode fixint LE + FF FF FF FF)
  - tcbee-process/src/bindings/tcp_packet.rs:46-111 (downstream decode)

Run:  python tests/golden/make_kat.py   (rewrites the JSON deterministically)
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

ETH_V4 = bytes.fromhex("020000000002" "020000000001" "0800")
ETH_V6 = bytes.fromhex("020000000002" "020000000001" "86dd")


def ipv4(src, dst, proto=6, ihl=5, options=b"", tot=40):
    vihl = 0x40 | ihl
    hdr = struct.pack("!BBHHHBBH4s4s", vihl, 0, tot, 0x1234, 0x4000, 64, proto, 0,
                      bytes(src), bytes(dst))
    return hdr + options


def ipv6(src, dst, nexthdr=6, plen=20):
    return struct.pack("!IHBB16s16s", 0x60000000, plen, nexthdr, 64, bytes(src), bytes(dst))


def tcp(sport, dport, seq, ack, b12, b13, window, check, urg=0):
    return struct.pack("!HHIIBBHHH", sport, dport, seq, ack, b12, b13, window, check, urg)


A1 = [10, 0, 0, 1]
A2 = [10, 0, 0, 2]
V6A = bytes.fromhex("20010db8000000000000000000000001")
V6B = bytes.fromhex("20010db8000000000000000000000002")
T = 0x0102030405060708  # record time stamp (trace ts_ns)
TLE = T.to_bytes(8, "little").hex()

vectors = []


def add(name, frame, expect, filter_port=0, note="", decode=None):
    vectors.append({"name": name, "frame": frame.hex(), "caplen": len(frame), "ts": T,
                    "filter_port": filter_port,
                    "expect": expect, "decode": decode, "note": note})


# KAT-1 IPv4, SYN+ACK (flags byte 0x12) -> all record flags 0 (quirk)
kat1 = ETH_V4 + ipv4(A1, A2) + tcp(12345, 5201, 0x01020304, 0x0A0B0C0D, 0x50, 0x12,
                                   0xFAF0, 0xABCD)
assert len(kat1) == 54
kat1_rec = (TLE + "0100000a" + "0200000a" + "00" * 32 + "3930" + "5114" + "04030201"
            + "0d0c0b0a" + "f0fa" + "00" * 6 + "cdab" + "ffffffff")
add("KAT-1 ipv4 syn-ack", kat1, kat1_rec,
    decode={"tuple": ["10.0.0.1", "10.0.0.2", 12345, 5201, 6],
            "fields": {"SEQ_NUM": 16909060, "ACK_NUM": 168496141, "WINDOW": 64240,
                       "CHECKSUM": 43981}})

# KAT-2 IPv6 PSH+ACK
kat2 = ETH_V6 + ipv6(V6A, V6B) + tcp(443, 50000, 1, 2, 0x50, 0x18, 0x0200, 0x1234)
assert len(kat2) == 74
kat2_rec = (TLE + "00000000" + "00000000" + V6A.hex() + V6B.hex() + "bb01" + "50c3"
            + "01000000" + "02000000" + "0002" + "00" * 6 + "3412" + "ffffffff")
add("KAT-2 ipv6 psh-ack", kat2, kat2_rec,
    decode={"tuple": ["2001:db8::1", "2001:db8::2", 443, 50000, 6],
            "fields": {"SEQ_NUM": 1, "ACK_NUM": 2, "WINDOW": 512, "CHECKSUM": 4660}})

# KAT-3 no record: UDP, ARP, VLAN-tagged IPv4/TCP, unknown ethertype
add("KAT-3 udp", ETH_V4 + ipv4(A1, A2, proto=17) + bytes(20), None)
add("KAT-3 arp", bytes.fromhex("ffffffffffff" "020000000001" "0806") + bytes(28), None)
add("KAT-3 vlan", bytes.fromhex("020000000002" "020000000001" "8100" "0005" "0800")
    + ipv4(A1, A2) + tcp(1, 2, 3, 4, 0x50, 0x10, 5, 6), None)
add("KAT-3 ethertype 0x88cc", bytes.fromhex("0180c200000e" "020000000001" "88cc") + bytes(60),
    None)

# KAT-4 length boundaries
add("KAT-4 ipv4 53B", kat1[:53], None)
add("KAT-4 ipv4 54B", kat1, kat1_rec)
add("KAT-4 ipv4 33B", kat1[:33], None)
add("KAT-4 13B", kat1[:13], None)
add("KAT-4 ipv6 73B", kat2[:73], None)
add("KAT-4 ipv6 74B", kat2, kat2_rec)
add("KAT-4 ipv6 53B", kat2[:53], None)

# KAT-5 IPv4 IHL=6: TCP still read at frame offset 34, i.e. from the options
opts = bytes([0x01, 0x01, 0x01, 0x00])
kat5 = ETH_V4 + ipv4(A1, A2, ihl=6, options=opts, tot=44) + tcp(12345, 5201, 0x01020304,
                                                                 0x0A0B0C0D, 0x50, 0x12,
                                                                 0xFAF0, 0xABCD)
assert len(kat5) == 58
# frame[34:52] = 01 01 | 01 00 | 30 39 14 51 | 01 02 03 04 | 0a 0b | 0c 0d | 50 12
#   read as tcp[0..18]: sport 0x0101=257, dport 0x0100=256, seq 0x30391451,
#   ack 0x01020304, flag bytes 0a 0b, window 0x0c0d, check 0x5012
kat5_rec = (TLE + "0100000a" + "0200000a" + "00" * 32 + "0101" + "0001" + "51143930"
            + "04030201" + "0d0c" + "00" * 6 + "1250" + "ffffffff")
add("KAT-5 ipv4 ihl=6 fixed offset", kat5, kat5_rec,
    note="IHL ignored (config.rs:30-33): option bytes parsed as TCP")

# KAT-6 FILTER_PORT=5201
f80 = ETH_V4 + ipv4(A1, A2) + tcp(80, 1234, 7, 8, 0x50, 0x10, 9, 10)
add("KAT-6 filter 5201, 80->1234", f80, None, filter_port=5201)
fd = ETH_V4 + ipv4(A1, A2) + tcp(40000, 5201, 7, 8, 0x50, 0x10, 9, 10)
fd_rec = (TLE + "0100000a" + "0200000a" + "00" * 32 + "409c" + "5114" + "07000000"
          + "08000000" + "0900" + "00" * 6 + "0a00" + "ffffffff")
add("KAT-6 filter 5201, dport 5201", fd, fd_rec, filter_port=5201)
fs = ETH_V4 + ipv4(A2, A1) + tcp(5201, 40000, 7, 8, 0x50, 0x10, 9, 10)
fs_rec = (TLE + "0200000a" + "0100000a" + "00" * 32 + "5114" + "409c" + "07000000"
          + "08000000" + "0900" + "00" * 6 + "0a00" + "ffffffff")
add("KAT-6 filter 5201, sport 5201", fs, fs_rec, filter_port=5201)
add("KAT-6 no filter, 80->1234", f80, (TLE + "0100000a" + "0200000a" + "00" * 32 + "5000"
                                       + "d204" + "07000000" + "08000000" + "0900"
                                       + "00" * 6 + "0a00" + "ffffffff"))

# KAT-7 IPv4 saddr 0.0.0.0 -> downstream keys the flow as IPv6 ::/::
z = ETH_V4 + ipv4([0, 0, 0, 0], A2) + tcp(1000, 2000, 0, 0, 0x50, 0x02, 0, 0)
z_rec = (TLE + "00000000" + "0200000a" + "00" * 32 + "e803" + "d007" + "00000000"
         + "00000000" + "0000" + "00" * 6 + "0000" + "ffffffff")
add("KAT-7 ipv4 saddr 0", z, z_rec,
    decode={"tuple": ["::", "::", 1000, 2000, 6], "fields": {}})

# KAT-8 IPv6 hop-by-hop (nexthdr 0) before TCP -> no record
add("KAT-8 ipv6 nexthdr 0", ETH_V6 + ipv6(V6A, V6B, nexthdr=0) + bytes(8)
    + tcp(1, 2, 3, 4, 0x50, 0x10, 5, 6), None)

# KAT-9 all six flag bits set -> still all zero in the record
allf = ETH_V4 + ipv4(A1, A2) + tcp(1, 2, 3, 4, 0x50, 0x3F, 5, 6)
allf_rec = (TLE + "0100000a" + "0200000a" + "00" * 32 + "0100" + "0200" + "03000000"
            + "04000000" + "0500" + "00" * 6 + "0600" + "ffffffff")
add("KAT-9 all flags set", allf, allf_rec,
    decode={"tuple": ["10.0.0.1", "10.0.0.2", 1, 2, 6],
            "fields": {"SEQ_NUM": 3, "ACK_NUM": 4, "WINDOW": 5, "CHECKSUM": 6}})

# KAT-10 IPv6 v4-compatible address: IpTuple identical to an IPv4 frame's
v4c = bytes(12) + bytes(A1)
v4d = bytes(12) + bytes(A2)
k10 = ETH_V6 + ipv6(v4c, v4d) + tcp(12345, 5201, 1, 1, 0x50, 0x10, 1, 1)
k10_rec = (TLE + "00000000" + "00000000" + v4c.hex() + v4d.hex() + "3930" + "5114"
           + "01000000" + "01000000" + "0100" + "00" * 6 + "0100" + "ffffffff")
add("KAT-10 ipv6 ::10.0.0.1", k10, k10_rec,
    note="FLOWS key equals the IPv4 10.0.0.1:12345->10.0.0.2:5201 key (xdp.rs:116-119)")

# The IpTuple key (flow.rs:4-12 + 2 zero bytes) expected for a few vectors
keys = {
    "KAT-1 ipv4 syn-ack": (bytes(12) + bytes(A1) + bytes(12) + bytes(A2)
                           + struct.pack("<HHBxxx", 12345, 5201, 6)).hex(),
    "KAT-2 ipv6 psh-ack": (V6A + V6B + struct.pack("<HHBxxx", 443, 50000, 6)).hex(),
    "KAT-10 ipv6 ::10.0.0.1": (v4c + v4d + struct.pack("<HHBxxx", 12345, 5201, 6)).hex(),
}
for v in vectors:
    v["key"] = keys.get(v["name"])
    if v["expect"] is not None:
        assert len(bytes.fromhex(v["expect"])) == 74, v["name"]

with open(os.path.join(HERE, "kat_vectors.json"), "w") as f:
    json.dump({"source": "hand-derived from reference source, SURVEY.md Appendix B",
               "vectors": vectors}, f, indent=1)
print(f"wrote {len(vectors)} vectors")
