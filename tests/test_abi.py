"""C-ABI library checks that need no GPU: it loads, exports exactly what
include/tcbee_amd.h declares, and its host-side pieces agree with the oracle."""
import os
import re
import struct

import numpy as np
import pytest

import tcbee_amd
from tcbee_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "tcbee_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tcbee_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    L = tcbee_amd.lib()
    declared = header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/tcbee_amd.h but not exported"
    assert sorted(_lib.EXPORTED) == declared


def test_abi_version_and_errors():
    L = tcbee_amd.lib()
    assert L.tcbee_abi_version() == 5
    assert L.tcbee_strerror(0) == b"ok"
    assert L.tcbee_strerror(_lib.EFLOWFULL) == b"flow table full"
    assert b"first record" in L.tcbee_strerror(_lib.ESHARD)


def test_device_count_does_not_crash():
    assert tcbee_amd.device_count() >= 0


def test_ctx_create_fails_loudly_without_gpu():
    if tcbee_amd.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(tcbee_amd.TcbeeError) as e:
        tcbee_amd.PacketParser(max_frames=16)
    assert e.value.code == _lib.ENODEV


def test_ctx_create_rejects_oversized_table():
    """max_flows past 2^24 (a 2 GiB table: K1's probe buffer resource and u32 slot
    offsets end there) is refused before any device work."""
    with pytest.raises(tcbee_amd.TcbeeError) as e:
        tcbee_amd.PacketParser(max_frames=16, max_flows=(1 << 24) + 1)
    assert e.value.code == _lib.ECAPACITY


def test_flow_hash_matches_oracle(oracle):
    rng = np.random.default_rng(0)
    for _ in range(200):
        k = bytes(rng.integers(0, 256, 40, dtype=np.uint8))
        assert tcbee_amd.flow_hash64(k) == oracle.flow_hash64(k)


def test_generator_config2_frame0():
    tr = tcbee_amd.synth_trace(3, sizes="64")
    f0 = tr.frame(0)
    assert len(f0) == 64
    assert f0[12:14] == b"\x08\x00" and f0[14] == 0x45 and f0[23] == 6
    assert f0[26:30] == bytes([10, 0, 0, 1]) and f0[30:34] == bytes([10, 0, 0, 2])
    sport, dport, seq, ack = struct.unpack("!HHII", f0[34:46])
    assert (sport, dport, seq, ack) == (40000, 5201, 1000, 1)
    assert f0[46:48] == b"\x50\x18"
    assert struct.unpack("!H", f0[48:50])[0] == 502
    f2 = tr.frame(2)
    assert struct.unpack("!I", f2[38:42])[0] == 1020
    assert struct.unpack("!H", f2[50:52])[0] == ((2 * 2654435761) & 0xFFFFFFFF) >> 16
    assert f0[54:] == bytes(10)
    # IPv4 header checksum verifies
    s = sum(struct.unpack("!10H", f0[14:34]))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    assert s == 0xFFFF


def test_generator_records_through_oracle(oracle):
    tr = tcbee_amd.synth_trace(1000, sizes="64")
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert len(rec) == 1000 and len(table) == 1 and int(table["pkts"][0]) == 1000
    r = rec[7].tobytes()
    assert struct.unpack("<Q", r[:8])[0] == 1_000_000_000 + 7000
    assert struct.unpack("<I", r[52:56])[0] == 1070


def test_imix_proportions():
    off, ln, ts, alen = tcbee_amd.synth_index(120000, sizes="imix")
    c = np.bincount(np.searchsorted([64, 576, 1500], ln))
    frac = c / c.sum()
    assert np.allclose(frac, [7 / 12, 4 / 12, 1 / 12], atol=0.01)
    assert alen == int(ln.sum()) and int(off[-1]) + int(ln[-1]) == alen
    assert np.all(np.diff(ts.astype(np.int64)) > 0)


def test_multiflow_generator_flow_count(oracle):
    tr = tcbee_amd.synth_trace(20000, sizes="imix", kind=1, n_flows=100)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert len(rec) == 20000
    assert len(table) == 100
    assert int(table["bytes"].sum()) == int(tr.caplen.sum())


def test_ipv6_generator_flows(oracle):
    """kind 3 (IPv6/TCP, IMIX6 sizes): every frame accepted as IPv6, the requested
    flow count, addresses in the v6 record fields only."""
    from tcbee_amd.trace import GEN_MULTI_V6
    tr = tcbee_amd.synth_trace(20000, sizes="imix6", kind=GEN_MULTI_V6, n_flows=300)
    assert int(tr.caplen.min()) == 78
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert len(rec) == 20000 and len(table) == 300
    assert not rec[:, 8:16].any() and rec[:, 16:48].any()  # v4 fields 0, v6 set
    assert int(table["bytes"].sum()) == int(tr.caplen.sum())


def test_exchange_calls_validate_before_device_work():
    """The context-free exchange entry points refuse bad arguments with
    TCBEE_EINVAL before touching a device (no GPU needed)."""
    import ctypes as C
    L = tcbee_amd.lib()
    buf = (C.c_uint64 * 8)()
    ids = (C.c_uint32 * 8)()
    p, q = C.cast(buf, C.c_void_p), C.cast(ids, C.c_void_p)
    q2 = C.c_void_p(C.addressof(ids) + 4)
    E = _lib.EINVAL
    # global ids: rank >= world, world 0, n_stride 1, gbase in == out, NULL arrays
    assert L.tcbee_global_ids_device(p, p, 2, 2, 2, 4, q, 8, None, None, None) == E
    assert L.tcbee_global_ids_device(p, p, 2, 0, 0, 4, q, 8, None, None, None) == E
    assert L.tcbee_global_ids_device(p, p, 1, 2, 0, 4, q, 8, None, None, None) == E
    assert L.tcbee_global_ids_device(p, p, 2, 2, 0, 4, q, 8, p, p, None) == E
    assert L.tcbee_global_ids_device(None, p, 2, 2, 0, 4, q, 8, None, None, None) == E
    assert L.tcbee_global_ids_device(p, p, 2, 2, 0, 4, None, 8, None, None, None) == E
    # owner return / apply: world 0, seg_cap 0, NULL buffers, a map length without a map
    assert L.tcbee_owner_return_device(q, p, 0, 4, q, 8, q2, None) == E
    assert L.tcbee_owner_return_device(q, p, 2, 0, q, 8, q2, None) == E
    assert L.tcbee_owner_return_device(None, p, 2, 4, q, 8, q2, None) == E
    assert L.tcbee_owner_return_device(q, p, 2, 4, None, 8, q2, None) == E
    assert L.tcbee_owner_apply_device(q, q, p, 0, 4, q2, 8, None) == E
    assert L.tcbee_owner_apply_device(q, q, None, 2, 4, q2, 8, None) == E
    assert L.tcbee_owner_apply_device(q, q, p, 2, 4, None, 8, None) == E
    # context calls with no context
    assert L.tcbee_owner_bucket_device(None, 2, 4, 8, p, q, p, None) == E
    assert L.tcbee_status_raise_device(None, p, 2, 4, None) == E
    assert L.tcbee_flow_first_seen_device(None, p, 4, p, None) == E
    assert L.tcbee_flow_first_frames_device(None, p, 4, p, None, p, 4, 4, None) == E


def test_variants_library_exports_the_same_abi():
    """libtcbee_amd_variants.so (test hooks + A/B variants) is the same ABI."""
    V = _lib.lib(variants=True)
    for name in header_functions():
        assert hasattr(V, name), name
    assert V.tcbee_abi_version() == tcbee_amd.lib().tcbee_abi_version()


def test_product_library_reads_no_environment():
    """the product library carries no TCBEE_* variable name (no
    getenv of an ablation, A/B variant or test hook: the dispatch is compiled into
    the variants build only), while the variants build does."""
    prod = open(_lib.LIB_PATH, "rb").read()
    var = open(_lib.VARIANTS_LIB_PATH, "rb").read()
    for name in (b"TCBEE_TEST_K3_TWOPASS", b"TCBEE_TEST_K3_WIDE", b"TCBEE_TEST_WITHHOLD",
                 b"TCBEE_TEST_NOPACK", b"TCBEE_NO_FUSE_RANK", b"TCBEE_PIPE_NT", b"TCBEE_FPL"):
        assert name in var, name
    # round 5: the timing-only ablations and refuted A/B variants are
    # gone from both builds
    for name in (b"TCBEE_ABLATE", b"TCBEE_K3ABL", b"TCBEE_K1V", b"TCBEE_STAGE", b"TCBEE_NT\0",
                 b"TCBEE_PROBE_AUX", b"TCBEE_REMAP_GRID", b"TCBEE_PIPE_CTHREADS"):
        assert name not in var and name not in prod, name
    assert re.search(rb"TCBEE_[A-Z0-9_]{2,}", prod) is None
    assert b"getenv" not in prod
