"""ctypes view of oracle/liboracle.so — the CPU restatement used as the checker.

TEST INFRASTRUCTURE ONLY. Parity unpinned (see oracle/tcbee_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")


class OrcTrace(C.Structure):
    _fields_ = [("time", C.c_uint64), ("saddr", C.c_uint32), ("daddr", C.c_uint32),
                ("saddr_v6", C.c_uint8 * 16), ("daddr_v6", C.c_uint8 * 16),
                ("sport", C.c_uint16), ("dport", C.c_uint16), ("seq", C.c_uint32),
                ("ack", C.c_uint32), ("window", C.c_uint16),
                ("flag_urg", C.c_uint8), ("flag_ack", C.c_uint8), ("flag_psh", C.c_uint8),
                ("flag_rst", C.c_uint8), ("flag_syn", C.c_uint8), ("flag_fin", C.c_uint8),
                ("checksum", C.c_uint16)]


class OrcIpTuple(C.Structure):
    _fields_ = [("src_ip", C.c_uint8 * 16), ("dst_ip", C.c_uint8 * 16),
                ("sport", C.c_uint16), ("dport", C.c_uint16), ("protocol", C.c_uint8),
                ("_pad", C.c_uint8)]


class OrcCounters(C.Structure):
    _fields_ = [("ingress", C.c_uint64), ("egress", C.c_uint64),
                ("handled", C.c_uint64), ("dropped", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class OrcPacket(C.Structure):
    _fields_ = [("t", OrcTrace), ("div", C.c_uint8 * 4)]


class OrcDbTuple(C.Structure):
    _fields_ = [("is_v4", C.c_int), ("src", C.c_uint8 * 16), ("dst", C.c_uint8 * 16),
                ("sport", C.c_int64), ("dport", C.c_int64), ("l4proto", C.c_int64)]


assert C.sizeof(OrcTrace) == 72, C.sizeof(OrcTrace)
assert C.sizeof(OrcIpTuple) == 38

vp = C.c_void_p
u64 = C.c_uint64


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        L = C.CDLL(path)
        L.orc_xdp_hook.argtypes = [vp, C.c_uint32, u64, C.c_uint16, C.POINTER(OrcTrace),
                                   C.POINTER(OrcIpTuple)]
        L.orc_tc_hook.argtypes = L.orc_xdp_hook.argtypes
        L.orc_serialize.argtypes = [C.POINTER(OrcTrace), vp]
        L.orc_deserialize.argtypes = [vp, C.POINTER(OrcPacket)]
        L.orc_marker_ok.argtypes = [C.POINTER(OrcPacket)]
        L.orc_get_ip_tuple.argtypes = [C.POINTER(OrcPacket), C.POINTER(OrcDbTuple)]
        L.orc_get_field.argtypes = [C.POINTER(OrcPacket), C.c_int, C.POINTER(C.c_int64)]
        L.orc_key40.argtypes = [C.POINTER(OrcIpTuple), vp]
        L.orc_flow_hash64.argtypes = [vp]
        L.orc_flow_hash64.restype = u64
        L.orc_flowtab_new.argtypes = [u64]
        L.orc_flowtab_new.restype = vp
        L.orc_flowtab_free.argtypes = [vp]
        L.orc_flowtab_count.argtypes = [vp]
        L.orc_flowtab_count.restype = u64
        L.orc_flowtab_export.argtypes = [vp, vp, u64]
        L.orc_flowtab_export.restype = u64
        L.orc_parse_batch.argtypes = [vp, vp, vp, vp, u64, C.c_uint16, C.c_int, vp, u64,
                                      vp, vp, vp, u64, C.POINTER(OrcCounters)]
        L.orc_parse_batch.restype = u64
        L.orc_accept_mask.argtypes = [vp, vp, vp, u64, C.c_uint16, C.c_int, vp]
        L.orc_accept_mask.restype = None
        L.orc_baseline_run.argtypes = [vp, vp, vp, vp, u64, C.c_uint16, C.c_int, vp]
        L.orc_baseline_run.restype = u64
        L.orc_baseline_file.argtypes = [vp, vp, vp, vp, u64, C.c_uint16, C.c_char_p]
        L.orc_baseline_file.restype = u64
        L.orc_ref_flows.argtypes = [vp, vp, vp, u64, C.c_uint16, C.c_int, u64, vp]
        L.orc_ref_flows.restype = u64
        self.L = L

    # -- single frame --------------------------------------------------------
    def hook(self, frame: bytes, ts: int = 0, filter_port: int = 0, direction: int = 0):
        """(record74 bytes | None, key40 bytes | None)"""
        t = OrcTrace()
        k = OrcIpTuple()
        buf = (C.c_uint8 * max(len(frame), 1)).from_buffer_copy(frame or b"\0")
        fn = self.L.orc_tc_hook if direction else self.L.orc_xdp_hook
        if not fn(buf, len(frame), ts, filter_port, C.byref(t), C.byref(k)):
            return None, None
        rec = (C.c_uint8 * 74)()
        self.L.orc_serialize(C.byref(t), rec)
        key = (C.c_uint8 * 40)()
        self.L.orc_key40(C.byref(k), key)
        return bytes(rec), bytes(key)

    def flow_hash64(self, key40: bytes) -> int:
        buf = (C.c_uint8 * 40).from_buffer_copy(key40)
        return int(self.L.orc_flow_hash64(buf))

    def decode(self, rec74: bytes) -> dict:
        """tcbee-process view of one record (tcp_packet.rs:31-124, db_writer.rs:76-82)."""
        buf = (C.c_uint8 * 74).from_buffer_copy(rec74)
        p = OrcPacket()
        ok = bool(self.L.orc_deserialize(buf, C.byref(p)))
        tup = OrcDbTuple()
        self.L.orc_get_ip_tuple(C.byref(p), C.byref(tup))
        fields = {}
        names = ["SEQ_NUM", "ACK_NUM", "WINDOW", "FLAG_URG", "FLAG_ACK", "FLAG_PSH",
                 "FLAG_RST", "FLAG_SYN", "FLAG_FIN", "CHECKSUM"]
        for i, nm in enumerate(names):
            v = C.c_int64()
            if self.L.orc_get_field(C.byref(p), i, C.byref(v)):
                fields[nm] = int(v.value)
        import ipaddress
        if tup.is_v4:
            src = str(ipaddress.IPv4Address(bytes(tup.src)[:4]))
            dst = str(ipaddress.IPv4Address(bytes(tup.dst)[:4]))
        else:
            src = str(ipaddress.IPv6Address(bytes(tup.src)))
            dst = str(ipaddress.IPv6Address(bytes(tup.dst)))
        return {"decoded": ok, "marker_ok": bool(self.L.orc_marker_ok(C.byref(p))),
                "time": int(p.t.time), "tuple": (src, dst, int(tup.sport), int(tup.dport),
                                                 int(tup.l4proto)),
                "fields": fields}

    # -- batch ------------------------------------------------------------------
    def new_flowtab(self, cap: int = 1024):
        return self.L.orc_flowtab_new(cap)

    def free_flowtab(self, ft):
        self.L.orc_flowtab_free(ft)

    def flows(self, ft) -> np.ndarray:
        from tcbee_amd.parser import FLOW_DTYPE
        n = int(self.L.orc_flowtab_count(ft))
        out = np.zeros(max(n, 1), dtype=FLOW_DTYPE)
        self.L.orc_flowtab_export(ft, out.ctypes.data, n)
        return out[:n]

    def parse(self, trace, filter_port: int = 0, direction: int = 0, out_cap=None,
              ft=None, record_base: int = 0, flows: bool = True):
        n = trace.n
        cap = n if out_cap is None else int(out_cap)
        rec = np.zeros((max(cap, 1), 74), dtype=np.uint8)
        fh = np.zeros(max(cap, 1), dtype=np.uint32)
        fi = np.zeros(max(cap, 1), dtype=np.uint32)
        own = False
        if flows and ft is None:
            ft = self.new_flowtab(1024)
            own = True
        ctr = OrcCounters()
        arena = trace.arena if len(trace.arena) else np.zeros(1, np.uint8)
        k = self.L.orc_parse_batch(arena.ctypes.data, trace.offset.ctypes.data,
                                   trace.caplen.ctypes.data, trace.ts_ns.ctypes.data, n,
                                   filter_port, direction, rec.ctypes.data, cap,
                                   fh.ctypes.data, fi.ctypes.data,
                                   ft if flows else None, record_base, C.byref(ctr))
        table = self.flows(ft) if flows else None
        if own:
            self.free_flowtab(ft)
        return rec[:k], fh[:k], fi[:k], ctr.as_dict(), table

    def accept_mask(self, trace, filter_port: int = 0, direction: int = 0) -> np.ndarray:
        """bool per frame: does the hook emit a record for it."""
        out = np.zeros(max(trace.n, 1), dtype=np.uint8)
        arena = trace.arena if len(trace.arena) else np.zeros(1, np.uint8)
        self.L.orc_accept_mask(arena.ctypes.data, trace.offset.ctypes.data,
                               trace.caplen.ctypes.data, trace.n, filter_port, direction,
                               out.ctypes.data)
        return out[:trace.n].astype(bool)

    def baseline_file(self, trace, path: str, filter_port: int = 0) -> int:
        """CPU-1-file: one thread, records appended to `path` (drain-task buffering)."""
        import os
        k = self.L.orc_baseline_file(trace.arena.ctypes.data, trace.offset.ctypes.data,
                                     trace.caplen.ctypes.data, trace.ts_ns.ctypes.data,
                                     trace.n, filter_port, os.fsencode(path))
        if k == 0xFFFFFFFFFFFFFFFF:
            raise OSError(f"orc_baseline_file: I/O error on {path}")
        return int(k)

    def baseline(self, trace, threads: int = 1, filter_port: int = 0):
        out = np.empty((max(trace.n, 1), 74), dtype=np.uint8)
        k = self.L.orc_baseline_run(trace.arena.ctypes.data, trace.offset.ctypes.data,
                                    trace.caplen.ctypes.data, trace.ts_ns.ctypes.data,
                                    trace.n, filter_port, threads, out.ctypes.data)
        return int(k)

    def ref_flows(self, trace, filter_port: int = 0, direction: int = 0, max_flows: int = 100):
        out = np.zeros((max_flows, 40), dtype=np.uint8)
        k = self.L.orc_ref_flows(trace.arena.ctypes.data, trace.offset.ctypes.data,
                                 trace.caplen.ctypes.data, trace.n, filter_port, direction,
                                 max_flows, out.ctypes.data)
        return out[:k]
