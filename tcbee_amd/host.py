"""ctypes binding of libtcbee_host.so (include/tcbee_host.h): the callers either
side of the GPU record path — classic-pcap ingest, the ``.tcp`` record files,
the tcbee-process flow/time-series stage with its SQLite sink, metrics.json.

No GPU is needed for anything here. The library is built in-tree by
``make -C tcbee_amd/host`` / ``__graft_entry__.build()``; there is no Python
fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import EDB, EFORMAT, OK, Counters, Frames, RECORD_BYTES, TcbeeError
from .trace import Trace

_HERE = os.path.dirname(os.path.abspath(__file__))
# TCBEE_HOST_LIB: an alternative build of the same library (the sanitizer build
# tests/test_sanitize.py loads)
HOST_LIB_PATH = os.environ.get("TCBEE_HOST_LIB") or os.path.join(_HERE, "lib", "libtcbee_host.so")

SINK_DURABLE = 0x1
# DataValue::type_to_int (ts-storage/src/lib.rs:74-95)
T_INT, T_FLOAT, T_BOOL, T_TEXT = 0, 1, 2, 3


class PcapInfo(C.Structure):
    _fields_ = [("linktype", C.c_uint32), ("snaplen", C.c_uint32),
                ("nanosecond", C.c_uint32), ("swapped", C.c_uint32),
                ("n", C.c_uint64), ("truncated", C.c_uint64), ("file_bytes", C.c_uint64)]


class TsTuple(C.Structure):
    _fields_ = [("src", C.c_char * 48), ("dst", C.c_char * 48), ("sport", C.c_int64),
                ("dport", C.c_int64), ("l4proto", C.c_int64)]

    def as_tuple(self):
        return (self.src.decode(), self.dst.decode(), int(self.sport), int(self.dport),
                int(self.l4proto))


class SinkStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("records", "flows", "series_created",
                                          "series_deleted", "points", "batches",
                                          "failed_batches", "failed_records")]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# tcbee_packet (C layout: 74 bytes of fields, padded to 80 by the u64 alignment)
PACKET_DTYPE = np.dtype({
    "names": ["time", "saddr", "daddr", "saddr_v6", "daddr_v6", "sport", "dport", "seq", "ack",
              "window", "flag_urg", "flag_ack", "flag_psh", "flag_rst", "flag_syn", "flag_fin",
              "checksum", "div"],
    "formats": ["<u8", "<u4", "<u4", ("u1", 16), ("u1", 16), "<u2", "<u2", "<u4", "<u4", "<u2",
                "u1", "u1", "u1", "u1", "u1", "u1", "<u2", ("u1", 4)],
    "offsets": [0, 8, 12, 16, 32, 48, 50, 52, 56, 60, 62, 63, 64, 65, 66, 67, 68, 70],
    "itemsize": 80,
})

vp, u64, i64, cint, dbl, cstr = (C.c_void_p, C.c_uint64, C.c_int64, C.c_int, C.c_double,
                                 C.c_char_p)
_SIGS = {
    "tcbee_host_abi_version": (cint, []),
    "tcbee_pcap_open": (cint, [C.POINTER(vp), cstr]),
    "tcbee_pcap_frames": (cint, [vp, C.POINTER(Frames)]),
    "tcbee_pcap_get_info": (cint, [vp, C.POINTER(PcapInfo)]),
    "tcbee_pcap_close": (cint, [vp]),
    "tcbee_pcap_write": (cint, [cstr, C.POINTER(Frames), cint, C.c_uint32]),
    "tcbee_tcp_decode": (cint, [vp, u64, vp, C.POINTER(u64)]),
    "tcbee_tcp_check": (cint, [vp, u64, C.POINTER(u64)]),
    "tcbee_tcp_tuple": (cint, [vp, C.POINTER(TsTuple)]),
    "tcbee_tcpfile_open": (cint, [C.POINTER(vp), cstr, u64]),
    "tcbee_tcpfile_append": (cint, [vp, vp, u64]),
    "tcbee_tcpfile_close": (cint, [vp]),
    "tcbee_sink_open": (cint, [C.POINTER(vp), cstr, C.c_uint32]),
    "tcbee_sink_packets": (cint, [vp, vp, u64]),
    "tcbee_sink_packets_grouped": (cint, [vp, vp, vp, u64, u64]),
    "tcbee_sink_close": (cint, [vp, C.POINTER(SinkStats)]),
    "tcbee_sink_get_stats": (cint, [vp, C.POINTER(SinkStats)]),
    "tcbee_process_files": (cint, [cstr, cstr, C.c_uint32, C.POINTER(SinkStats)]),
    "tcbee_tsdb_create_flow": (cint, [vp, cstr, cstr, i64, i64, i64, C.POINTER(i64)]),
    "tcbee_tsdb_delete_flow": (cint, [vp, cstr, cstr, i64, i64, i64]),
    "tcbee_tsdb_create_series": (cint, [vp, i64, cstr, cint, C.POINTER(i64)]),
    "tcbee_tsdb_delete_series": (cint, [vp, i64, cstr]),
    "tcbee_tsdb_insert_points": (cint, [vp, i64, cint, vp, vp, vp, u64]),
    "tcbee_tsdb_add_attribute": (cint, [vp, i64, cstr, cint, i64, dbl, cstr]),
    "tcbee_tsdb_set_attribute": (cint, [vp, i64, cstr, cint, i64, dbl, cstr]),
    "tcbee_tsdb_delete_attribute": (cint, [vp, i64, cstr]),
    "tcbee_metrics_write": (cint, [cstr, C.POINTER(Counters), u64, u64]),
    "tcbee_flowhash_owner": (cint, [C.POINTER(Frames), C.c_uint32, C.c_uint32, vp]),
    "tcbee_flowhash_owner_rss": (cint, [C.POINTER(Frames), C.c_uint32, vp, C.c_uint32,
                                        C.c_uint32, vp]),
    "tcbee_flowhash_load": (cint, [C.POINTER(Frames), C.c_uint32, C.c_uint32, vp]),
}
HOST_EXPORTED = tuple(_SIGS)

_hlib = None


def hlib() -> C.CDLL:
    global _hlib
    if _hlib is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise ImportError(f"{HOST_LIB_PATH} is missing: build it with "
                              "`make -C tcbee_amd/host` or __graft_entry__.build()")
        L = C.CDLL(HOST_LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _hlib = L
    return _hlib


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise TcbeeError(rc, what)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def _frames_of(t: Trace) -> Frames:
    return Frames(_ptr(t.arena), t.arena.size, _ptr(t.offset), _ptr(t.caplen), _ptr(t.ts_ns),
                  t.n)


# ---- pcap -------------------------------------------------------------------
class Pcap:
    """A memory-mapped classic pcap. ``trace()`` is a zero-copy Trace over it."""

    def __init__(self, path: str):
        h = C.c_void_p()
        _check(hlib().tcbee_pcap_open(C.byref(h), os.fsencode(path)), f"pcap_open {path}")
        self._h = h
        info = PcapInfo()
        _check(hlib().tcbee_pcap_get_info(h, C.byref(info)), "pcap_get_info")
        self.info = {k: int(getattr(info, k)) for k, _ in info._fields_}
        fr = Frames()
        _check(hlib().tcbee_pcap_frames(h, C.byref(fr)), "pcap_frames")
        self.frames = fr
        n = int(fr.n)

        def view(ptr, dtype, count):
            if count == 0:
                return np.zeros(0, dtype)
            buf = (C.c_uint8 * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dtype, count=count)
        self._trace = Trace.__new__(Trace)
        self._trace.arena = view(fr.arena, np.uint8, int(fr.arena_len))
        self._trace.offset = view(fr.offset, np.uint64, n)
        self._trace.caplen = view(fr.caplen, np.uint32, n)
        self._trace.ts_ns = view(fr.ts_ns, np.uint64, n)

    @property
    def n(self) -> int:
        return int(self.frames.n)

    def trace(self) -> Trace:
        """Zero-copy view (valid until close())."""
        return self._trace

    def close(self):
        if getattr(self, "_h", None):
            hlib().tcbee_pcap_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def flowhash_owner(trace: Trace, world: int, threads: int = 8, rss=None) -> np.ndarray:
    """GPU owning each frame under the flow-hash partition (tcbee_flowhash_owner:
    the NIC-RSS step; frames the hook cannot key go round robin). rss: an RSS
    indirection table (uint16, entries < world; trace.rss_table) instead of
    fold32(hash) % world (tcbee_flowhash_owner_rss)."""
    out = np.empty(max(trace.n, 1), dtype=np.uint16)
    fr = _frames_of(trace)
    if rss is None:
        _check(hlib().tcbee_flowhash_owner(C.byref(fr), world, threads, _ptr(out)),
               "tcbee_flowhash_owner")
    else:
        tab = np.ascontiguousarray(rss, dtype=np.uint16)
        _check(hlib().tcbee_flowhash_owner_rss(C.byref(fr), world, _ptr(tab), len(tab), threads,
                                               _ptr(out)), "tcbee_flowhash_owner_rss")
    return out[:trace.n]


def flowhash_load(trace: Trace, rss_len: int = 4096, threads: int = 8) -> np.ndarray:
    """Keyed frames per RSS bucket (fold32(flow hash) % rss_len): the observed load
    an RSS table is balanced on (tcbee_flowhash_load)."""
    out = np.zeros(rss_len, dtype=np.uint64)
    fr = _frames_of(trace)
    _check(hlib().tcbee_flowhash_load(C.byref(fr), rss_len, threads, _ptr(out)),
           "tcbee_flowhash_load")
    return out


def flowhash_shard(trace: Trace, world: int, rank: int, threads: int = 8, rss=None):
    """(rank's frames as a zero-copy Trace, their global frame indices)."""
    gidx = np.nonzero(flowhash_owner(trace, world, threads, rss) == rank)[0].astype(np.int64)
    return trace.select(gidx), gidx


def write_pcap(path: str, trace: Trace, nanosecond: bool = True, snaplen: int = 262144) -> None:
    fr = _frames_of(trace)
    _check(hlib().tcbee_pcap_write(os.fsencode(path), C.byref(fr), int(nanosecond), snaplen),
           f"pcap_write {path}")


# ---- .tcp records -------------------------------------------------------------
def _as_records(rec) -> np.ndarray:
    a = np.ascontiguousarray(np.frombuffer(rec, np.uint8) if isinstance(rec, (bytes, bytearray))
                             else np.asarray(rec, dtype=np.uint8).reshape(-1))
    if a.size % RECORD_BYTES:
        raise ValueError("record buffer is not a whole number of 74-byte entries")
    return a


def decode_records(rec) -> tuple[np.ndarray, int]:
    """(PACKET_DTYPE array, number of entries that fell back to the default)."""
    a = _as_records(rec)
    n = a.size // RECORD_BYTES
    out = np.zeros(n, PACKET_DTYPE)
    nd = C.c_uint64(0)
    _check(hlib().tcbee_tcp_decode(_ptr(a), n, _ptr(out), C.byref(nd)), "tcp_decode")
    return out, int(nd.value)


def check_records(rec) -> int:
    """Index of the first entry failing the marker check, or the entry count."""
    a = _as_records(rec)
    first = C.c_uint64(0)
    rc = hlib().tcbee_tcp_check(_ptr(a), a.size // RECORD_BYTES, C.byref(first))
    if rc not in (OK, EFORMAT):
        _check(rc, "tcp_check")
    return int(first.value)


def packet_tuple(pkt: np.ndarray) -> tuple:
    """tcbee-process' IpTuple of one decoded packet: (src, dst, sport, dport, 6)."""
    one = np.ascontiguousarray(np.asarray(pkt, PACKET_DTYPE).reshape(1))
    t = TsTuple()
    _check(hlib().tcbee_tcp_tuple(_ptr(one), C.byref(t)), "tcp_tuple")
    return t.as_tuple()


class TcpFile:
    """Append-only .tcp writer (BufferHandler semantics)."""

    def __init__(self, path: str, buffer_bytes: int = 0):
        h = C.c_void_p()
        _check(hlib().tcbee_tcpfile_open(C.byref(h), os.fsencode(path), buffer_bytes),
               f"tcpfile_open {path}")
        self._h = h

    def append(self, rec) -> None:
        a = _as_records(rec)
        _check(hlib().tcbee_tcpfile_append(self._h, _ptr(a), a.size // RECORD_BYTES),
               "tcpfile_append")

    def close(self) -> None:
        if self._h:
            h, self._h = self._h, None
            _check(hlib().tcbee_tcpfile_close(h), "tcpfile_close")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---- SQLite sink ----------------------------------------------------------------
class Sink:
    """tcbee-process' DBWriter on a SQLite file (see include/tcbee_host.h)."""

    def __init__(self, db_path: str, durable: bool = False):
        h = C.c_void_p()
        _check(hlib().tcbee_sink_open(C.byref(h), os.fsencode(db_path),
                                      SINK_DURABLE if durable else 0), f"sink_open {db_path}")
        self._h = h

    def packets(self, rec) -> None:
        """In-order DBWriter::run over 74-byte entries. Raises TcbeeError(EFORMAT) at
        the first entry failing the marker check (where tcbee-process panics)."""
        a = _as_records(rec)
        _check(hlib().tcbee_sink_packets(self._h, _ptr(a), a.size // RECORD_BYTES),
               "sink_packets")

    def packets_grouped(self, rec, flow_id: np.ndarray, n_ids: int | None = None) -> None:
        """Same result from entries pre-classified by the GPU (dense flow ids)."""
        a = _as_records(rec)
        ids = np.ascontiguousarray(flow_id, dtype=np.uint32)
        n = a.size // RECORD_BYTES
        if ids.size < n:
            raise ValueError("flow_id shorter than the record count")
        if n_ids is None:
            n_ids = int(ids[:n].max()) + 1 if n else 0
        _check(hlib().tcbee_sink_packets_grouped(self._h, _ptr(a), _ptr(ids), n, n_ids),
               "sink_packets_grouped")

    def stats(self) -> dict:
        st = SinkStats()
        _check(hlib().tcbee_sink_get_stats(self._h, C.byref(st)), "sink_get_stats")
        return st.as_dict()

    def close(self) -> dict:
        st = SinkStats()
        if self._h:
            h, self._h = self._h, None
            _check(hlib().tcbee_sink_close(h, C.byref(st)), "sink_close")
        return st.as_dict()

    # ts-storage primitives (TSDBInterface)
    def create_flow(self, src, dst, sport, dport, l4proto=6) -> int:
        i = C.c_int64()
        _check(hlib().tcbee_tsdb_create_flow(self._h, src.encode(), dst.encode(), sport, dport,
                                             l4proto, C.byref(i)), "create_flow")
        return int(i.value)

    def delete_flow(self, src, dst, sport, dport, l4proto=6) -> None:
        _check(hlib().tcbee_tsdb_delete_flow(self._h, src.encode(), dst.encode(), sport, dport,
                                             l4proto), "delete_flow")

    def create_series(self, flow_id: int, name: str, value_type: int) -> int:
        i = C.c_int64()
        _check(hlib().tcbee_tsdb_create_series(self._h, flow_id, name.encode(), value_type,
                                               C.byref(i)), "create_series")
        return int(i.value)

    def delete_series(self, flow_id: int, name: str) -> None:
        _check(hlib().tcbee_tsdb_delete_series(self._h, flow_id, name.encode()),
               "delete_series")

    def insert_points(self, series_id: int, value_type: int, timestamps, values) -> bool:
        """insert_multiple_points: True if inserted, False if the batch was rejected."""
        t = np.ascontiguousarray(timestamps, dtype=np.float64)
        if value_type == T_FLOAT:
            fv, iv = np.ascontiguousarray(values, dtype=np.float64), None
        else:
            fv, iv = None, np.ascontiguousarray(values, dtype=np.int64)
        rc = hlib().tcbee_tsdb_insert_points(self._h, series_id, value_type, _ptr(t), _ptr(iv),
                                             _ptr(fv), t.size)
        if rc == EDB:
            return False
        _check(rc, "insert_points")
        return True

    def _attr(self, fn, flow_id, name, value_type, value):
        iv, fv, tv = 0, 0.0, None
        if value_type == T_TEXT:
            tv = str(value).encode()
        elif value_type == T_FLOAT:
            fv = float(value)
        else:
            iv = int(value)
        _check(fn(self._h, flow_id, name.encode(), value_type, iv, fv, tv), fn.__name__)

    def add_attribute(self, flow_id, name, value_type, value):
        self._attr(hlib().tcbee_tsdb_add_attribute, flow_id, name, value_type, value)

    def set_attribute(self, flow_id, name, value_type, value):
        self._attr(hlib().tcbee_tsdb_set_attribute, flow_id, name, value_type, value)

    def delete_attribute(self, flow_id, name):
        _check(hlib().tcbee_tsdb_delete_attribute(self._h, flow_id, name.encode()),
               "delete_attribute")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def process_files(source_prefix: str, db_path: str, durable: bool = False) -> dict:
    """tcbee-process -s <source_prefix> -o <db_path> -q over xdp.tcp / tc.tcp."""
    st = SinkStats()
    _check(hlib().tcbee_process_files(os.fsencode(source_prefix), os.fsencode(db_path),
                                      SINK_DURABLE if durable else 0, C.byref(st)),
           "process_files")
    return st.as_dict()


def write_metrics(dir_prefix: str, counters: dict, ingress_calls: int = 0,
                  egress_calls: int = 0) -> str:
    """Writes <dir_prefix>metrics.json; returns its path."""
    c = Counters(**{k: int(counters.get(k, 0)) & 0xFFFFFFFFFFFFFFFF
                    for k in ("ingress", "egress", "handled", "dropped")})
    _check(hlib().tcbee_metrics_write(os.fsencode(dir_prefix), C.byref(c), ingress_calls,
                                      egress_calls), "metrics_write")
    return dir_prefix + "metrics.json"
