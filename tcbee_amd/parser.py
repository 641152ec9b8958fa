"""The packet-record path on an MI355X: a Python handle over ``tcbee_ctx``.

One :class:`PacketParser` = one ``tcbee_ctx`` = one HIP stream and one flow
table. It plays the role the reference gives to the attached XDP/TC programs
(tcbee-record/tcbee-ebpf/src/main.rs:69-83) plus the drain task that
serializes their ring entries (tcbee-record/tcbee/src/handlers/mod.rs:94-146):
frames in, 74-byte ``*.tcp`` records out, in input order.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .trace import Trace

FLOW_DTYPE = np.dtype([("tuple", np.uint8, (40,)), ("pkts", np.uint64),
                       ("bytes", np.uint64), ("first_seen", np.uint64)])
assert FLOW_DTYPE.itemsize == 64


@dataclass
class ParseResult:
    records: np.ndarray              # uint8 [n, 74]
    flow_hash: np.ndarray | None     # uint32 [n]
    flow_id: np.ndarray | None       # uint32 [n]
    counters: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return len(self.records)

    def tobytes(self) -> bytes:
        """The bytes tcbee-record would have appended to xdp.tcp / tc.tcp."""
        return self.records.tobytes()


def _ptr(x) -> int:
    """Raw address of a numpy array, torch tensor or int."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    raise TypeError(type(x))


class PacketParser:
    def __init__(self, device: int = 0, max_frames: int = 1 << 20, max_arena: int = 0,
                 max_flows: int = 1 << 16, variants: bool = False,
                 max_wide_flows: int | None = None):
        """variants=True: a context of the variants build (libtcbee_amd_variants.so),
        whose test hooks / A/B variants follow TCBEE_* environment variables read at
        creation — for tests of those alternative paths; the product library ignores
        the environment. max_wide_flows: the bound on non-IPv4-form (IPv6) keys that
        sizes the 64-B wide slots (tcbee_ctx_create_ex; None = max_flows)."""
        L = _lib.lib(variants)
        self._L = L
        h = C.c_void_p()
        wide = max_flows if max_wide_flows is None else max_wide_flows
        if hasattr(L, "tcbee_ctx_create_ex"):
            _lib.check(L.tcbee_ctx_create_ex(C.byref(h), device, C.c_uint64(max_frames),
                                             C.c_uint64(max_arena), C.c_uint64(max_flows),
                                             C.c_uint64(wide)),
                       "tcbee_ctx_create_ex")
        else:  # an ABI-4 library under TCBEE_AB_LIB (A/B tooling only)
            _lib.check(L.tcbee_ctx_create(C.byref(h), device, C.c_uint64(max_frames),
                                          C.c_uint64(max_arena), C.c_uint64(max_flows)),
                       "tcbee_ctx_create")
        self._h = h
        self._owned = True
        self.device = device
        self.max_frames = max_frames
        self.max_arena = max_arena
        self.max_flows = max_flows

    @classmethod
    def _borrow(cls, handle: C.c_void_p, device: int, max_frames: int, max_flows: int,
                lib: C.CDLL | None = None):
        """A non-owning view of a context owned elsewhere (e.g. an ingest pipeline;
        `lib`: the library that created it)."""
        self = cls.__new__(cls)
        self._h, self._owned, self._L = handle, False, lib or _lib.lib()
        self.device, self.max_frames, self.max_arena, self.max_flows = (device, max_frames, 0,
                                                                        max_flows)
        return self

    # -- lifetime -----------------------------------------------------------
    def close(self) -> None:
        if self._h:
            if self._owned:
                self._L.tcbee_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        _lib.check(self._L.tcbee_ctx_stream(self._h, C.byref(s)), "tcbee_ctx_stream")
        return s.value or 0

    def sync(self) -> None:
        _lib.check(self._L.tcbee_ctx_sync(self._h), "tcbee_ctx_sync")

    def status(self) -> int:
        """Sticky in-kernel status since the last call (OK / EFLOWFULL / ESPIN)."""
        return self._L.tcbee_ctx_status(self._h)

    # -- host-pointer path ---------------------------------------------------
    def parse(self, trace: Trace, filter_port: int = 0, direction: int = _lib.DIR_INGRESS,
              flows: bool = True, out_cap: int | None = None) -> ParseResult:
        """Synchronous: H2D frames, parse, D2H records (+ flow hash / id)."""
        n = trace.n
        cap = n if out_cap is None else int(out_cap)
        rec = np.empty((max(cap, 1), _lib.RECORD_BYTES), dtype=np.uint8)
        fh = np.empty(max(cap, 1), dtype=np.uint32) if flows else None
        fi = np.empty(max(cap, 1), dtype=np.uint32) if flows else None
        fr = _lib.Frames(trace.arena.ctypes.data if len(trace.arena) else 0, len(trace.arena),
                         trace.offset.ctypes.data, trace.caplen.ctypes.data,
                         trace.ts_ns.ctypes.data, n)
        cfg = _lib.Cfg(filter_port, direction, 0, 0 if flows else _lib.F_NO_FLOWS)
        nout = C.c_uint64(0)
        ctr = _lib.Counters()
        _lib.check(self._L.tcbee_parse_batch(
            self._h, C.byref(fr), C.byref(cfg), rec.ctypes.data, C.c_uint64(cap),
            _ptr(fh), _ptr(fi), C.byref(nout), C.byref(ctr)), "tcbee_parse_batch")
        k = nout.value
        return ParseResult(rec[:k], fh[:k] if flows else None, fi[:k] if flows else None,
                           ctr.as_dict())

    # -- device-resident path -------------------------------------------------
    def parse_device(self, arena, arena_len: int, offset, caplen, ts_ns, n: int,
                     out_rec, out_cap: int, out_hash=None, out_id=None, out_n=None,
                     counters=None, filter_port: int = 0,
                     direction: int = _lib.DIR_INGRESS, flows: bool = True,
                     stream: int | None = None, out_frame=None, defer_ids: bool = False,
                     ids_stream: int | None = None) -> None:
        """Asynchronous parse of frames already in HBM (pointers or torch tensors).

        out_n: device u64[1]; counters: device u64[4] (accumulated); out_frame:
        device u32[out_cap], the batch-local frame index of each record; defer_ids:
        stop before K3 (finish_device writes ids, pkts/bytes, counters, out_n);
        ids_stream: run K3 there, beside the next batch's K1 (order readers of
        out_id / out_n / counters after that stream)."""
        fr = _lib.Frames(_ptr(arena), arena_len, _ptr(offset), _ptr(caplen), _ptr(ts_ns), n)
        cfg = _lib.Cfg(filter_port, direction, 0, 0 if flows else _lib.F_NO_FLOWS)
        if out_frame is None and not defer_ids and not ids_stream:
            _lib.check(self._L.tcbee_parse_batch_device(
                self._h, C.byref(fr), C.byref(cfg), _ptr(out_rec), C.c_uint64(out_cap),
                _ptr(out_hash), _ptr(out_id), _ptr(out_n), _ptr(counters),
                C.c_void_p(stream or 0)), "tcbee_parse_batch_device")
            return
        ex = _lib.ParseEx(_ptr(out_frame), (_lib.EX_DEFER_IDS if defer_ids else 0)
                          | (_lib.EX_ASYNC_IDS if ids_stream else 0), 0, ids_stream or None)
        _lib.check(self._L.tcbee_parse_batch_device_ex(
            self._h, C.byref(fr), C.byref(cfg), _ptr(out_rec), C.c_uint64(out_cap),
            _ptr(out_hash), _ptr(out_id), _ptr(out_n), _ptr(counters), C.byref(ex),
            C.c_void_p(stream or 0)), "tcbee_parse_batch_device_ex")

    def finish_device(self, id_map=None, map_len: int = 0, stream: int | None = None) -> None:
        """K3 of a defer_ids parse: out_id = id_map[local id] (or the local id)."""
        _lib.check(self._L.tcbee_parse_finish_device(
            self._h, _ptr(id_map), C.c_uint64(map_len if id_map is not None else 0),
            C.c_void_p(stream or 0)), "tcbee_parse_finish_device")

    def count_mode(self) -> int:
        """K3 mode of the last batch (0 bins, 1 buckets, 2 atomics, 3 claim ranges)."""
        m = C.c_int(-1)
        _lib.check(self._L.tcbee_ctx_count_mode(self._h, C.byref(m)), "tcbee_ctx_count_mode")
        return m.value

    # -- measurement --------------------------------------------------------------
    def profile(self, enable: bool = True) -> None:
        _lib.check(self._L.tcbee_ctx_profile(self._h, int(enable)), "tcbee_ctx_profile")

    def profile_read(self):
        """(summed K1 ms, K1 launches) since profile(True)."""
        ms = C.c_double(0)
        k = C.c_uint64(0)
        _lib.check(self._L.tcbee_ctx_profile_read(self._h, C.byref(ms), C.byref(k)),
                   "tcbee_ctx_profile_read")
        return ms.value, k.value

    # -- flow table -------------------------------------------------------------
    def flow_count(self) -> int:
        n = C.c_uint64(0)
        _lib.check(self._L.tcbee_flow_count(self._h, C.byref(n)), "tcbee_flow_count")
        return n.value

    def flows(self) -> np.ndarray:
        """Flow table in dense-id (first-seen) order, dtype FLOW_DTYPE."""
        cnt = self.flow_count()
        out = np.zeros(max(cnt, 1), dtype=FLOW_DTYPE)
        n = C.c_uint64(0)
        _lib.check(self._L.tcbee_flow_export(self._h, out.ctypes.data, C.c_uint64(cnt),
                                                C.byref(n)), "tcbee_flow_export")
        return out[:n.value]

    def reset_flows(self, stream: int | None = None, sync: bool = True) -> None:
        if sync:
            _lib.check(self._L.tcbee_flow_reset(self._h), "tcbee_flow_reset")
        else:
            _lib.check(self._L.tcbee_flow_reset_device(self._h, C.c_void_p(stream or 0)),
                       "tcbee_flow_reset_device")

    # -- device-side flow tables (multi-GPU merge) ---------------
    def export_device(self, out, cap: int, meta=None, stream: int | None = None) -> None:
        """out[id] = flow entry (u64[8]) for ids < cap; meta (device u64[2]) receives
        {flows exported, accepted frames so far}. Asynchronous."""
        _lib.check(self._L.tcbee_flow_export_device(
            self._h, _ptr(out), C.c_uint64(cap), _ptr(meta), C.c_void_p(stream or 0)),
            "tcbee_flow_export_device")

    def export_global_device(self, out, cap: int, meta, frame_gidx, n_frames: int,
                             rec_frame=None, rec_frame_cap: int = 0,
                             stream: int | None = None) -> None:
        """As export_device, first_seen = global frame index of each flow's first
        record (frame_gidx[rec_frame[r]], or frame_gidx[r] when every frame was
        accepted); meta[1] = 0. The table must hold one batch's flows."""
        _lib.check(self._L.tcbee_flow_export_global_device(
            self._h, _ptr(out), C.c_uint64(cap), _ptr(meta), _ptr(rec_frame), _ptr(frame_gidx),
            C.c_uint64(n_frames), C.c_uint64(rec_frame_cap), C.c_void_p(stream or 0)),
            "tcbee_flow_export_global_device")

    def first_frames_device(self, out, cap: int, n_dev, frame_gidx, n_frames: int,
                            rec_frame=None, rec_frame_cap: int = 0,
                            stream: int | None = None) -> None:
        """For the flows first seen in the last batch (local ids fbase..): out[id -
        fbase] = global frame index of the flow's first record; n_dev = {n_new,
        fbase} (the flow-hash exchange's per-rank input)."""
        _lib.check(self._L.tcbee_flow_first_frames_device(
            self._h, _ptr(out), C.c_uint64(cap), _ptr(n_dev), _ptr(rec_frame), _ptr(frame_gidx),
            C.c_uint64(n_frames), C.c_uint64(rec_frame_cap), C.c_void_p(stream or 0)),
            "tcbee_flow_first_frames_device")

    def records_before_device(self, rec_frame, frame_gidx, n_rec_dev, n_rec_max: int,
                              out_counts, cap: int, stream: int | None = None) -> None:
        """out_counts[id] = this rank's records whose global frame index is below
        merged flow id's first_seen (a global frame index)."""
        _lib.check(self._L.tcbee_flow_records_before_device(
            self._h, _ptr(rec_frame), _ptr(frame_gidx), _ptr(n_rec_dev), C.c_uint64(n_rec_max),
            _ptr(out_counts), C.c_uint64(cap), C.c_void_p(stream or 0)),
            "tcbee_flow_records_before_device")

    def set_first_seen_device(self, fs_by_id, cap: int, stream: int | None = None) -> None:
        _lib.check(self._L.tcbee_flow_set_first_seen_device(
            self._h, _ptr(fs_by_id), C.c_uint64(cap), C.c_void_p(stream or 0)),
            "tcbee_flow_set_first_seen_device")

    def owner_bucket_device(self, world: int, seg_cap: int, map_cap: int, ent, lid, meta,
                            stream: int | None = None) -> None:
        """The table's flows into `world` owner segments of seg_cap entries (owner
        exchange, contiguous shards); meta (world + 2 words) = {entries per owner...,
        records, entries dropped}."""
        if meta.numel() < world + 2:
            raise ValueError(f"owner meta needs world + 2 = {world + 2} words")
        _lib.check(self._L.tcbee_owner_bucket_device(
            self._h, world, C.c_uint64(seg_cap), C.c_uint64(map_cap), _ptr(ent), _ptr(lid),
            _ptr(meta),
            C.c_void_p(stream or 0)), "tcbee_owner_bucket_device")

    def status_raise_device(self, v, n: int, stride: int, stream: int | None = None) -> None:
        """TCBEE_ESHARD on this context if any v[i * stride] (i < n, device u64) is
        non-zero: a peer's dropped owner entries (OwnerExchange)."""
        _lib.check(self._L.tcbee_status_raise_device(
            self._h, _ptr(v), C.c_uint64(n), C.c_uint64(stride), C.c_void_p(stream or 0)),
            "tcbee_status_raise_device")

    def first_seen_device(self, out, cap: int, n_dev, stream: int | None = None) -> None:
        """out[id] = first_seen of flow id (ascending in id); n_dev = {flows, 0}."""
        _lib.check(self._L.tcbee_flow_first_seen_device(
            self._h, _ptr(out), C.c_uint64(cap), _ptr(n_dev), C.c_void_p(stream or 0)),
            "tcbee_flow_first_seen_device")

    def merge_device(self, entries, nseg: int, stride: int, seg_meta, max_total_records: int,
                     out_ids, stream: int | None = None) -> None:
        """Replace this context's table by the merge of nseg exported tables."""
        _lib.check(self._L.tcbee_flow_merge_device(
            self._h, _ptr(entries), C.c_uint64(nseg), C.c_uint64(stride), _ptr(seg_meta),
            C.c_uint64(max_total_records), _ptr(out_ids), C.c_void_p(stream or 0)),
            "tcbee_flow_merge_device")


def gen_frames_device(arena, offset, caplen, n: int, kind: int, n_flows: int, seed: int,
                      stream: int | None = None, first_index: int = 0) -> None:
    """Device generator: header bytes of frames whose index is already in HBM.
    kind 2 (Zipf) ships the CDF table (trace.zipf_cdf) to the device first."""
    if kind == 2:
        import torch
        from .trace import zipf_cdf
        z = torch.from_numpy(zipf_cdf(n_flows).view(np.int64).copy()).to(arena.device)
        # the table copy (torch's stream) lands before the kernel (`stream`), and z
        # stays alive until the kernel is done: synchronous on both sides
        torch.cuda.synchronize(arena.device)
        _lib.check(_lib.lib().tcbee_gen_frames_zipf_device(
            _ptr(arena), _ptr(offset), _ptr(caplen), C.c_uint64(n), C.c_uint64(first_index),
            C.c_uint64(n_flows), C.c_uint64(seed), _ptr(z), C.c_void_p(stream or 0)),
            "tcbee_gen_frames_zipf_device")
        torch.cuda.synchronize(arena.device)
        return
    _lib.check(_lib.lib().tcbee_gen_frames_device(
        _ptr(arena), _ptr(offset), _ptr(caplen), C.c_uint64(n), C.c_uint64(first_index), kind,
        C.c_uint64(n_flows), C.c_uint64(seed), C.c_void_p(stream or 0)),
        "tcbee_gen_frames_device")


def gen_frames_index_device(arena, offset, caplen, gidx, n: int, kind: int, n_flows: int,
                            seed: int, stream: int | None = None) -> None:
    """Device generator, local frame j = global frame gidx[j] (a flow-hash shard)."""
    _lib.check(_lib.lib().tcbee_gen_frames_index_device(
        _ptr(arena), _ptr(offset), _ptr(caplen), _ptr(gidx), C.c_uint64(n), kind,
        C.c_uint64(n_flows), C.c_uint64(seed), C.c_void_p(stream or 0)),
        "tcbee_gen_frames_index_device")


def gen_shard_index_device(n_global: int, world: int, rank: int, kind: int, n_flows: int,
                           seed: int, imix: bool, out_gidx, out_caplen, cap: int, scratch,
                           n_out, stream: int | None = None, rss=None) -> None:
    """Global indices + caplens of rank's flow-hash shard of the synthetic trace.
    rss: an RSS indirection table on the device (uint16/int16 tensor, entries <
    world: tcbee_gen_shard_index_rss_device), or None for fold32(hash) % world.
    n_out receives TCBEE_RSS_INVALID (~0; -1 in an int64 tensor) for a table the
    device finds an entry >= world in."""
    if rss is None:
        _lib.check(_lib.lib().tcbee_gen_shard_index_device(
            C.c_uint64(n_global), world, rank, kind, C.c_uint64(n_flows), C.c_uint64(seed),
            int(bool(imix)), _ptr(out_gidx), _ptr(out_caplen), C.c_uint64(cap), _ptr(scratch),
            _ptr(n_out), C.c_void_p(stream or 0)), "tcbee_gen_shard_index_device")
        return
    import torch
    if rss.dtype not in (torch.int16, torch.uint16) or not rss.is_cuda or not rss.is_contiguous():
        # (the kernel reads the table as contiguous u16 words in device memory: an
        #  int32/int64 table would be read as interleaved zeros — ADVICE r3)
        raise ValueError("RSS table: a contiguous int16/uint16 device tensor")
    n_rss = int(rss.numel())
    if n_rss == 0 or n_rss > 4096 or int((rss.view(-1).to(torch.int32) & 0xFFFF).max().item()) >= world:
        # (a table entry >= world would drop that bucket's frames on every rank: the
        #  C ABI cannot see device memory without a copy, so the wrapper checks)
        raise ValueError(f"RSS table: 1..4096 entries, each < world={world}")
    _lib.check(_lib.lib().tcbee_gen_shard_index_rss_device(
        C.c_uint64(n_global), world, rank, kind, C.c_uint64(n_flows), C.c_uint64(seed),
        int(bool(imix)), _ptr(rss), C.c_uint32(int(rss.numel())), _ptr(out_gidx),
        _ptr(out_caplen), C.c_uint64(cap), _ptr(scratch), _ptr(n_out),
        C.c_void_p(stream or 0)), "tcbee_gen_shard_index_rss_device")


def gen_rss_load_device(n_frames: int, kind: int, n_flows: int, seed: int, counts,
                        stream: int | None = None, first_frame: int = 0) -> None:
    """Frames per RSS bucket of global frames [first_frame, first_frame + n_frames)
    of the synthetic trace into the int64 device tensor `counts` (its length = the
    table length)."""
    _lib.check(_lib.lib().tcbee_gen_rss_load_range_device(
        C.c_uint64(first_frame), C.c_uint64(n_frames), kind, C.c_uint64(n_flows),
        C.c_uint64(seed), C.c_uint32(int(counts.numel())), _ptr(counts),
        C.c_void_p(stream or 0)), "tcbee_gen_rss_load_range_device")


def gen_shard_scratch_words(n_global: int) -> int:
    return int(_lib.lib().tcbee_gen_shard_scratch(C.c_uint64(n_global)))


def remap_ids_device(ids, n_max: int, n_dev, id_map, map_len: int,
                     stream: int | None = None) -> None:
    """ids[p] = id_map[ids[p]] for p < min(*n_dev, n_max). Without a stream the
    remap goes on torch's current stream (the C ABI would read NULL as HIP's null
    stream, which other streams do not wait for)."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().tcbee_remap_ids_device(
        _ptr(ids), C.c_uint64(n_max), _ptr(n_dev), _ptr(id_map), C.c_uint64(map_len),
        C.c_void_p(stream or 0)), "tcbee_remap_ids_device")


def global_ids_device(all_first, all_n, world: int, rank: int, stride: int, out_map,
                      map_cap: int, gbase_in=None, gbase_out=None,
                      stream: int | None = None, n_stride: int = 2) -> None:
    """Global ids of `rank`'s flows new in this window, from the all-gathered
    first-frame arrays ({n_new, fbase} of rank r at all_n[r * n_stride]); gbase_in/out:
    device u64 words holding the global flow count before / after the window."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().tcbee_global_ids_device(
        _ptr(all_first), _ptr(all_n), C.c_uint64(n_stride), world, rank, C.c_uint64(stride),
        _ptr(out_map),
        C.c_uint64(map_cap), _ptr(gbase_in), _ptr(gbase_out), C.c_void_p(stream or 0)),
        "tcbee_global_ids_device")


def flow_hash64(key40: bytes) -> int:
    buf = (C.c_uint8 * 40).from_buffer_copy(bytes(key40))
    return int(_lib.lib().tcbee_flow_hash64(buf))


def owner_return_device(ids, seg_meta, world: int, seg_cap: int, gmap, gmap_len: int, ret,
                        stream: int | None = None) -> None:
    """ret[e] = gmap[ids[e]] for the valid received entries of the owner exchange."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().tcbee_owner_return_device(
        _ptr(ids), _ptr(seg_meta), world, C.c_uint64(seg_cap), _ptr(gmap), C.c_uint64(gmap_len),
        _ptr(ret), C.c_void_p(stream)), "tcbee_owner_return_device")


def owner_apply_device(back, lid, meta, world: int, seg_cap: int, id_map, map_cap: int,
                       stream: int | None = None) -> None:
    """id_map[lid[e]] = back[e] for the valid sent entries: local -> global ids."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().tcbee_owner_apply_device(
        _ptr(back), _ptr(lid), _ptr(meta), world, C.c_uint64(seg_cap), _ptr(id_map),
        C.c_uint64(map_cap), C.c_void_p(stream)), "tcbee_owner_apply_device")
