"""The packet-record path over several GPUs: one process per GPU,
every frame parsed once on one GPU (no frame exchange); only flow identities and
counters cross GPUs, over RCCL:

* FlowHashExchange — flow-hash shards (north_star's partition, NIC-RSS style):
  disjoint tables, global first-seen ids from one all-gather of first frames;
* OwnerExchange — contiguous shards: each flow merged at its hash owner
  (all-to-all of owner segments, SURVEY.md §8(e) option 2);
* FlowMerge / OverlappedMerge — the general all-gather table merge (any
  partition; the merged table on request);
* replay_pcap_sharded — a pcap replayed over the ranks into one .tcp file.

The reference has no multi-node story; its per-CPU FLOWS maps
(tcbee-ebpf/src/flow_tracker.rs:12-13) are the single-host analogue of the
per-rank tables merged here.
"""
from __future__ import annotations

import contextlib
import os
import shutil
import time

import numpy as np
import torch
import torch.distributed as dist

from . import parser as _parser

ENTRY_WORDS = 8  # tcbee_flow_entry = 64 B = u64[8]


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Frames [lo, hi) of rank `rank`: contiguous, sizes differ by at most one."""
    return n_total * rank // world, n_total * (rank + 1) // world


@contextlib.contextmanager
def rank_stream(parser: "_parser.PacketParser", stream: int | None):
    """The ONE stream a step's device calls AND its collectives run on.

    The C ABI reads a NULL stream as the context's own non-blocking stream, while
    torch issues RCCL / gloo collectives and tensor ops on its CURRENT stream; with
    torch's default stream (handle 0) the two differ, so a collective could read
    `first` / `ctr` before the kernels writing them ran. Here:
      * `stream` is torch's current stream: used as is (the caller's contract);
      * `stream` is 0 / None: the context's stream, made torch's current stream for
        the step (collectives included) after waiting for the caller's current
        stream (its producers of the inputs), and the caller's stream waits for it on
        exit (its readers of the outputs);
      * any other handle: the same, on that stream.
    Yields the handle to pass to every device call of the step."""
    cur = torch.cuda.current_stream()
    if stream and int(stream) == cur.cuda_stream:
        yield int(stream)
        return
    tgt = torch.cuda.ExternalStream(int(stream) if stream else parser.stream, device=cur.device)
    tgt.wait_stream(cur)
    with torch.cuda.stream(tgt):
        yield tgt.cuda_stream
    cur.wait_stream(tgt)


def all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = concat over ranks of inp (RCCL all_gather_into_tensor; list form on gloo)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        parts = list(out.chunk(dist.get_world_size(group)))
        tmp = [torch.empty_like(inp) for _ in parts]
        dist.all_gather(tmp, inp, group=group)
        for p, t in zip(parts, tmp):
            p.copy_(t)


def all_to_all_flat(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """Equal-split all-to-all: chunk r of inp goes to rank r, rank r's chunk for this
    rank lands at chunk r of out (RCCL all_to_all_single; through host memory on
    gloo, which exchanges CPU tensors)."""
    if dist.get_backend(group) == "nccl":
        dist.all_to_all_single(out, inp, group=group)
    else:
        tmp = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(tmp, inp.cpu(), group=group)
        out.copy_(tmp)


def gather_tables(entries: torch.Tensor, meta: torch.Tensor, group=None):
    """entries [cap, 8] int64 (this rank's exported table, padded to cap),
    meta [2] int64 {valid entries, records} -> (all_entries [world*cap, 8],
    all_meta [world*2]) on every rank. Fixed-size exchange: no host round trip."""
    world = dist.get_world_size(group)
    all_ent = torch.empty((world * entries.shape[0], ENTRY_WORDS), dtype=entries.dtype,
                          device=entries.device)
    all_meta = torch.empty(world * 2, dtype=meta.dtype, device=meta.device)
    all_gather_flat(all_meta, meta, group)
    all_gather_flat(all_ent, entries, group)
    return all_ent, all_meta


class FlowMerge:
    """Per-rank state of the RCCL flow-table merge.

    step(): export the local table (device), all-gather tables + {count, records}
    over RCCL, merge them on this GPU into `merged` (identical on every rank),
    then rewrite this rank's record flow ids from local to global ids.

    Two partitions of one global frame stream:
      contiguous ranges (gidx None): segment r's first_seen is local to rank r and
        the merge rebases it by the records of ranks < r;
      any other partition, e.g. flow-hash shards (gidx = global frame index of each
        local frame, ascending): the export carries the global FRAME index of each
        flow's first record (through the record -> frame map `rec_frame` when
        frames were rejected), the merge ranks flows by it, and the merged
        first_seen is turned back into the global RECORD index by one all-reduce
        of per-rank record counts (tcbee_flow_records_before_device). Tables of
        one step only: the local table is reset before every parse."""

    def __init__(self, local: "_parser.PacketParser", merged: "_parser.PacketParser",
                 cap: int, max_total_records: int, group=None, nbuf: int = 1):
        self.local, self.merged, self.cap = local, merged, cap
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.max_total = max_total_records
        dev = torch.device("cuda", torch.cuda.current_device())
        # nbuf export slots: a slot is read by the all-gather while the next step may
        # already export into another one (OverlappedMerge)
        self.ent = [torch.zeros((cap, ENTRY_WORDS), dtype=torch.int64, device=dev)
                    for _ in range(nbuf)]
        self.meta = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self.ids = torch.empty(self.world * cap, dtype=torch.int32, device=dev)
        # non-contiguous partitions (set by the caller): global frame index of each
        # local frame (device int64, ascending)
        self.gidx: torch.Tensor | None = None
        self.fs_counts = torch.zeros(self.world * cap, dtype=torch.int64, device=dev)

    def export(self, slot: int = 0, stream: int | None = None, rec_frame=None,
               rec_cap: int = 0) -> None:
        """Snapshot of the local table into export slot `slot` (before the next parse).
        Pass a non-NULL stream handle: NULL means the context's own stream.
        With `gidx` set, first_seen becomes the global frame index of each flow's
        first record: via rec_frame (the parse's out_frame, rec_cap entries) or,
        without it, assuming every frame was accepted (checked on the device:
        otherwise the local context's status reports TCBEE_ESHARD)."""
        with rank_stream(self.local, stream) as s:
            if self.gidx is None:
                self.local.export_device(self.ent[slot], self.cap, self.meta[slot], stream=s)
            else:
                self.local.export_global_device(self.ent[slot], self.cap, self.meta[slot],
                                                self.gidx, self.gidx.numel(), rec_frame=rec_frame,
                                                rec_frame_cap=rec_cap, stream=s)

    def merge(self, slot: int, out_id: torch.Tensor | None, n_dev: torch.Tensor | None,
              n_max: int, stream: int | None = None, rec_frame=None):
        """All-gather slot's tables (RCCL, current torch stream), merge them on this GPU
        and rewrite out_id from local to global ids, on `stream` (rank_stream)."""
        with rank_stream(self.merged, stream) as s:
            all_ent, all_meta = gather_tables(self.ent[slot], self.meta[slot], self.group)
            self.merged.merge_device(all_ent, self.world, self.cap, all_meta, self.max_total,
                                     self.ids, stream=s)
            if self.gidx is not None:
                # merged first_seen: global frame index -> global record index
                mcap = self.world * self.cap
                self.fs_counts.zero_()
                self.merged.records_before_device(rec_frame, self.gidx, n_dev, n_max,
                                                  self.fs_counts, mcap, stream=s)
                dist.all_reduce(self.fs_counts, group=self.group)
                self.merged.set_first_seen_device(self.fs_counts, mcap, stream=s)
            if out_id is not None:
                lo = self.rank * self.cap
                _parser.remap_ids_device(out_id, n_max, n_dev, self.ids[lo:lo + self.cap],
                                         self.cap, stream=s)
        return all_ent, all_meta

    def step(self, out_id: torch.Tensor | None, n_dev: torch.Tensor | None, n_max: int,
             stream: int | None = None, rec_frame=None):
        """export + merge on one stream (rank_stream: torch's current one, or with
        stream 0 / None the local context's, made current for the collectives)."""
        with rank_stream(self.local, stream) as s:
            self.export(0, stream=s, rec_frame=rec_frame, rec_cap=n_max)
            return self.merge(0, out_id, n_dev, n_max, stream=s, rec_frame=rec_frame)


class OverlappedMerge:
    """Step i's exchange (all-gather, merge, id remap, counter all-reduce) runs on a
    side stream and overlaps step i+1's parse on the main stream. Output buffers
    rotate over `nbuf` slots; acquire(slot) makes the main stream wait until the
    slot's previous exchange is done with them. Only the export (a snapshot of the
    local table) stays on the main stream, ahead of the next step's table reset."""

    def __init__(self, fm: FlowMerge, nbuf: int = 2, timing: bool = False):
        assert len(fm.ent) >= nbuf
        self.fm, self.nbuf = fm, nbuf
        self.side = torch.cuda.Stream()
        self.done = [None] * nbuf
        self.timing = timing
        self.spans = []  # (start, done) event pairs of the side-stream exchanges

    def exchange_ms(self) -> float | None:
        """Mean side-stream duration of the exchanges submitted since spans was
        last cleared (all-gather + merge + remap + all-reduce, while overlapping the
        next parse); None without timing."""
        if not self.spans:
            return None
        self.spans[-1][1].synchronize()
        return sum(a.elapsed_time(b) for a, b in self.spans) / len(self.spans)

    def acquire(self, slot: int) -> None:
        if self.done[slot] is not None:
            torch.cuda.current_stream().wait_event(self.done[slot])

    def submit(self, slot: int, out_id: torch.Tensor | None, n_dev: torch.Tensor | None,
               n_max: int, ctr: torch.Tensor | None = None, rec_frame=None) -> None:
        main = torch.cuda.current_stream()
        self.fm.export(slot, stream=main.cuda_stream, rec_frame=rec_frame, rec_cap=n_max)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            start = None
            if self.timing:
                start = torch.cuda.Event(enable_timing=True)
                start.record(self.side)
            self.fm.merge(slot, out_id, n_dev, n_max, stream=self.side.cuda_stream,
                          rec_frame=rec_frame)
            if ctr is not None:
                dist.all_reduce(ctr, group=self.fm.group)  # global INGRESS/HANDLED/DROPPED
            done = torch.cuda.Event(enable_timing=self.timing)
            done.record(self.side)
        if start is not None:
            self.spans.append((start, done))
        self.done[slot] = done


class FlowHashExchange:
    """The exchange of north_star's partition: flow-hash shards (tcbee_flowhash_owner /
    the NIC-RSS step) give every rank a DISJOINT set of flows, so the global
    first-seen ids need only each flow's global first frame — no table merge.
    Per step, between K2 and K3 on the rank's stream:
      tcbee_flow_first_frames_device (u64 per flow new in this batch, ascending)
      -> ONE RCCL all-gather of those arrays with {n_new, fbase} appended (8 B x
         (cap + 2) per rank)
      -> tcbee_global_ids_device (binary searches in the other ranks' arrays)
      -> K3 (tcbee_parse_finish_device) writes the GLOBAL ids directly: no per-record
         remap pass, and per-flow counters stay with their one owner (nothing to
         reduce). The counters are all-reduced by the caller; the merged flow table
         is assembled only on request (merged_flows).
    Steps are WINDOWS of one global trace (every rank's step k covers the same global
    frame range, each rank parsing its shard's frames inside it): the flow table and
    the local -> global id map (gmap, map_cap local flows) persist across windows, and
    the global flow count rides a device ping-pong pair (gtot), so a stream of windows
    gets the ids one parse of the whole trace would give. cap bounds the flows new in
    one window on one rank; reset() goes with the context's reset_flows()."""

    def __init__(self, local: "_parser.PacketParser", cap: int, gidx: torch.Tensor, group=None,
                 map_cap: int | None = None):
        self.local, self.cap, self.gidx, self.group = local, cap, gidx, group
        self.map_cap = map_cap or cap
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = gidx.device
        # one all-gather per window: rank r's new-flow first frames, then its
        # {n_new, fbase}, at r * (cap + 2)
        self.buf = torch.zeros(cap + 2, dtype=torch.int64, device=dev)
        self.first, self.n = self.buf[:cap], self.buf[cap:]
        self.all_buf = torch.empty(self.world * (cap + 2), dtype=torch.int64, device=dev)
        self.gmap = torch.empty(self.map_cap, dtype=torch.int32, device=dev)
        self.gtot = torch.zeros(2, dtype=torch.int64, device=dev)
        self.windows = 0
        self.spans = []  # (start, end) events of the exchange per step, when timing
        self.timing = False

    def reset(self) -> None:
        """Forget the global flow count (call with the context's reset_flows())."""
        self.gtot.zero_()
        self.windows = 0

    def exchange_ms(self) -> float | None:
        """Mean span of the timed steps' exchanges (first frames -> global ids,
        the all-gather included); synchronizes."""
        if not self.spans:
            return None
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.spans) / len(self.spans)

    def step(self, arena, arena_len: int, offset, caplen, ts_ns, n: int, out_rec, out_cap: int,
             out_hash, out_id, out_n, counters, stream: int, filter_port: int = 0,
             direction: int = 0, rec_frame=None, ids_stream: int | None = None,
             gidx: torch.Tensor | None = None) -> None:
        """Parse this rank's frames of the next window with global flow ids, every call
        and collective on one stream (rank_stream: torch's current stream, or with
        stream 0 / None the context's own, ordered after and before the caller's). gidx: the window's local frame -> global
        frame index (default: the one given at construction). rec_frame (u32[out_cap]):
        the record -> frame map, needed when the shard holds frames the hook rejects;
        without it every frame must be accepted (checked on the device: the context's
        status then reports TCBEE_ESHARD). ids_stream: K3 (global ids, pkts/bytes,
        counters, out_n) runs there, beside the next step's parse; order readers of
        those outputs after it."""
        gidx = self.gidx if gidx is None else gidx
        with rank_stream(self.local, stream) as s:
            self.local.parse_device(arena, arena_len, offset, caplen, ts_ns, n, out_rec, out_cap,
                                    out_hash, out_id, out_n, counters, filter_port=filter_port,
                                    direction=direction, stream=s, out_frame=rec_frame,
                                    defer_ids=True, ids_stream=ids_stream)
            if self.timing:  # the exchange's span on the stream: first frames .. global ids
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            self.local.first_frames_device(self.first, self.cap, self.n, gidx, gidx.numel(),
                                           rec_frame=rec_frame, rec_frame_cap=out_cap, stream=s)
            all_gather_flat(self.all_buf, self.buf, self.group)
            b = self.windows & 1
            _parser.global_ids_device(self.all_buf, self.all_buf[self.cap:], self.world,
                                      self.rank, self.cap + 2, self.gmap, self.map_cap,
                                      gbase_in=self.gtot[b:b + 1],
                                      gbase_out=self.gtot[1 - b:2 - b], stream=s,
                                      n_stride=self.cap + 2)
            if self.timing:
                ev1.record()
                self.spans.append((ev0, ev1))
            self.windows += 1
            self.local.finish_device(self.gmap, self.map_cap, stream=s)

    def merged_flows(self, merged: "_parser.PacketParser", n_dev, n_max: int,
                     max_total_records: int, rec_frame=None):
        """The global flow table (FLOW_DTYPE, global id order, first_seen = global
        record index) on every rank: the global-order export, all-gather and merge of
        FlowMerge, run once on request (collective: every rank must call it). Needs the
        table to hold one window (reset() + reset_flows() before each step): a flow
        first seen in an earlier window has no first record in the last batch's
        record -> frame map (TCBEE_ESHARD)."""
        fm = FlowMerge(self.local, merged, self.cap, max_total_records, self.group)
        fm.gidx = self.gidx
        s = torch.cuda.current_stream().cuda_stream
        fm.step(None, n_dev, n_max, stream=s, rec_frame=rec_frame)
        torch.cuda.synchronize()
        return merged.flows()


class OwnerExchange:
    """Global flow ids for CONTIGUOUS shards (every rank may hold every flow) by flow
    ownership — SURVEY.md §8(e) option 2 — instead of every rank merging every
    table (FlowMerge): flow f is merged at rank fold32(flow_hash64(key)) % world.
    Per step, between K2 and K3 on the rank's stream:
      tcbee_owner_bucket_device (the local flows by owner: key + local first_seen)
      -> all-gather of the per-owner counts and record counts
      -> RCCL all-to-all of the owner segments (seg_cap entries of 64 B each)
      -> the owner's merge of what it received (tcbee_flow_merge_device on `owner`:
         first_seen rebased to the global record stream, min over ranks)
      -> its flows' first_seen (ascending in its ids), one all-gather, global ids by
         binary search (tcbee_global_ids_device, as the flow-hash exchange)
      -> each received entry's global id back to its sender (all-to-all, 4 B)
      -> the local -> global id map -> K3 writes global ids (no remap pass).
    Traffic per rank: 64 B x its flows out and in, vs 64 B x every rank's flows in
    with the all-gather merge. One batch per table (reset before each step), as
    FlowMerge; merged_flows() assembles the global table on request."""

    def __init__(self, local: "_parser.PacketParser", owner: "_parser.PacketParser",
                 seg_cap: int, owner_cap: int, map_cap: int, max_total_records: int,
                 group=None):
        self.local, self.owner, self.group = local, owner, group
        self.seg_cap, self.owner_cap, self.map_cap = seg_cap, owner_cap, map_cap
        self.max_total = max_total_records
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = torch.device("cuda", torch.cuda.current_device())
        W = self.world
        self.send = torch.zeros((W * seg_cap, ENTRY_WORDS), dtype=torch.int64, device=dev)
        self.recv = torch.zeros_like(self.send)
        self.lid = torch.zeros(W * seg_cap, dtype=torch.int32, device=dev)
        # {entries per owner..., records, entries dropped} per rank
        self.meta = torch.zeros(W + 2, dtype=torch.int64, device=dev)
        self.all_meta = torch.zeros(W * (W + 2), dtype=torch.int64, device=dev)
        self.seg_meta = torch.zeros((W, 2), dtype=torch.int64, device=dev)
        self.recv_ids = torch.zeros(W * seg_cap, dtype=torch.int32, device=dev)
        self.fs = torch.zeros(owner_cap + 2, dtype=torch.int64, device=dev)
        self.all_fs = torch.empty(W * (owner_cap + 2), dtype=torch.int64, device=dev)
        self.gmap_o = torch.zeros(owner_cap, dtype=torch.int32, device=dev)
        self.ret = torch.zeros(W * seg_cap, dtype=torch.int32, device=dev)
        self.back = torch.zeros(W * seg_cap, dtype=torch.int32, device=dev)
        self.gmap = torch.zeros(map_cap, dtype=torch.int32, device=dev)

    def step(self, arena, arena_len: int, offset, caplen, ts_ns, n: int, out_rec, out_cap: int,
             out_hash, out_id, out_n, counters, stream: int, filter_port: int = 0,
             direction: int = 0) -> None:
        """Parse this rank's contiguous shard with global flow ids (one stream for every
        call and collective: rank_stream); the caller all-reduces the counters."""
        with rank_stream(self.local, stream) as s:
            self._step(arena, arena_len, offset, caplen, ts_ns, n, out_rec, out_cap, out_hash,
                       out_id, out_n, counters, s, filter_port, direction)

    def _step(self, arena, arena_len, offset, caplen, ts_ns, n, out_rec, out_cap, out_hash,
              out_id, out_n, counters, stream, filter_port, direction) -> None:
        W, C = self.world, self.seg_cap
        self.local.parse_device(arena, arena_len, offset, caplen, ts_ns, n, out_rec, out_cap,
                                out_hash, out_id, out_n, counters, filter_port=filter_port,
                                direction=direction, stream=stream, defer_ids=True)
        self.local.owner_bucket_device(W, C, self.map_cap, self.send, self.lid, self.meta,
                                       stream=stream)
        all_gather_flat(self.all_meta, self.meta, self.group)
        # any rank's dropped entries (segment or id-map overflow) shift the global ids
        # of every rank: flag TCBEE_ESHARD here too, not only on the dropping rank
        self.local.status_raise_device(self.all_meta[W + 1:], W, W + 2, stream=stream)
        am = self.all_meta.view(W, W + 2)
        # segment r of what this rank receives: rank r's entries for it, rank r's records
        self.seg_meta[:, 0] = am[:, self.rank].clamp(max=C)
        self.seg_meta[:, 1] = am[:, W]
        all_to_all_flat(self.recv, self.send, self.group)
        self.owner.merge_device(self.recv, W, C, self.seg_meta, self.max_total, self.recv_ids,
                                stream=stream)
        oc = self.owner_cap
        self.owner.first_seen_device(self.fs[:oc], oc, self.fs[oc:], stream=stream)
        all_gather_flat(self.all_fs, self.fs, self.group)
        _parser.global_ids_device(self.all_fs, self.all_fs[oc:], W, self.rank, oc + 2,
                                  self.gmap_o, oc, stream=stream, n_stride=oc + 2)
        _parser.owner_return_device(self.recv_ids, self.seg_meta, W, C, self.gmap_o, oc,
                                    self.ret, stream=stream)
        all_to_all_flat(self.back, self.ret, self.group)
        _parser.owner_apply_device(self.back, self.lid, self.meta, W, C, self.gmap,
                                   self.map_cap, stream=stream)
        self.local.finish_device(self.gmap, self.map_cap, stream=stream)

    def merged_flows(self, merged: "_parser.PacketParser", n_dev, n_max: int):
        """The global flow table on every rank (collective): the all-gather merge of
        FlowMerge, once, on request. The ranks' map_cap may differ; the all-gather
        takes the largest (its segments must be the same size everywhere)."""
        cap = torch.tensor([self.map_cap], dtype=torch.int64, device=self.gmap.device)
        dist.all_reduce(cap, op=dist.ReduceOp.MAX, group=self.group)
        fm = FlowMerge(self.local, merged, int(cap.item()), self.max_total, self.group)
        s = torch.cuda.current_stream().cuda_stream
        fm.step(None, n_dev, n_max, stream=s)
        torch.cuda.synchronize()
        return merged.flows()


def replay_pcap_sharded(pcap_path: str, out_prefix: str, direction: int = 0,
                        filter_port: int = 0, db_path: str | None = None, metrics: bool = True,
                        window: int = 64, chunk_frames: int = 1 << 20, threads: int = 8,
                        group=None) -> dict:
    """replay_pcap over the ranks of `group` (one process per GPU, collective): rank
    r streams the contiguous frames shard_range(n, r, world) of the capture (a
    zero-copy view of one mapping) through its own pinned pipeline into
    <out_prefix><xdp|tc>.tcp.part<r>; rank 0 then appends the parts in rank order to
    <out_prefix>xdp.tcp (or tc.tcp; BufferHandler append semantics: the bytes equal a
    one-GPU replay), optionally runs the tcbee-process stage into db_path and writes
    metrics.json with the all-reduced counters. Records only: no flow table is
    needed for the files (tcbee-process assigns flows itself). Returns the global
    counters, records and the slowest rank's seconds."""
    from . import _lib, host
    from .pipeline import Pipeline
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    name = "tc.tcp" if direction == _lib.DIR_EGRESS else "xdp.tcp"
    part = f"{out_prefix}{name}.part{rank}"
    if os.path.exists(part):
        os.remove(part)
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    with host.Pcap(pcap_path) as pc, Pipeline(device=torch.cuda.current_device(), window=window,
                                              chunk_frames=chunk_frames,
                                              threads=threads) as pipe:
        tr = pc.trace()
        lo, hi = shard_range(tr.n, rank, world)
        sub = tr.select(np.arange(lo, hi, dtype=np.int64))
        with host.TcpFile(part) as tf:
            res = pipe.run(sub, filter_port=filter_port, direction=direction, flows=False,
                           collect=False, sink=lambda rec, ids, first: tf.append(rec))
        frames = tr.n
    secs = time.perf_counter() - t0
    keys = ("ingress", "egress", "handled", "dropped")
    v = torch.tensor([res.counters[k] for k in keys] + [res.n], dtype=torch.int64,
                     device=dev if nccl else "cpu")
    dist.all_reduce(v, group=group)
    t = torch.tensor([secs], dtype=torch.float64, device=dev if nccl else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    v, t = v.cpu().tolist(), float(t.item())
    counters = dict(zip(keys, v[:4]))
    out = {"frames": frames, "records": v[4], "counters": counters, "seconds": t,
           "mpkts": frames / t / 1e6 if t > 0 else None, "ranks": world}
    dist.barrier(group=group)
    if rank == 0:
        with open(out_prefix + name, "ab") as dst:
            for r in range(world):
                p = f"{out_prefix}{name}.part{r}"
                with open(p, "rb") as src:
                    shutil.copyfileobj(src, dst, 1 << 24)
                os.remove(p)
        if db_path:
            out["sink"] = host.process_files(out_prefix, db_path)
        if metrics:
            host.write_metrics(out_prefix, counters)
    dist.barrier(group=group)
    return out
