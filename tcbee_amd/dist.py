"""The packet-record path over several GPUs: one process per GPU, each parsing a
contiguous shard of one global frame stream (no frame exchange), then one RCCL
exchange of the compact per-rank flow tables so that every rank holds the same
merged table and global dense flow ids.

The reference has no multi-node story; its per-CPU FLOWS maps
(tcbee-ebpf/src/flow_tracker.rs:12-13) are the single-host analogue of the
per-rank tables merged here.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import parser as _parser

ENTRY_WORDS = 8  # tcbee_flow_entry = 64 B = u64[8]


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Frames [lo, hi) of rank `rank`: contiguous, sizes differ by at most one."""
    return n_total * rank // world, n_total * (rank + 1) // world


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
    then rewrite this rank's record flow ids from local to global ids."""

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
        # flow-hash shards (set by the caller): global frame index of each local frame
        self.gidx: torch.Tensor | None = None

    def export(self, slot: int = 0, stream: int | None = None) -> None:
        """Snapshot of the local table into export slot `slot` (before the next parse).
        Pass a non-NULL stream handle: NULL means the context's own stream.

        With `gidx` set (flow-hash shards: a rank's frames are a subsequence of the
        global stream, and its flows are its own), first_seen becomes the global
        index of the flow's first record and the merge rebases nothing. That needs
        record k == local frame k, i.e. every frame accepted (true for the synthetic
        IPv4/TCP traces this mode is built for)."""
        self.local.export_device(self.ent[slot], self.cap, self.meta[slot], stream=stream)
        if self.gidx is not None:
            ent, meta = self.ent[slot], self.meta[slot]
            valid = torch.arange(self.cap, device=ent.device) < meta[0]
            fs = ent[:, 7].clamp(0, self.gidx.numel() - 1)
            ent[:, 7] = torch.where(valid, self.gidx[fs], ent[:, 7])
            meta[1] = 0

    def merge(self, slot: int, out_id: torch.Tensor | None, n_dev: torch.Tensor | None,
              n_max: int, stream: int | None = None):
        """All-gather slot's tables (RCCL, current torch stream), merge them on this GPU
        and rewrite out_id from local to global ids, on `stream`."""
        all_ent, all_meta = gather_tables(self.ent[slot], self.meta[slot], self.group)
        self.merged.merge_device(all_ent, self.world, self.cap, all_meta, self.max_total,
                                 self.ids, stream=stream)
        if out_id is not None:
            lo = self.rank * self.cap
            _parser.remap_ids_device(out_id, n_max, n_dev, self.ids[lo:lo + self.cap],
                                     self.cap, stream=stream)
        return all_ent, all_meta

    def step(self, out_id: torch.Tensor | None, n_dev: torch.Tensor | None, n_max: int,
             stream: int | None = None):
        """export + merge on one stream (the torch current stream must be `stream`)."""
        self.export(0, stream=stream)
        return self.merge(0, out_id, n_dev, n_max, stream=stream)


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
               n_max: int, ctr: torch.Tensor | None = None) -> None:
        main = torch.cuda.current_stream()
        self.fm.export(slot, stream=main.cuda_stream)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            start = None
            if self.timing:
                start = torch.cuda.Event(enable_timing=True)
                start.record(self.side)
            self.fm.merge(slot, out_id, n_dev, n_max, stream=self.side.cuda_stream)
            if ctr is not None:
                dist.all_reduce(ctr, group=self.fm.group)  # global INGRESS/HANDLED/DROPPED
            done = torch.cuda.Event(enable_timing=self.timing)
            done.record(self.side)
        if start is not None:
            self.spans.append((start, done))
        self.done[slot] = done
