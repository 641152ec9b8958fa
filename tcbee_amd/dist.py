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
                 cap: int, max_total_records: int, group=None):
        self.local, self.merged, self.cap = local, merged, cap
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.max_total = max_total_records
        dev = torch.device("cuda", torch.cuda.current_device())
        self.ent = torch.zeros((cap, ENTRY_WORDS), dtype=torch.int64, device=dev)
        self.meta = torch.zeros(2, dtype=torch.int64, device=dev)
        self.ids = torch.empty(self.world * cap, dtype=torch.int32, device=dev)

    def step(self, out_id: torch.Tensor | None, n_dev: torch.Tensor | None, n_max: int,
             stream: int | None = None):
        self.local.export_device(self.ent, self.cap, self.meta, stream=stream)
        all_ent, all_meta = gather_tables(self.ent, self.meta, self.group)
        self.merged.merge_device(all_ent, self.world, self.cap, all_meta, self.max_total,
                                 self.ids, stream=stream)
        if out_id is not None:
            lo = self.rank * self.cap
            _parser.remap_ids_device(out_id, n_max, n_dev, self.ids[lo:lo + self.cap],
                                     self.cap, stream=stream)
        return all_ent, all_meta
