"""Worker for the world-size-2 gloo test of the multi-GPU choreography (CPU)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def run(rank, world, port, n, cap, result_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from merge_ref import entries_to_table, merge, table_to_entries
    from oracle_py import Oracle
    from tracegen import mixed_trace

    from tcbee_amd.dist import gather_tables, shard_range

    tr = mixed_trace(n, seed=404, n_flows=700)
    lo, hi = shard_range(tr.n, rank, world)
    orc = Oracle()
    rec, fh, fi, ctr, table = orc.parse(tr.slice(lo, hi))
    ent = torch.from_numpy(table_to_entries(table, cap))
    meta = torch.tensor([len(table), len(rec)], dtype=torch.int64)
    all_ent, all_meta = gather_tables(ent, meta)
    all_ent = all_ent.numpy().reshape(world, cap, 8)
    all_meta = all_meta.numpy().reshape(world, 2)
    tables = [entries_to_table(all_ent[r], int(all_meta[r, 0])) for r in range(world)]
    merged, maps = merge(tables, [int(all_meta[r, 1]) for r in range(world)])
    gids = maps[rank][fi] if len(fi) else fi
    np.savez(os.path.join(result_dir, f"rank{rank}.npz"), merged=merged.view(np.uint8),
             gids=gids, lo=lo, hi=hi, nrec=len(rec))
    dist.barrier()
    dist.destroy_process_group()
