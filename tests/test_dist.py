"""Multi-rank path on CPU: world-size-2 gloo run of the shard + table-exchange
choreography (tcbee_amd.dist) against the oracle on the unsharded trace."""
import os
import socket

import numpy as np
import pytest


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_everything():
    from tcbee_amd.dist import shard_range
    for n in (0, 1, 7, 1000, 12345):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))


def test_reference_merge_equals_unsharded(oracle):
    from merge_ref import merge
    from tracegen import mixed_trace
    tr = mixed_trace(30_000, seed=8, n_flows=900)
    full = oracle.parse(tr)
    tables, recs, ids = [], [], []
    cuts = [0, 7000, 7001, 19000, 30000]
    for lo, hi in zip(cuts, cuts[1:]):
        r = oracle.parse(tr.slice(lo, hi))
        tables.append(r[4])
        recs.append(len(r[0]))
        ids.append(r[2])
    merged, maps = merge(tables, recs)
    assert np.array_equal(merged, full[4])
    gids = np.concatenate([m[i] for m, i in zip(maps, ids)])
    assert np.array_equal(gids, full[2])


def test_gloo_world2_choreography(oracle, tmp_path):
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    n, cap, world = 40_000, 2048, 2
    mp.spawn(dist_worker.run, args=(world, free_port(), n, cap, str(tmp_path)), nprocs=world,
             join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    full = oracle.parse(tr)
    from tcbee_amd.parser import FLOW_DTYPE
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for r in res:
        assert np.array_equal(r["merged"].view(FLOW_DTYPE), full[4])
    gids = np.concatenate([r["gids"] for r in res])
    assert np.array_equal(gids, full[2])
