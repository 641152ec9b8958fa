"""The N>1 path on the GPU (tcbee_amd.dist): world-size-2 gloo ranks sharing
device 0 run the device export -> all-gather -> tcbee_flow_merge_device ->
remap choreography, on one stream (FlowMerge.step) and overlapped with the
next step's parse on a side stream (OverlappedMerge, as bench.py). Records,
global flow ids, global counters and the merged table vs the oracle on the
unsharded trace."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["step", "overlap"])
def test_gpu_world2_merge(gpu, oracle, tmp_path, mode):
    import torch.multiprocessing as mp

    import dist_worker
    from tracegen import mixed_trace
    from tcbee_amd.parser import FLOW_DTYPE
    n, cap, world = 60_000, 2048, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), mode),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=700)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    assert np.array_equal(np.concatenate([r["rec"] for r in res]), rec)
    assert np.array_equal(np.concatenate([r["gids"] for r in res]), fi)
    for r in res:
        assert np.array_equal(r["merged"].view(FLOW_DTYPE), table)
        assert int(r["ctr"][0]) == ctr["ingress"] and int(r["ctr"][2]) == ctr["handled"]


def test_gpu_world2_flowhash_shards(gpu, oracle, tmp_path):
    """Flow-hash shards (config 4's NIC-RSS view): each rank's frames are the
    global frames whose flow hash % world is its rank (device shard generator);
    records, global flow ids and the merged table vs the oracle over the global
    trace, and the shards partition the trace."""
    import torch.multiprocessing as mp

    import dist_worker
    import tcbee_amd
    from tcbee_amd.parser import FLOW_DTYPE
    n, cap, world = 120_000, 4096, 2
    mp.spawn(dist_worker.run_gpu, args=(world, free_port(), n, cap, str(tmp_path), "flowhash"),
             nprocs=world, join=True)
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=3000)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    owner = fh % world
    all_g = np.concatenate([r["gidx"] for r in res])
    assert len(all_g) == n and np.array_equal(np.sort(all_g), np.arange(n))
    for r, x in enumerate(res):
        g = x["gidx"]
        assert np.array_equal(g, np.nonzero(owner == r)[0])
        assert np.array_equal(x["rec"], rec[g])
        assert np.array_equal(x["gids"], fi[g])
        assert np.array_equal(x["merged"].view(FLOW_DTYPE), table)
        assert int(x["ctr"][0]) == ctr["ingress"]
