"""bench.py's own N>1 path, end to end, on the one-GPU box.

The driver's scaling run launches ``python -m torch.distributed.run ... bench.py
--gpus N`` over RCCL on N GPUs. RCCL refuses two ranks on one device, so this test
runs the SAME command at world 2 with the ranks sharing device 0 over gloo
(TCBEE_DIST_BACKEND=gloo), at reduced frame counts: the config-3 headline as
flow-hash shards with the held-out RSS table and the FlowHashExchange between K2
and K3, then the config-4 leg (1M flows of BASELINE.json configs[3], flow-hash
shards, FlowHashExchange), each ending with every rank's oracle check MIN-reduced
into ``all_ranks_bit_exact`` (bench.all_ranks_check). The JSON line it prints is
the one the driver records.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


from ports import free_port  # noqa: E402


def launch(world: int, args: list[str], timeout: int, **env_extra):
    env = dict(os.environ, TCBEE_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    env.update(env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), "bench.py", "--gpus", str(world)] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def run_bench_world(world: int, args: list[str], timeout: int = 420, **env_extra) -> dict:
    r = launch(world, args, timeout, **env_extra)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints ONE line
    return json.loads(lines[0])


def check_leg(chk: dict, world: int, full: bool = True):
    """full: every rank checked ALL of its shard — records, hashes,
    global ids vs a host recomputation of the global first-seen order, its rows of
    the merged table — not a 200k-record sample."""
    assert chk["all_ranks_bit_exact"] is True
    assert chk["ranks_checked"] == world
    assert chk["global_frames_ok"] and chk["global_pkts_ok"] and chk["global_ingress_ok"]
    assert chk["shard_imbalance"] < 1.01
    assert chk["status"] == 0
    if full:
        assert chk["full_bit_exact"] and chk["global_ids_exact"] and chk["merged_rows_exact"]
        assert chk["records_hashes_exact"] and chk["full_records"] == chk["frames_local"]
        assert chk["all_ranks_checked_in_full"] is True
        assert chk["ranks_full_bit_exact"] == [True] * world
    else:
        assert chk["sample_bit_exact"]


def test_bench_world2_flowhash_and_config4_leg(gpu):
    out = run_bench_world(2, ["--frames", "4000000", "--steps", "2", "--warmup", "1",
                              "--c4-frames", "6000000", "--c4-steps", "2"])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["dist"] == {"backend": "gloo", "world_size": 2}
    assert out["config"]["shard"] == "flowhash" and out["config"]["parallelism"] == "shard2"
    assert out["value"] > 0 and out["roofline"]["frac"] > 0
    # the measured binary is named: the in-tree product library
    assert out["lib_path"] == "tcbee_amd/lib/libtcbee_amd.so" and not out["ab_lib"]
    assert len(out["lib_sha256_16"]) == 16
    chk = out["check"]
    check_leg(chk, 2)
    assert chk["flows"] == 10_000 and chk["pkts_total"] == 2 * 4_000_000
    # the RSS table was balanced on frames outside the measured trace
    assert chk["rss"]["held_out"] is True
    assert chk["rss"]["balanced_on_frames"][0] == 2 * 4_000_000
    c4 = out["config4_flowhash"]
    assert c4["frames_global"] == 12_000_000 and c4["flows"] == 1_000_000
    assert c4["mpkts"] > 0 and c4["ms_per_step"] > 0
    check_leg(c4["check"], 2)
    # 12M IMIX frames of 1M uniform flows: almost every flow appears
    assert 990_000 < c4["check"]["flows"] <= 1_000_000
    assert c4["check"]["pkts_total"] == 12_000_000


def test_bench_world4_flowhash_and_config4_leg(gpu):
    """World 4 (four ranks on device 0 over gloo): both legs bit-exact on every rank,
    the exchange capacity sized from the RSS table's flows per rank."""
    out = run_bench_world(4, ["--frames", "2000000", "--steps", "2", "--warmup", "1",
                              "--c4-frames", "3000000", "--c4-steps", "2", "--no-cpu"],
                          timeout=600)
    assert out["n_gpus"] == 4 and out["dist"] == {"backend": "gloo", "world_size": 4}
    chk = out["check"]
    check_leg(chk, 4)
    assert chk["flows"] == 10_000 and chk["pkts_total"] == 4 * 2_000_000
    lo, hi = chk["flows_per_rank"]
    assert 0 < lo <= hi < 1.1 * 10_000 / 4
    c4 = out["config4_flowhash"]
    assert c4["frames_global"] == 12_000_000 and c4["flows"] == 1_000_000
    check_leg(c4["check"], 4)
    assert c4["check"]["pkts_total"] == 12_000_000
    lo4, hi4 = c4["check"]["flows_per_rank"]
    assert 240_000 < lo4 <= hi4 < 260_000


def test_bench_skewed_rss_refused_before_timing(gpu):
    """A deliberately skewed RSS table (every bucket but a few on rank 0) is refused
    while the shards are being sized — before any step is timed — with a clear
    message on every rank, instead of overflowing the exchange after the run."""
    import time
    t0 = time.perf_counter()
    r = launch(2, ["--frames", "2000000", "--steps", "2", "--warmup", "1", "--no-cpu",
                   "--no-extra"], timeout=300, TCBEE_BENCH_RSS="skew")
    assert r.returncode != 0
    assert "refused before the timed region" in r.stderr
    assert "steps in" not in r.stderr  # bench.run_device's "N steps in X ms" never logged
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert time.perf_counter() - t0 < 240


@pytest.mark.parametrize("shard", ["flowhash", "contig"])
def test_bench_world1_over_rccl(gpu, shard):
    """The RCCL branch of the exchange (dist.all_gather_flat / all_to_all_flat on
    "nccl", device tensors, no host staging) at world 1: torchrun with one rank,
    TCBEE_BENCH_FORCE_MERGE=1 so the N>1 code path (FlowHashExchange for flow-hash
    shards, OwnerExchange for contiguous ones, the counter all-reduce) runs over a
    one-rank RCCL communicator — RCCL refuses two ranks on one GPU, so this is the
    most of the collective path a one-GPU box can run; every record bit-exact."""
    out = run_bench_world(1, ["--frames", "4000000", "--steps", "2", "--warmup", "1",
                              "--no-cpu", "--no-extra", "--shard", shard],
                          TCBEE_DIST_BACKEND="nccl", TCBEE_BENCH_FORCE_MERGE="1")
    assert out["dist"] == {"backend": "nccl", "world_size": 1}
    assert out["config"]["shard"] == shard
    chk = out["check"]
    check_leg(chk, 1, full=shard == "flowhash")
    assert chk["flows"] == 10_000 and chk["pkts_total"] == 4_000_000


def test_k1_beside_a_second_process(gpu):
    """K1's look-back under another process's kernels on the same GPU (two gloo ranks
    on device 0, their K1s launched together): a predecessor whose XCD fell behind is
    polled for a bounded time, then recounted and published for the other waiters.
    With the old poll-count bound this took ~290x the K1 of one process alone
    (profiles/r05_lookback_contention.log); now ~2.7x. Bound: 15x."""
    args = ["--frames", "10000000", "--steps", "30", "--warmup", "3", "--no-cpu",
            "--no-extra", "--sample-check"]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    solo = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    both = run_bench_world(2, args, timeout=400)
    assert both["check"]["all_ranks_bit_exact"] is True
    k1_solo, k1_both = solo["roofline"]["k1_ms"], both["roofline"]["k1_ms"]
    assert k1_both < 15 * k1_solo, (k1_solo, k1_both)
