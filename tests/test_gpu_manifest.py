"""HIP path (C ABI, host entry point tcbee_parse_batch) against the golden
manifest: the pinned sha256 of records, flow hashes, dense ids and the exported
flow table, with the counters — no oracle run at test time (the manifest was
written by the oracle, tests/golden/make_manifest.py; tests/test_manifest.py
keeps the oracle on it)."""
import json
import os

import pytest

import tcbee_amd
from manifest_traces import CASES, result_digest, trace_digest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
MANIFEST = json.load(open(os.path.join(HERE, "golden", "trace_manifest.json")))["cases"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_hip_path_matches_manifest(gpu, name):
    build, port, direction = CASES[name]
    want = MANIFEST[name]
    tr = build()
    assert trace_digest(tr) == want["sha256_input"]
    with tcbee_amd.PacketParser(device=0, max_frames=tr.n, max_arena=len(tr.arena) + 64,
                                max_flows=1 << 16) as p:
        res = p.parse(tr, filter_port=port, direction=direction)
        got = result_digest(res.records, res.flow_hash, res.flow_id, res.counters, p.flows())
        assert p.status() == 0
    for k, v in got.items():
        assert v == want[k], (name, k)
