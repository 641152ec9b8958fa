"""The golden manifest (tests/golden/trace_manifest.json, written by
tests/golden/make_manifest.py): the seeded traces are regenerated bit for bit by
the host generator, and the CPU oracle still produces exactly the pinned records,
flow hashes, ids, counters and flow table for them. The GPU side of the same
manifest is tests/test_gpu_manifest.py."""
import json
import os

import pytest

from manifest_traces import CASES, result_digest, trace_digest

HERE = os.path.dirname(os.path.abspath(__file__))
MANIFEST = json.load(open(os.path.join(HERE, "golden", "trace_manifest.json")))["cases"]


def test_manifest_covers_every_case():
    assert sorted(MANIFEST) == sorted(CASES)


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_manifest(oracle, name):
    build, port, direction = CASES[name]
    want = MANIFEST[name]
    tr = build()
    assert tr.n == want["frames"]
    assert trace_digest(tr) == want["sha256_input"], "generator drifted"
    got = result_digest(*oracle.parse(tr, filter_port=port, direction=direction))
    for k, v in got.items():
        assert v == want[k], (name, k)
