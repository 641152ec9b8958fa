"""The seeded traces of the golden manifest (tests/golden/trace_manifest.json):
one definition shared by the generator script and the tests, so the manifest,
the CPU check of the oracle and the GPU check of the HIP path all see the same
bytes. Sizes follow SURVEY.md §8(c)/(d): config 2 in full (1M x 64 B, one flow),
slices of config 3 (IMIX, 10k flows; uniform and Zipf), IPv6 frames, and a mixed
adversarial trace through both hooks with and without FILTER_PORT."""
from __future__ import annotations

import hashlib

import numpy as np

import tcbee_amd
from tcbee_amd.trace import GEN_MULTI, GEN_MULTI_V6, GEN_SINGLE, GEN_ZIPF

SEED = 0x7CBEE

# name -> (builder, filter_port, direction)
CASES = {
    "config2_1M_64B": (lambda: tcbee_amd.synth_trace(1_000_000, sizes="64", kind=GEN_SINGLE,
                                                     n_flows=1, seed=SEED), 0, 0),
    "config3_imix_2M": (lambda: tcbee_amd.synth_trace(2_000_000, sizes="imix", kind=GEN_MULTI,
                                                      n_flows=10_000, seed=SEED), 0, 0),
    "config3_zipf_1M": (lambda: tcbee_amd.synth_trace(1_000_000, sizes="imix", kind=GEN_ZIPF,
                                                      n_flows=10_000, seed=SEED), 0, 0),
    "ipv6_imix6_500k": (lambda: tcbee_amd.synth_trace(500_000, sizes="imix6",
                                                      kind=GEN_MULTI_V6, n_flows=10_000,
                                                      seed=SEED), 0, 0),
    "mixed_300k_xdp": (lambda: _mixed(), 0, 0),
    "mixed_300k_tc_port5201": (lambda: _mixed(), 5201, 1),
}


def _mixed():
    from tracegen import mixed_trace
    return mixed_trace(300_000, seed=2025, n_flows=4096)


def _sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def trace_digest(tr) -> str:
    """sha256 over the input: arena bytes, then offset u64, caplen u32, ts u64."""
    return _sha(tr.arena, tr.offset, tr.caplen, tr.ts_ns)


def result_digest(rec, fh, fi, ctr, table) -> dict:
    """What the manifest pins for one parse: record count, flow count, counters and
    sha256 of the 74-B records, the flow hashes, the dense flow ids and the exported
    flow table (FLOW_DTYPE rows), plus the first and last two records in hex."""
    rec = np.asarray(rec, dtype=np.uint8).reshape(-1, 74)
    n = len(rec)
    ends = sorted(set(list(range(min(n, 2))) + list(range(max(0, n - 2), n))))
    return {
        "records": n,
        "flows": int(len(table)),
        "counters": {k: int(v) for k, v in ctr.items()},
        "sha256_records": _sha(rec),
        "sha256_flow_hash": _sha(np.asarray(fh, dtype=np.uint32)),
        "sha256_flow_id": _sha(np.asarray(fi, dtype=np.uint32)),
        "sha256_flow_table": _sha(table),
        "records_hex": {str(i): rec[i].tobytes().hex() for i in ends},
    }
