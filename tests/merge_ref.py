"""Reference (numpy) merge of per-rank flow tables — the checker for the device
merge (tcbee_flow_merge_device) and for the gloo choreography tests.

Semantics: segments are consecutive slices of one record stream;
flows equal by key are one flow; pkts/bytes summed; first_seen = records of
earlier segments + local first_seen, minimised; ids in global first-seen order.
"""
import numpy as np

from tcbee_amd.parser import FLOW_DTYPE


def entries_to_table(ent: np.ndarray, count: int) -> np.ndarray:
    """int64 [cap, 8] -> FLOW_DTYPE [count]"""
    return np.ascontiguousarray(ent[:count]).view(FLOW_DTYPE).reshape(-1)


def table_to_entries(table: np.ndarray, cap: int) -> np.ndarray:
    out = np.zeros((cap, 8), dtype=np.int64)
    out[:len(table)] = table.view(np.int64).reshape(-1, 8)
    return out


def merge(tables, records):
    """tables: list of FLOW_DTYPE arrays (per segment); records: records per segment.
    Returns (merged FLOW_DTYPE table in id order, [per-segment local->global id maps])."""
    base = np.concatenate([[0], np.cumsum(records)[:-1]]).astype(np.uint64)
    acc = {}
    order = []
    for r, t in enumerate(tables):
        for e in t:
            k = e["tuple"].tobytes()
            fs = int(e["first_seen"]) + int(base[r])
            if k not in acc:
                acc[k] = [int(e["pkts"]), int(e["bytes"]), fs]
                order.append(k)
            else:
                a = acc[k]
                a[0] += int(e["pkts"])
                a[1] += int(e["bytes"])
                a[2] = min(a[2], fs)
    keys = sorted(order, key=lambda k: acc[k][2])
    gid = {k: i for i, k in enumerate(keys)}
    out = np.zeros(len(keys), dtype=FLOW_DTYPE)
    for i, k in enumerate(keys):
        out[i]["tuple"] = np.frombuffer(k, dtype=np.uint8)
        out[i]["pkts"], out[i]["bytes"], out[i]["first_seen"] = acc[k]
    maps = [np.array([gid[e["tuple"].tobytes()] for e in t], dtype=np.uint32) for t in tables]
    return out, maps
