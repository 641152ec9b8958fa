"""Dump the reference's committed ts-storage/db.sqlite into a JSON fixture.

That database is what the reference's own test (ts-storage/tests/sqlite.rs.rs,
`all_func`) leaves behind: flow create/delete, attribute add/set/delete, one
time series, a single point, a 4-point batch, a REJECTED 2-point batch with a
duplicate timestamp (99.0 twice), then an accepted batch reusing 99.0. It pins
the schema and the all-or-nothing semantics of insert_multiple_points.

Run here (where /root/reference exists); the JSON is committed. The database is
opened read-only with the standard sqlite3 module (data only, nothing executed).

  python tests/golden/make_tsdb_fixture.py [/root/reference/ts-storage/db.sqlite]
"""
import json
import os
import sqlite3
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/ts-storage/db.sqlite"


def schema(c):
    out = {}
    for (t,) in c.execute("SELECT name FROM sqlite_master WHERE type='table' ORDER BY name"):
        out[t] = {
            "columns": [list(r) for r in c.execute(f"PRAGMA table_info({t})")],
            "foreign_keys": [list(r)[2:] for r in c.execute(f"PRAGMA foreign_key_list({t})")],
            "unique": sorted([[r[2], [x[2] for x in c.execute(f"PRAGMA index_info({r[1]})")]]
                              for r in c.execute(f"PRAGMA index_list({t})")]),
        }
    return out


def main():
    c = sqlite3.connect(f"file:{SRC}?mode=ro", uri=True)
    rows = {}
    for t, order in (("flows", "id"), ("flow_attributes", "id"),
                     ("time_series", "time_series_id"),
                     ("time_series_data", "time_series_id, timestamp"),
                     ("sqlite_sequence", "name")):
        rows[t] = [list(r) for r in c.execute(f"SELECT * FROM {t} ORDER BY {order}")]
    doc = {"source": "ts-storage/db.sqlite (reference, left by tests/sqlite.rs.rs all_func)",
           "schema": schema(c), "rows": rows}
    with open(os.path.join(HERE, "ts_storage_db.json"), "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", os.path.join(HERE, "ts_storage_db.json"))


if __name__ == "__main__":
    main()
