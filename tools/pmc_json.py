#!/usr/bin/env python3
"""Median per-launch PMC values of selected kernels from rocprofv3 --pmc passes.

  python tools/pmc_json.py OUT.json "WORKLOAD TEXT" KERNEL_SUBSTR[,..] PASS_DIR...
reads gpurun_out/<PASS_DIR>/run_counter_collection.csv for each pass and writes
{kernel: {counter: median over launches}} plus derived per-wave and HBM figures
(FETCH_SIZE x2: the gfx950 half-count correction, MI355X_MICROARCH.md "HBM").
"""
import collections
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out, workload, kernels, passes = sys.argv[1], sys.argv[2], sys.argv[3].split(","), sys.argv[4:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in passes:
        path = os.path.join(ROOT, "gpurun_out", p, "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            for k in kernels:
                if k in r["Kernel_Name"]:
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"workload": workload, "passes": passes, "kernels": {}}
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        d = {"median_per_launch": med}
        w = med.get("SQ_WAVES")
        if w:
            d["per_wave"] = {c[3:]: round(v / w, 1) for c, v in med.items()
                             if c.startswith("SQ_") and c not in ("SQ_WAVES",)}
        if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
            d["wait_any_fraction"] = round(med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"], 3)
        if "SQ_LDS_BANK_CONFLICT" in med and med.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_fraction"] = round(med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"], 3)
        if "TCC_HIT_sum" in med:
            d["l2_hit_rate"] = round(med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 3)
        if "FETCH_SIZE" in med:
            d["hbm_read_bytes_corrected"] = med["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in med:
            d["hbm_write_bytes"] = med["WRITE_SIZE"] * 1024
        res["kernels"][k] = d
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
