"""Per-kernel durations and the gaps between consecutive kernels (end -> next start)
from a rocprofv3 --kernel-trace CSV, over the last N kernels.
  python tools/gap_trace.py gpurun_out/c2tr [--last 400]
"""
import argparse
import csv
import glob
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=400)
    a = ap.parse_args()
    f = glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-a.last:]
    gaps, durs = defaultdict(list), defaultdict(list)
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:36]
    for x, y in zip(rows, rows[1:]):
        gaps[f"{name(x)} -> {name(y)}"].append((int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3)
    for r in rows:
        durs[name(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in durs.items():
        print(f"kernel {k}: {len(v)} x {sum(v) / len(v):.2f} us")
    for k, v in gaps.items():
        print(f"gap {k}: {len(v)} x {sum(v) / len(v):.2f} us")


if __name__ == "__main__":
    main()
