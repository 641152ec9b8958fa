#!/usr/bin/env python3
"""Per-kernel median durations (us) of the K3 kernels in gpurun_out/k3ab_<lib>_<i>/
kernel traces (tools/k3_ab.sh), split by workload in launch order."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

nwl = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for d in sorted(glob.glob("gpurun_out/k3ab_*_*/")):
    rows = []
    for f in glob.glob(d + "**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    for r in rows:
        k = r["Kernel_Name"]
        if not any(x in k for x in ("k_count", "k_parse")):
            continue
        per[k.split("(")[0].replace("void ", "").replace("tcbee::", "")].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for k, v in sorted(per.items()):
        if len(v) < nwl:
            continue
        step = len(v) // nwl
        out.append(f"{k}: " + " / ".join(f"{statistics.median(v[i * step:(i + 1) * step]):.1f}"
                                          for i in range(nwl)))
    print(d, "; ".join(out))
