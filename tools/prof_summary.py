#!/usr/bin/env python3
"""Turn rocprofv3 outputs under gpurun_out/ into committed summaries under profiles/.

  python tools/prof_summary.py ROUND_TAG
reads  gpurun_out/prof/run_kernel_stats.csv (+ run_kernel_trace.csv)
       gpurun_out/pmc_fetch/run_counter_collection.csv, gpurun_out/pmc_write/...
writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_summary.md,
       profiles/pmc_k_parse.json (read by bench.py for roofline.traffic)

HBM traffic per k_parse launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes):
on gfx950 FETCH_SIZE counts exactly half the bytes of a wide streaming read
(MI355X_MICROARCH.md "HBM"); calibrated on this kernel by the 64-B workload,
whose reads are known (arena 64 B + index 20 B per frame).
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def pmc_values(path, kernel_sub):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if kernel_sub in r["Kernel_Name"]]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    lines = [f"# rocprofv3 summary — {tag}", ""]
    stats = os.path.join(OUT, "prof", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
        lines += ["Command: `rocprofv3 --kernel-trace --stats -- python bench.py --steps 10 "
                  "--no-cpu --no-extra --sample-check` (config 3: 100M IMIX frames, 10k flows).", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(stats)):
            lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | "
                         f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    f = os.path.join(OUT, "pmc_fetch", "run_counter_collection.csv")
    w = os.path.join(OUT, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(f) and os.path.exists(w):
        fk = pmc_values(f, "k_parse")
        wk = pmc_values(w, "k_parse")
        fetch = statistics.median(fk) * 1024 * 2
        write = statistics.median(wk) * 1024
        traffic = fetch + write
        pmc = {"kernel": "k_parse", "workload": "config3 100M IMIX 10k flows",
               "frames": 100_000_000, "sizes": "imix", "flows": 10_000,
               "fetch_bytes_corrected": fetch, "write_bytes": write,
               "traffic_bytes_per_launch": traffic, "fetch_size_kib_raw": statistics.median(fk),
               "write_size_kib_raw": statistics.median(wk), "dispatches": len(fk),
               "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KiB->B"}
        json.dump(pmc, open(os.path.join(PROF, "pmc_k_parse.json"), "w"), indent=1)
        lines += ["## HBM traffic of k_parse (separate --pmc passes)", "",
                  f"- FETCH_SIZE {statistics.median(fk):.0f} KiB raw -> {fetch / 1e9:.2f} GB "
                  "(x2 gfx950 correction)",
                  f"- WRITE_SIZE {statistics.median(wk):.0f} KiB -> {write / 1e9:.2f} GB",
                  f"- traffic per launch {traffic / 1e9:.2f} GB = {traffic / 1e8:.1f} B/frame "
                  "(algorithmic 156 B/frame)", ""]
        for name in ("pmc_fetch", "pmc_write"):
            src = os.path.join(OUT, name, "run_counter_collection.csv")
            dst = os.path.join(PROF, f"{tag}_{name}.csv")
            with open(src) as fi, open(dst, "w") as fo:
                rd = csv.DictReader(fi)
                cols = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size",
                        "LDS_Block_Size", "VGPR_Count", "Counter_Name", "Counter_Value"]
                wr = csv.writer(fo)
                wr.writerow(cols)
                for r in rd:
                    if "tcbee" in r["Kernel_Name"]:
                        wr.writerow([r[c] for c in cols])
    c4 = os.path.join(OUT, "c4prof", "run_kernel_stats.csv")
    if os.path.exists(c4):
        shutil.copy(c4, os.path.join(PROF, f"{tag}_config4_kernel_stats.csv"))
        lines += ["## config 4, one GPU's share", "",
                  "Command: `rocprofv3 --kernel-trace --stats -- python bench.py --config4 "
                  "--virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra --sample-check` "
                  "(rank 0's flow-hash shard of 1B IMIX frames / 8 GPUs: ~125M frames, "
                  "~125k flows; K3 in its bucketed mode).", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(c4)):
            if "tcbee" in r["Name"]:
                lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | "
                             f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    bench_log = os.path.join(OUT, "bench.log")
    if os.path.exists(bench_log):
        for ln in open(bench_log):
            if ln.startswith("{"):
                shutil.copy(bench_log, os.path.join(PROF, f"{tag}_bench.json"))
                with open(os.path.join(PROF, f"{tag}_bench.json"), "w") as fo:
                    fo.write(ln)
                lines += ["## bench.py line", "", "```", ln.strip(), "```", ""]
    open(os.path.join(PROF, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
