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


def leg_frames(leg: str) -> int:
    """Frames per k_parse launch of a PMC leg: the bench's own "<n> frames resident"
    log line (gpurun_out/pmc_<leg>_fetch.log, tools/pmc_c4.sh), else the nominal config size."""
    import re
    log = os.path.join(OUT, f"pmc_{leg}_fetch.log")
    try:
        m = re.search(r"rank 0: (\d+) frames resident", open(log).read())
        if m:
            return int(m.group(1))
    except OSError:
        pass
    if leg == "c4v8":
        sys.exit(f"{log}: no 'frames resident' line (the shard size is seed-dependent)")
    return 100_000_000 if leg == "c3" else 125_000_000


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if tag.startswith("-") or "/" in tag:
        sys.exit(f"usage: {sys.argv[0]} ROUND_TAG  (a tag such as r03; got {tag!r})")
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
    if not os.path.exists(f):  # tools/pmc_c4.sh layout (config-3 leg)
        f = os.path.join(OUT, "pmc_c3_fetch", "run_counter_collection.csv")
        w = os.path.join(OUT, "pmc_c3_write", "run_counter_collection.csv")
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
            if not os.path.exists(src):
                src = os.path.join(OUT, name.replace("pmc_", "pmc_c3_"), "run_counter_collection.csv")
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
                  "~125k flows).", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(c4)):
            if "tcbee" in r["Name"]:
                lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | "
                             f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    legs = {"c3": ("config 3: 100M IMIX frames, 10k flows", ""),
            "c4": ("config 4, whole 1M-flow trace on one GPU: 125M IMIX frames", "--config4"),
            "c4v8": ("config 4, one GPU's flow-hash share at N=8: ~125M frames, ~125k flows",
                     "--config4 --virtual-world 8"),
            "v6": ("config 3 over IPv6/TCP: 100M IMIX6 (78/576/1500) frames, 10k flows",
                   "--sizes imix6")}
    pmc_legs = {}
    for leg, (what, args) in legs.items():
        paths = {k: os.path.join(OUT, f"pmc_{leg}_{k}", "run_counter_collection.csv")
                 for k in ("fetch", "write", "rdreq")}
        if not all(os.path.exists(x) for x in paths.values()):
            continue
        fk = statistics.median(pmc_values(paths["fetch"], "k_parse"))
        wk = statistics.median(pmc_values(paths["write"], "k_parse"))
        rd = {}
        for r in csv.DictReader(open(paths["rdreq"])):
            if "k_parse" in r["Kernel_Name"]:
                rd.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        rd = {k: statistics.median(v) for k, v in rd.items()}
        # frames the PMC'd k_parse launches parsed: from the leg's bench log ("N frames
        # resident"), written beside the counter CSVs by tools/pmc_c4.sh
        frames = leg_frames(leg)
        fetch, write = fk * 1024 * 2, wk * 1024
        pmc_legs[leg] = {"workload": what, "command": "bench.py --steps 2 --warmup 1 --no-cpu "
                         f"--no-extra --sample-check {args}".strip(), "frames": frames,
                         "fetch_bytes_corrected": fetch, "write_bytes": write,
                         "read_B_per_frame": round(fetch / frames, 1),
                         "write_B_per_frame": round(write / frames, 1),
                         "traffic_B_per_frame": round((fetch + write) / frames, 1),
                         "rdreq": rd, "rdreq_per_frame": round(rd.get("TCC_EA0_RDREQ_sum", 0) / frames, 3)}
        for k, src in paths.items():
            with open(src) as fi, open(os.path.join(PROF, f"{tag}_pmc_{leg}_{k}.csv"), "w") as fo:
                rdr = csv.DictReader(fi)
                cols = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size",
                        "LDS_Block_Size", "VGPR_Count", "Counter_Name", "Counter_Value"]
                wr = csv.writer(fo)
                wr.writerow(cols)
                for r in rdr:
                    if "tcbee" in r["Kernel_Name"]:
                        wr.writerow([r[c] for c in cols])
    if pmc_legs:
        json.dump(pmc_legs, open(os.path.join(PROF, f"{tag}_pmc_legs.json"), "w"), indent=1)
        lines += ["## k_parse HBM-side traffic per leg (separate --pmc passes; FETCH x2)", "",
                  "| leg | read B/frame | write B/frame | total B/frame | L2->fabric read requests/frame |",
                  "|---|---|---|---|---|"]
        for leg, v in pmc_legs.items():
            lines.append(f"| {v['workload']} | {v['read_B_per_frame']} | {v['write_B_per_frame']} | "
                         f"{v['traffic_B_per_frame']} | {v['rdreq_per_frame']} |")
        lines.append("")
    c4f = os.path.join(OUT, "c4fprof", "run_kernel_stats.csv")
    if os.path.exists(c4f):
        shutil.copy(c4f, os.path.join(PROF, f"{tag}_config4_whole_kernel_stats.csv"))
        lines += ["## config 4, the whole 1M-flow trace on one GPU", "",
                  "Command: `rocprofv3 --kernel-trace --stats -- python bench.py --config4 "
                  "--shard contig --steps 5 --warmup 1 --no-cpu --no-extra --sample-check` "
                  "(125M IMIX frames, 1M flows: every flow in one table).", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(c4f)):
            if "tcbee" in r["Name"]:
                lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | "
                             f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    small = os.path.join(OUT, "smallprof", "run_kernel_stats.csv")
    if os.path.exists(small):
        shutil.copy(small, os.path.join(PROF, f"{tag}_config2_kernel_stats.csv"))
        lines += ["## config 2 (1M x 64 B, 1 flow)", "",
                  "Command: `rocprofv3 --kernel-trace --stats -- python tools/k1_sweep.py "
                  "--frames 1000000 --fpl 2 --workloads 64B1 --rounds 1 --iters 20` "
                  "(flows on and off variants).", "",
                  "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
        for r in csv.DictReader(open(small)):
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
