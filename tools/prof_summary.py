#!/usr/bin/env python3
"""Turn one box's rocprofv3 outputs (tools/prof_legs.sh) into committed summaries.

  python tools/prof_summary.py TAG [--prefix r06prof]

reads only the directories of THIS run (no stale gpurun_out/ entries of older rounds):
  gpurun_out/<prefix>_c3/   kernel trace + stats of the headline command, and
  gpurun_out/<prefix>_c3.json  the bench line that same process printed
  gpurun_out/<prefix>_c4v8/ one GPU's flow-hash share of config 4 at N=8 (+ .json)
  gpurun_out/<prefix>_c4/   the whole 1M-flow config-4 trace on one GPU (+ .json)
  gpurun_out/<prefix>_c2/, _v6/  config 2 (per-launch breakdown of its step) and the
                            IPv6 leg (+ .json)
  gpurun_out/pmc_<leg>_{fetch,write,rdreq}/  K1 PMC passes (tools/pmc_c4.sh), legs
                            c3 / c4v8 / c4 / v6 when present and newer than the trace
writes profiles/<TAG>_summary.md, <TAG>_kernel_stats.csv, <TAG>_bench.json,
       <TAG>_config4_share_kernel_stats.csv, <TAG>_config4_whole_kernel_stats.csv,
       <TAG>_pmc_<leg>_*.csv, <TAG>_pmc_legs.json and profiles/pmc_k_parse.json (read by
       bench.py for roofline.traffic).

HBM traffic per k_parse launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on
gfx950 FETCH_SIZE counts half the bytes of a wide streaming read (MI355X_MICROARCH.md
"HBM"); the doubling is confirmed on this kernel by the TCC_EA0_RDREQ_128B pass.
"""
import argparse
import csv
import json
import os
import re
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")

LEGS = {"c3": ("config 3: 100M IMIX frames, 10k flows", "", "--no-extra --no-cpu"),
        "c4v8": ("config 4, one GPU's flow-hash share at N=8: ~125M frames, ~125k flows",
                 "--config4 --virtual-world 8",
                 "--config4 --virtual-world 8 --steps 5 --warmup 1 --no-cpu --no-extra"),
        "c4": ("config 4, the whole 1M-flow trace on one GPU: 125M IMIX frames",
               "--config4", "--config4 --shard contig --steps 5 --warmup 1 --no-cpu --no-extra"),
        "v6": ("config 3 over IPv6/TCP: 100M IMIX6 frames, 10k flows", "--sizes imix6",
               "--sizes imix6 --no-extra --no-cpu"),
        "c2": ("config 2: 1M 64-B frames, 1 flow", "--frames 1000000 --sizes 64 --flows 1",
               "--frames 1000000 --sizes 64 --flows 1 --steps 200 --warmup 20 --no-extra --no-cpu")}


def pmc_values(path, kernel_sub):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if kernel_sub in r["Kernel_Name"]]


def frames_of(log_path, fallback):
    try:
        m = re.search(r"rank 0: (\d+) frames resident", open(log_path).read())
        if m:
            return int(m.group(1))
    except OSError:
        pass
    return fallback


def stats_table(path):
    rows = ["| kernel | calls | avg us | min us | max us |", "|---|---|---|---|---|"]
    for r in csv.DictReader(open(path)):
        if "tcbee" in r["Name"]:
            rows.append(f"| `{r['Name'].split('(')[0].replace('void ', '')[:60]}` | {r['Calls']} | "
                        f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                        f"{float(r['MaxNs']) / 1e3:.1f} |")
    return rows


def trace_k1(path):
    """k_parse launches of a kernel trace: (all-launch average us, timed-step average
    us = the launches after the warm-up ones, their count)."""
    ds = [(int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
          for r in csv.DictReader(open(path)) if "k_parse" in r["Kernel_Name"]]
    ds = [d for _, d in sorted(ds)]
    return statistics.mean(ds) if ds else None, ds


def c2_breakdown(path, skip=20):
    """Config 2's step launch by launch (the timed steps of a trace: warm-up skipped):
    the average duration of each kernel of a step and the gaps between consecutive
    launches, from start/end timestamps."""
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1])
                   for r in csv.DictReader(open(path)) if "tcbee" in r["Kernel_Name"]))
    steps, cur = [], []
    for row in rows:  # a step starts at each k_prep or (fused small contexts) each k_parse
        if row[2] in ("k_prep", "k_parse") and cur and any(x[2] == "k_parse" for x in cur):
            steps.append(cur)
            cur = []
        cur.append(row)
    if cur:
        steps.append(cur)
    steps = [s for s in steps if any(x[2] == "k_parse" for x in s)][skip:]
    if not steps:
        return []
    shape = [x[2] for x in steps[0]]
    steps = [s for s in steps if [x[2] for x in s] == shape]
    out = [f"Per-launch breakdown over {len(steps)} timed steps (kernel trace timestamps):", "",
           "| # | kernel | avg us | gap before (us) |", "|---|---|---|---|"]
    for i, name in enumerate(shape):
        dur = statistics.mean((s[i][1] - s[i][0]) / 1e3 for s in steps)
        gap = statistics.mean((s[i][0] - s[i - 1][1]) / 1e3 for s in steps) if i else \
            statistics.mean((b[0][0] - a[-1][1]) / 1e3 for a, b in zip(steps, steps[1:]))
        out.append(f"| {i} | `{name}` | {dur:.1f} | {gap:.1f} |")
    span = statistics.mean((b[0][0] - a[0][0]) / 1e3 for a, b in zip(steps, steps[1:]))
    out += ["", f"Start-to-start step period {span:.1f} us."]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--prefix", default="r06prof")
    a = ap.parse_args()
    tag, pre = a.tag, a.prefix
    os.makedirs(PROF, exist_ok=True)
    lines = [f"# rocprofv3 summary — {tag}", ""]
    c3 = os.path.join(OUT, f"{pre}_c3")
    if os.path.isdir(c3):
        shutil.copy(os.path.join(c3, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_kernel_stats.csv"))
        line = next(ln for ln in open(os.path.join(OUT, f"{pre}_c3.json")) if ln.startswith("{"))
        open(os.path.join(PROF, f"{tag}_bench.json"), "w").write(line)
        b = json.loads(line)
        avg, ds = trace_k1(os.path.join(c3, "run_kernel_trace.csv"))
        timed = ds[b["warmup"]:b["warmup"] + b["steps"]]
        n = b["config"]["frames_per_gpu"]
        alg = n * b["roofline"]["alg_bytes_per_frame"]
        lines += [f"Command: `rocprofv3 --kernel-trace --stats -- python bench.py {LEGS['c3'][2]}` "
                  f"({LEGS['c3'][0]}); the bench line below is the one this process printed.", ""]
        lines += stats_table(os.path.join(c3, "run_kernel_stats.csv")) + [""]
        lines += [f"k_parse: {len(ds)} launches, average {avg:.1f} us over all of them (warm-up "
                  f"included); the {len(timed)} timed steps' launches average "
                  f"{statistics.mean(timed):.1f} us -> {alg / statistics.mean(timed) / 1e3:.1f} GB/s "
                  f"algorithmic = frac {alg / statistics.mean(timed) / 1e3 / 8000:.4f} of 8 TB/s; "
                  f"the line's HIP-event K1 {b['roofline']['k1_ms'] * 1e3:.1f} us "
                  f"(frac {b['roofline']['frac']}).", "",
                  "```", line.strip(), "```", ""]
    for leg, name, title in (("c4v8", "config4_share", "config 4, one GPU's flow-hash share at N=8"),
                             ("c4", "config4_whole", "config 4, the whole 1M-flow trace on one GPU"),
                             ("v6", "ipv6", "config 3 over IPv6/TCP (100M IMIX6 frames)"),
                             ("c2", "config2", "config 2 (1M x 64 B, one flow): the step per launch")):
        d = os.path.join(OUT, f"{pre}_{leg}")
        if not os.path.isdir(d):
            continue
        shutil.copy(os.path.join(d, "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_{name}_kernel_stats.csv"))
        lines += [f"## {title}", "",
                  f"Command: `rocprofv3 --kernel-trace --stats -- python bench.py {LEGS[leg][2]}`.", ""]
        lines += stats_table(os.path.join(d, "run_kernel_stats.csv")) + [""]
        if leg == "c2":
            lines += c2_breakdown(os.path.join(d, "run_kernel_trace.csv")) + [""]
        try:
            ln = next(x for x in open(os.path.join(OUT, f"{pre}_{leg}.json")) if x.startswith("{"))
            bl = json.loads(ln)
            lines += [f"Line: {bl['value']} Mpkt/s, {bl['ms_per_step']} ms/step, K1 "
                      f"{bl['roofline']['k1_ms']} ms (events), frames {bl['check'].get('frames_local', bl['config'].get('frames_per_gpu'))}, "
                      f"flows {bl['check'].get('flows')}.", ""]
        except (OSError, StopIteration):
            pass
    pmc_legs = {}
    t_trace = os.path.getmtime(c3) if os.path.isdir(c3) else 0
    for leg, (what, args, _) in LEGS.items():
        paths = {k: os.path.join(OUT, f"pmc_{leg}_{k}", "run_counter_collection.csv")
                 for k in ("fetch", "write", "rdreq")}
        if not all(os.path.exists(x) for x in paths.values()):
            continue
        if min(os.path.getmtime(x) for x in paths.values()) < t_trace - 3600:
            continue  # an older box's passes
        fk = statistics.median(pmc_values(paths["fetch"], "k_parse"))
        wk = statistics.median(pmc_values(paths["write"], "k_parse"))
        rd = {}
        for r in csv.DictReader(open(paths["rdreq"])):
            if "k_parse" in r["Kernel_Name"]:
                rd.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        rd = {k: statistics.median(v) for k, v in rd.items()}
        frames = frames_of(os.path.join(OUT, f"pmc_{leg}_fetch.log"),
                           {"c3": 100_000_000, "v6": 100_000_000,
                            "c2": 1_000_000}.get(leg, 125_000_000))
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
        if leg == "c3":  # bench.py's roofline.traffic (pmc_traffic reads these keys)
            json.dump({"kernel": "k_parse", "workload": "config3 100M IMIX 10k flows",
                       "frames": frames, "sizes": "imix", "flows": 10000,
                       "fetch_bytes_corrected": fetch, "write_bytes": write,
                       "traffic_bytes_per_launch": fetch + write, "fetch_size_kib_raw": fk,
                       "write_size_kib_raw": wk,
                       "dispatches": len(pmc_values(paths["fetch"], "k_parse")),
                       "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KiB->B",
                       "source": f"profiles/{tag}_pmc_c3_fetch.csv + {tag}_pmc_c3_write.csv"},
                      open(os.path.join(PROF, "pmc_k_parse.json"), "w"), indent=1)
    if pmc_legs:
        json.dump(pmc_legs, open(os.path.join(PROF, f"{tag}_pmc_legs.json"), "w"), indent=1)
        lines += ["## k_parse HBM-side traffic per leg (separate --pmc passes; FETCH x2)", "",
                  "| leg | read B/frame | write B/frame | total B/frame | L2->fabric read requests/frame |",
                  "|---|---|---|---|---|"]
        for leg, v in pmc_legs.items():
            lines.append(f"| {v['workload']} | {v['read_B_per_frame']} | {v['write_B_per_frame']} | "
                         f"{v['traffic_B_per_frame']} | {v['rdreq_per_frame']} |")
        lines.append("")
    open(os.path.join(PROF, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
