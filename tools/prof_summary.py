#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py (tools/prof_cfg.sh) into profiles/:

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim copy)
  <tag>_summary.json       per libdqrm kernel: calls, average and MEDIAN duration (us, the
                           median from the per-dispatch kernel trace, so a rare outlier
                           does not move roofline fractions), and the
                           per-launch HBM traffic from the separate --pmc passes:
                           FETCH_SIZE x 2 (gfx950 reports half the bytes of wide coalesced
                           reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, in bytes.
bench.py reads <tag>_summary.json (if present) to fill roofline.traffic.

usage: python tools/prof_summary.py gpurun_out/prof_tb profiles/r1_tb
"""
import collections
import csv
import json
import re
import shutil
import sys


def short(name: str) -> str:
    m = re.search(r"k_[a-z0-9_]+(<[^>]*>)?", name)
    return m.group(0) if m else name[:80]


def main(src: str, tag: str) -> None:
    stats = f"{src}_trace/tb_kernel_stats.csv"
    shutil.copy(stats, f"{tag}_kernel_stats.csv")
    out = {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        if k.startswith("k_"):
            out[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    trace = stats.replace("kernel_stats.csv", "kernel_trace.csv")
    try:
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(trace)):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in out.items():
            d = sorted(durs.get(k, []))
            if d:
                v["median_us"] = d[len(d) // 2]
                v["p10_us"], v["p90_us"] = d[len(d) // 10], d[(len(d) * 9) // 10]
    except (OSError, KeyError, ValueError):
        pass
    counters = {}
    for f, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f"{src}_{f}/tb_counter_collection.csv")):
            if r["Counter_Name"] == cname:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
        counters[cname] = {k: sum(v) / len(v) for k, v in acc.items()}
    for k, v in out.items():
        fe = counters["FETCH_SIZE"].get(k)
        wr = counters["WRITE_SIZE"].get(k)
        v["fetch_size_bytes"] = fe
        v["write_size_bytes"] = wr
        v["hbm_bytes_per_launch"] = (2.0 * fe + wr) if fe is not None and wr is not None else None
    # the profiled bench line's workload: bench.pmc_traffic only uses a summary of the same one
    workload = None
    try:
        lines = [x for x in open(f"{src}_trace.log") if x.startswith("{")]
        if lines:
            roof = json.loads(lines[-1]).get("roofline") or {}
            workload = roof.get("workload_profiled")
    except (OSError, ValueError):
        pass
    json.dump({"source": src, "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving)",
               "workload": workload, "kernels": out}, open(f"{tag}_summary.json", "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
        hb = v["hbm_bytes_per_launch"]
        print(f"{k:32s} calls={v['calls']:4d} avg={v['avg_us']:10.2f} us  median={v.get('median_us', float('nan')):8.2f}"
              f"  hbm/launch="
              f"{(hb / 1e6 if hb is not None else float('nan')):10.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
