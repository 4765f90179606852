#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py (tools/prof_cfg.sh) into profiles/:

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim copy)
  <tag>_summary.json       per libdqrm kernel: calls, average and MEDIAN duration (us, the
                           median from the per-dispatch kernel trace, so a rare outlier
                           does not move roofline fractions), and the
                           per-launch HBM traffic from the separate --pmc passes. Reads:
                           from the L2's memory-side read requests by size when the
                           request-size pass exists (128 x TCC_EA0_RDREQ_128B + 64 x _64B +
                           32 x _32B: exact for every access shape, profiles/r5_tcc_*),
                           else FETCH_SIZE x 2 (gfx950 tallies a 128-B request at 64 B,
                           MI355X_MICROARCH.md "HBM"; that doubles 64-B requests too).
                           Writes: WRITE_SIZE (64 B per 64-B request, 32 B per 32-B one:
                           exact). In bytes.
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
    # read requests by size (optional pass): bytes = 128 * _128B + 64 * _64B + 32 * _32B
    rd_exact = {}
    try:
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f"{src}_rdreq/tb_counter_collection.csv")):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in acc.items():
            mean = {c: sum(x) / len(x) for c, x in d.items()}
            rd_exact[k] = sum(mean.get(f"TCC_EA0_RDREQ_{n}B_sum", 0.0) * n for n in (32, 64, 128))
    except OSError:
        pass
    # write requests by size and L2 atomics (optional pass): where WRITE_SIZE goes
    wrq = {}
    try:
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f"{src}_wrreq/tb_counter_collection.csv")):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in acc.items():
            mean = {c: sum(x) / len(x) for c, x in d.items()}
            n64 = mean.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            wrq[k] = {"write_requests_64B": n64, "write_requests_32B": mean.get("TCC_EA0_WRREQ_sum", 0.0) - n64,
                      "atomic_requests": mean.get("TCC_EA0_ATOMIC_sum")}
    except OSError:
        pass
    for k, v in out.items():
        if k in wrq:
            v.update(wrq[k])
        fe = counters["FETCH_SIZE"].get(k)
        wr = counters["WRITE_SIZE"].get(k)
        v["fetch_size_bytes"] = fe
        v["write_size_bytes"] = wr
        v["read_bytes_by_request_size"] = rd_exact.get(k)
        rd = rd_exact.get(k, 2.0 * fe if fe is not None else None)
        v["hbm_bytes_per_launch"] = (rd + wr) if rd is not None and wr is not None else None
    # the profiled bench line's workload: bench.pmc_traffic only uses a summary of the same one
    workload = None
    try:
        lines = [x for x in open(f"{src}_trace.log") if x.startswith("{")]
        if lines:
            roof = json.loads(lines[-1]).get("roofline") or {}
            workload = roof.get("workload_profiled")
    except (OSError, ValueError):
        pass
    corr = ("hbm = reads by request size (128*RDREQ_128B + 64*RDREQ_64B + 32*RDREQ_32B) + WRITE_SIZE"
            if rd_exact else "hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving)")
    json.dump({"source": src, "correction": corr,
               "workload": workload, "kernels": out}, open(f"{tag}_summary.json", "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
        hb = v["hbm_bytes_per_launch"]
        print(f"{k:32s} calls={v['calls']:4d} avg={v['avg_us']:10.2f} us  median={v.get('median_us', float('nan')):8.2f}"
              f"  hbm/launch="
              f"{(hb / 1e6 if hb is not None else float('nan')):10.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
