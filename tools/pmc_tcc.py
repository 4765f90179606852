"""L2 memory-side request counters (TCC_EA0_*) of one program, one rocprofv3 --pmc pass per
counter group (at most 4 TCC counters per pass), summarised per kernel as per-launch means.

Used to explain a kernel's 2*FETCH_SIZE + WRITE_SIZE figure (tools/prof_summary.py): the
gfx950 halving of FETCH_SIZE (MI355X_MICROARCH.md "HBM") is calibrated on wide streaming
reads; random 32/64-B row accesses may be tallied differently, so the request-size split is
read here and calibrated on known byte counts (tools/pmc_calib.py).

usage: python tools/pmc_tcc.py <tag> <counter list file> -- <program and args>
Writes gpurun_out/tcc_<tag>_<pass>/ and prints one line per kernel and pass. Stops at the
first pass that fails (no retries)."""
import collections
import csv
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# counter groups, each within the TCC block's 4 counters; FETCH_SIZE takes 3, WRITE_SIZE 2
GROUPS = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"],
    ["TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"],
    ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"],
    ["TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_WRREQ_DRAM_sum"],
]


def main():
    tag, listing = sys.argv[1], sys.argv[2]
    prog = sys.argv[sys.argv.index("--") + 1:]
    text = open(listing).read() if os.path.exists(listing) else ""
    have = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", text))
    out_root = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_root, exist_ok=True)
    for gi, grp in enumerate(GROUPS):
        # a derived counter (FETCH_SIZE) or a _sum of a listed base counter
        use = [c for c in grp if c in have or c.removesuffix("_sum") in have]
        if not use:
            print(f"pass {gi}: none of {grp} listed")
            continue
        d = os.path.join(out_root, f"tcc_{tag}_{gi}")
        cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *use, "-d", d, "-o", "p",
               "--output-format", "csv", "--", *prog]
        with open(d + ".log", "w") as log:
            rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, cwd="/tmp").returncode
        if rc != 0:
            print(f"pass {gi} {use}: rc {rc}; stopping (see {d}.log)")
            sys.exit(1)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for f in files:
            for r in csv.DictReader(open(f)):
                acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, dd in sorted(acc.items()):
            n = max(len(v) for v in dd.values())
            print(f"pass {gi} {k:60s} n={n:4d} " + " ".join(f"{c}={sum(v) / len(v):.0f}" for c, v in dd.items()))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
