"""Per-kernel launch-duration statistics (count, avg, median, p10, p90 in us) from a rocprofv3
--kernel-trace output directory, for kernels whose name contains a filter string.
usage: python tools/kmedian.py <rocprof dir> [filter]"""
import csv
import glob
import re
import sys

import numpy as np

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "::k_"
dur = {}
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt in n:
            m = re.search(r"k_[a-z0-9_]+(<[^>]*>)?", n)
            dur.setdefault(m.group(0) if m else n[:48], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(dur.items()):
    a = np.array(v)
    print(f"{n:48s} n={a.size:5d} avg={a.mean():7.2f} med={np.median(a):7.2f} "
          f"p10={np.percentile(a, 10):7.2f} p90={np.percentile(a, 90):7.2f} us")
