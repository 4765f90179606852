"""Print libdqrm kernels of a rocprofv3 kernel_stats.csv: calls, avg / median-free min / max (us)."""
import csv
import sys

for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        if "anonymous namespace)::k_" in n:
            short = n.split("::", 1)[1].split("(")[0]
            print(f"  {short:28s} calls={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:7.2f}us "
                  f"min={float(r['MinNs']) / 1e3:7.2f} max={float(r['MaxNs']) / 1e3:7.2f}")
