# K4a/K4b average durations per table mix (tools/bwd_probe.py under rocprofv3 --kernel-trace --stats)
# usage: bash tools/probe_bwd.sh <tag> "<mix> <B> <mode>" ["<mix> <B> <mode>" ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  out=$R/gpurun_out/probe_${TAG}_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o p --output-format csv -- python3 $R/tools/bwd_probe.py $spec > $out.log 2>&1 || { tail -n 20 $out.log; exit 1; }
  grep -h "T=" $out.log
  python3 - $out/p_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "k_sort" in n or "k_bwd" in n or "finalize" in n:
        print(f"   {n[:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:7.2f} min_us={float(r['MinNs'])/1e3:7.2f}")
PY
done
