# one rocprofv3 --pmc pass over tools/bwd_probe.py; prints the counters of the backward kernel
# usage: bash tools/pmc_probe.sh <tag> "<counters>" "<mix> <B> <mode>"
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; CNT=$2; SPEC=$3
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
out=$R/gpurun_out/pmc_${TAG}
timeout -s KILL 90 rocprofv3 --pmc $CNT -d $out -o p --output-format csv -- python3 $R/tools/bwd_probe.py $SPEC > $out.log 2>&1 || { tail -n 5 $out.log; exit 1; }
python3 - $out/p_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "bwd" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(f"   {k:24s} per launch avg {sum(v)/len(v):14.1f}  (launches {len(v)})")
PY
