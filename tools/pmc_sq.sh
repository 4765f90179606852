# SQ counter passes (one rocprofv3 --pmc run per counter group, at most 8 SQ counters each) of a
# short bench.py run; prints each kernel's per-launch average of every counter.
# usage: bash tools/pmc_sq.sh <tag> "<bench args>" "<counters>" ["<counters>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ARGS=$2; shift 2
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "$@"; do
  i=$((i+1))
  out=$R/gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $out -o p --output-format csv -- python3 $R/bench.py $ARGS > $out.log 2>&1 || { tail -n 5 $out.log; exit 1; }
  python3 - $out/p_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    n = max(len(v) for v in d.values())
    print(f"{k:48s} n={n:4d}", " ".join(f"{c}={sum(v) / len(v):.0f}" for c, v in d.items()))
PY
done
