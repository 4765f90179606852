# instruction-fetch counters of the backward kernels (tools/bwd_probe.py), one pass per counter group
# usage: bash tools/pmc_icache.sh <tag> "<mix> <B> <mode>"
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; SPEC=$2
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  out=$R/gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 90 rocprofv3 --pmc $CNT -d $out -o p --output-format csv -- python3 $R/tools/bwd_probe.py $SPEC > $out.log 2>&1 || { tail -n 5 $out.log; exit 1; }
  python3 - $out/p_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.0f}" for c, v in d.items()))
PY
done
