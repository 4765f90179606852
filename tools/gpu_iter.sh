# One build -> measure iteration on the GPU box: selected GPU tests, the default bench line,
# and a rocprofv3 kernel-trace summary of a short bench run.
# usage: bash tools/gpu_iter.sh <tag> "<pytest -k expr>" ["<bench args>"]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; K=$2; BARGS=${3:-"--steps 20 --warmup 5"}
cd $R && mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -n 40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -n 2 gpurun_out/${TAG}_tests.log
fi
timeout -k 10 300 python bench.py $BARGS > gpurun_out/${TAG}_bench.log 2>&1 || { tail -n 20 gpurun_out/${TAG}_bench.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('BENCH', d['value'], d['us_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['kernels_ms'])" gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o p --output-format csv -- python3 $R/bench.py $BARGS --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > $R/gpurun_out/prof_${TAG}.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_${TAG}.log; exit 1; }
python3 - $R/gpurun_out/prof_${TAG}/p_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["AverageNs"]) < 200000:
        print(f"   {r['Name'][:64]:64s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
