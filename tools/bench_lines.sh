# The round's bench lines (BASELINE configs 2-5), one JSON line each under gpurun_out/.
# usage: bash tools/bench_lines.sh <tag> [names...]   (default: all)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-lines}
shift || true
cd $R && mkdir -p gpurun_out
declare -A LINES=(
  [tb]="--steps 20 --warmup 5"
  [tb_periodic]="--steps 400 --warmup 5 --scale-period 200 --use-packed --gather-batch 0 --mlp-iters 0 --cpu-baseline 0"
  [tb_unfused]="--steps 20 --warmup 5 --unfused-local --gather-batch 0 --mlp-iters 0 --cpu-baseline 0"
  [kaggle_dp]="--config kaggle --steps 50 --warmup 5 --gather-batch 0 --mlp-iters 0"
  [kaggle_fwd128]="--config kaggle --mode fwd --batch-per-gpu 128 --steps 200 --warmup 20 --gather-batch 0 --mlp-iters 0"
  [kaggle_fwd128_graph]="--config kaggle --mode fwd --batch-per-gpu 128 --steps 200 --warmup 24 --graph --gather-batch 0 --mlp-iters 0 --cpu-baseline 0"
  [kaggle_sgd128]="--config kaggle --mode sgd --batch-per-gpu 128 --steps 200 --warmup 20 --gather-batch 0 --mlp-iters 0"
  [kaggle_sgd128_graph]="--config kaggle --mode sgd --batch-per-gpu 128 --steps 200 --warmup 24 --graph --gather-batch 0 --mlp-iters 0 --cpu-baseline 0"
)
ORDER="tb tb_periodic tb_unfused kaggle_dp kaggle_fwd128 kaggle_fwd128_graph kaggle_sgd128 kaggle_sgd128_graph"
NAMES=${*:-$ORDER}
for n in $NAMES; do
  timeout -k 10 300 python bench.py ${LINES[$n]} > gpurun_out/${TAG}_bench_${n}.log 2>&1 || { echo "FAILED $n"; tail -n 20 gpurun_out/${TAG}_bench_${n}.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_bench_${n}.log > gpurun_out/${TAG}_bench_${n}.json
  echo "$n $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['us_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['kernels_ms'])" gpurun_out/${TAG}_bench_${n}.json)"
done
