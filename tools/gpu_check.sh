# GPU round check of the current tree (run through gpurun from the repo root):
#   all -m gpu tests, then short bench lines (TB dp, Kaggle dp, Kaggle config-3 sgd graph).
# usage: bash tools/gpu_check.sh <tag> [tests=1] [benches=1]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; TESTS=${2:-1}; BENCH=${3:-1}
cd $R && mkdir -p gpurun_out
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_gpu_tests.log; exit 1; }
  tail -n 1 gpurun_out/${T}_gpu_tests.log
fi
if [ "$BENCH" = 1 ]; then
  Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
  timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_bench_tb.log 2>&1 || { tail -n 20 gpurun_out/${T}_bench_tb.log; exit 1; }
  timeout -k 10 300 python bench.py --config kaggle $Q > gpurun_out/${T}_bench_kaggle.log 2>&1 || { tail -n 20 gpurun_out/${T}_bench_kaggle.log; exit 1; }
  timeout -k 10 300 python bench.py --config kaggle --mode sgd --batch-per-gpu 128 --graph --steps 400 --warmup 40 $Q > gpurun_out/${T}_bench_c3.log 2>&1 || { tail -n 20 gpurun_out/${T}_bench_c3.log; exit 1; }
  for f in tb kaggle c3; do tail -n 1 gpurun_out/${T}_bench_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['us_per_step'], d['kernels_ms'], d['roofline']['kernel'], d['roofline']['frac'])"; done
fi
