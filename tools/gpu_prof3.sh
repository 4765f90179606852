# GPU tests (optional) + rocprofv3 kernel traces of the three bench lines (TB dp, Kaggle dp,
# Kaggle config-3 sgd at B=128), default kernel choices.  usage: bash tools/gpu_prof3.sh <tag> [tests=1]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
if [ "${2:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_gpu_tests.log; exit 1; }
  tail -n 1 gpurun_out/${T}_gpu_tests.log
fi
cd /tmp && export TMPDIR=/tmp
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
run() {  # <name> <args...>
  n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p3_${T}_$n -o k --output-format csv -- python3 $R/bench.py "$@" $Q > $R/gpurun_out/p3_${T}_$n.log 2>&1 || { tail -n 20 $R/gpurun_out/p3_${T}_$n.log; exit 1; }
  echo "$n $(grep -o '"us_per_step": [0-9.]*' $R/gpurun_out/p3_${T}_$n.log)"
  python3 $R/tools/kstats.py $(find $R/gpurun_out/p3_${T}_$n -name "*kernel_stats.csv") | grep -E "apply|finalize|coalesce|emb_fwd|sgd|bwd"
}
run tb --config terabyte --steps 50 --warmup 10
run kaggle --config kaggle --steps 50 --warmup 10
run c3 --config kaggle --mode sgd --batch-per-gpu 128 --steps 200 --warmup 20
