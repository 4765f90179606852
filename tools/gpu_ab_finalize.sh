# A/B of the |W| hierarchy finalize: in-launch (default) vs separate launch (DQRM_FINALIZE=launch),
# TB + Kaggle dp lines and the config-3 line, then a kernel trace of the TB default.
# usage: bash tools/gpu_ab_finalize.sh <tag> [tests=0]
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
if [ "${2:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_gpu_tests.log; exit 1; }
  tail -n 1 gpurun_out/${T}_gpu_tests.log
fi
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for fin in inline launch; do
  export DQRM_FINALIZE=$fin
  timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_${fin}_tb.log 2>&1 || { tail -n 20 gpurun_out/${T}_${fin}_tb.log; exit 1; }
  timeout -k 10 300 python bench.py --config kaggle $Q > gpurun_out/${T}_${fin}_kaggle.log 2>&1 || { tail -n 20 gpurun_out/${T}_${fin}_kaggle.log; exit 1; }
  timeout -k 10 300 python bench.py --config kaggle --mode sgd --batch-per-gpu 128 --graph --steps 400 --warmup 40 $Q > gpurun_out/${T}_${fin}_c3.log 2>&1 || { tail -n 20 gpurun_out/${T}_${fin}_c3.log; exit 1; }
  for f in tb kaggle c3; do tail -n 1 gpurun_out/${T}_${fin}_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$fin $f', d['value'], d['us_per_step'], d['kernels_ms'])"; done
done
unset DQRM_FINALIZE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_tb -o tb --output-format csv -- python3 $R/bench.py $Q --steps 50 --warmup 10 > $R/gpurun_out/prof_${T}_tb.log 2>&1 || { tail -n 20 $R/gpurun_out/prof_${T}_tb.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_kaggle -o kg --output-format csv -- python3 $R/bench.py --config kaggle $Q --steps 50 --warmup 10 > $R/gpurun_out/prof_${T}_kaggle.log 2>&1 || exit 1
cd $R && for f in $(find gpurun_out/prof_${T}_tb gpurun_out/prof_${T}_kaggle -name "*kernel_stats.csv"); do echo $f; cut -d, -f1-8 $f | head -12; done
