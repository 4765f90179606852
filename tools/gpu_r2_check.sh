# Round check of the product tree: all GPU tests + smoke, bench lines (TB default, TB unfused,
# Kaggle), then rocprofv3 trace + FETCH/WRITE PMC passes for TB and Kaggle (tools/prof_cfg.sh).
# usage: bash tools/gpu_r2_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${T}_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_tb.log 2>&1 || { tail -n 20 gpurun_out/${T}_bench_tb.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --unfused-local > gpurun_out/${T}_bench_tb_unfused.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config kaggle --cpu-baseline 0 --mlp-iters 0 > gpurun_out/${T}_bench_kaggle.log 2>&1 || exit 1
for f in tb tb_unfused kaggle; do tail -n 1 gpurun_out/${T}_bench_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['us_per_step'], d['kernels_ms'], d['roofline']['frac'])"; done
bash tools/prof_cfg.sh ${T}_tb terabyte && bash tools/prof_cfg.sh ${T}_kaggle kaggle && echo prof ok
