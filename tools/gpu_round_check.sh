# all GPU tests, then the bench lines (TB fused / unfused, Kaggle) and a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/s4_gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/s4_gpu_tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/s4_bench_tb.log 2>&1 || { tail -n 20 gpurun_out/s4_bench_tb.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --unfused-local > gpurun_out/s4_bench_tb_unfused.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config kaggle --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/s4_bench_kaggle.log 2>&1 || exit 1
for f in gpurun_out/s4_bench_tb.log gpurun_out/s4_bench_tb_unfused.log gpurun_out/s4_bench_kaggle.log; do tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['ms_per_step'], d['kernels_ms'])"; done
bash tools/prof_trace.sh s4_trace terabyte && python tools/prof_summary.py 2>/dev/null; grep -h "k_" gpurun_out/prof_s4_trace/tb_kernel_stats.csv | cut -d, -f1-5 | head -12
