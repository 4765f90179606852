# GPU parity (all -m gpu tests), bench lines for TB and Kaggle, kernel traces of both
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s6_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/s6_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/s6_gpu_tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/s6_bench_tb.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config kaggle --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/s6_bench_kaggle.log 2>&1 || exit 1
for f in gpurun_out/s6_bench_tb.log gpurun_out/s6_bench_kaggle.log; do tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['ms_per_step'], d['kernels_ms'])"; done
bash tools/prof_trace.sh s6_tb terabyte && bash tools/prof_trace.sh s6_kaggle kaggle || exit 1
for c in s6_tb s6_kaggle; do python - $c <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/tb_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("k_table_finalize", "k_apply_local", "k_table_bwd")):
        print(sys.argv[1], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
