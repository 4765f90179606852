# config-3 check: the SGD parity tests (kernel k_sgd_small and the modules' fused SGD), the
# B=128 graph line and a kernel trace of the eager config-3 line.  usage: bash tools/gpu_r3_c3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --config kaggle --batch-per-gpu 128 --graph --graph-steps 32 --steps 384 --warmup 32 --mode sgd > gpurun_out/${T}_b128_sgd.log 2>&1 || { tail -n 20 gpurun_out/${T}_b128_sgd.log; exit 1; }
tail -n 1 gpurun_out/${T}_b128_sgd.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b128 sgd', d['value'], d['us_per_step'], d['kernels_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p3_${T}_c3 -o k --output-format csv -- python3 $R/bench.py --config kaggle --mode sgd --batch-per-gpu 128 --steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > $R/gpurun_out/p3_${T}_c3.log 2>&1 || { tail -n 20 $R/gpurun_out/p3_${T}_c3.log; exit 1; }
python3 $R/tools/kstats.py $(find $R/gpurun_out/p3_${T}_c3 -name "*kernel_stats.csv") | grep -E "sgd|emb_fwd"
