# config-3 SGD kernel check: its parity tests, phase clocks, the B=128 graph line; then the
# cycling-batch phase clocks of the one-launch step.  usage: bash tools/gpu_r3_sgd.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sgd or single_gpu" > gpurun_out/${T}_sgd_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_sgd_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_sgd_tests.log
timeout -k 10 120 python tools/diag_sgd.py 128 > gpurun_out/${T}_diag_sgd.log 2>&1 || { tail -n 20 gpurun_out/${T}_diag_sgd.log; exit 1; }
head -n 6 gpurun_out/${T}_diag_sgd.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --config kaggle --batch-per-gpu 128 --graph --steps 400 --warmup 16 --mode sgd > gpurun_out/${T}_b128_sgd.log 2>&1 || { tail -n 20 gpurun_out/${T}_b128_sgd.log; exit 1; }
tail -n 1 gpurun_out/${T}_b128_sgd.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b128 sgd', d['value'], d['us_per_step'], d['kernels_ms'])"
timeout -k 10 240 python tools/diag_coalesce.py terabyte 2048 apply > gpurun_out/${T}_diag_tb_apply.log 2>&1 || { tail -n 20 gpurun_out/${T}_diag_tb_apply.log; exit 1; }
head -n 2 gpurun_out/${T}_diag_tb_apply.log
timeout -k 10 240 python tools/diag_coalesce.py terabyte 2048 > gpurun_out/${T}_diag_tb.log 2>&1 || { tail -n 20 gpurun_out/${T}_diag_tb.log; exit 1; }
head -n 2 gpurun_out/${T}_diag_tb.log
