# The whole round-3 check in one call: every -m gpu test, smoke(), then the evidence of
# tools/gpu_r3_final.sh, the drop-in lines and the TB line with weight_syncc every 200 steps.
# usage: bash tools/gpu_r3_all.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -n 30 gpurun_out/${T}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${T}_smoke.log
bash tools/gpu_r3_final.sh $T || exit 1
bash tools/gpu_dropin.sh $T || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --sync-every 200 --steps 400 --warmup 20 > gpurun_out/${T}_tb_sync.log 2>&1 || { tail -n 20 gpurun_out/${T}_tb_sync.log; exit 1; }
tail -n 1 gpurun_out/${T}_tb_sync.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tb sync', d['value'], d['us_per_step'], d['weight_syncc'])"
