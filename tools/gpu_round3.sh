# tests + kernel profiles + drop-in lines + TB with weight_syncc every 200 steps
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && bash tools/gpu_prof3.sh $T ${2:-1} && bash tools/gpu_dropin.sh $T && \
timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --sync-every 200 --steps 400 --warmup 20 > gpurun_out/${T}_tb_sync.log 2>&1 && \
tail -n 1 gpurun_out/${T}_tb_sync.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tb sync', d['value'], d['us_per_step'], d['weight_syncc'])"
