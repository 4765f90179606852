# Round-5: 2-rank gloo rehearsal of the N>1 bench path on one GPU (1 GB TB-shaped tables: two
# replicas of the 198 GB slab do not fit one GPU), weak and strong scaling forms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5u}
A="--config terabyte_1g --steps 20 --warmup 5 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --dist-backend gloo"
for v in "weak|$A" "strong|$A --global-batch 2048"; do
  lab=${v%%|*}; args=${v#*|}
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
      bench.py --gpus 2 $args > gpurun_out/${T}_gloo2_$lab.log 2>&1 || { tail -n 30 gpurun_out/${T}_gloo2_$lab.log; exit 1; }
  grep "^{" gpurun_out/${T}_gloo2_$lab.log | tail -n 1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['n_gpus'], d['scaling'], d['config']['global_batch'], d['us_per_step'], d['replicas_bit_identical'], d['collectives'])"
done
