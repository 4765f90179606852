# Round-5: the fused forward's next-batch indices issued before the update (variant library) vs after the arrival,
# same-box A/B on the TB and Kaggle step-boundary lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5s}
N1="--steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for round in 1 2; do
for v in "tb||$N1" "tbearly|DQRM_LIB_PATH=tools/variants/libdqrm_earlyidx.so|$N1" "kg||$N1 --config kaggle" "kgearly|DQRM_LIB_PATH=tools/variants/libdqrm_earlyidx.so|$N1 --config kaggle"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
done
