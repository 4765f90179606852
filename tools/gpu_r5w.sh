# Round-5: table -> workgroup-group (XCD) placement by expected finish (DQRM_TABLE_GROUPS=critical)
# vs identity: parity under the permutation, then same-box A/B on the TB and Kaggle lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5w}
DQRM_TABLE_GROUPS=critical timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_next or fused_coalesce_apply or alternating" -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
N1="--steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for round in 1 2; do
for v in "tb||$N1" "tbcrit|DQRM_TABLE_GROUPS=critical|$N1" "kg||$N1 --config kaggle" "kgcrit|DQRM_TABLE_GROUPS=critical|$N1 --config kaggle"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_suite.log 2>&1 || { tail -n 40 gpurun_out/${T}_suite.log; exit 1; }
tail -n 1 gpurun_out/${T}_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${T}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${T}_smoke.log
