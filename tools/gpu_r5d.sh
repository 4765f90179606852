# Round-5: GPU tests (incl. the range-owned apply on every apply fixture), then the N>1 (RCCL
# forced) lines with the library-issued exchange: flat+finalize vs range-owned apply.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
A="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "tb2048flat|DQRM_APPLY=flat|" "tb2048ranges|DQRM_APPLY=ranges|" "tb256ranges|DQRM_APPLY=ranges|--batch-per-gpu 256" \
         "tb128ranges|DQRM_APPLY=ranges|--batch-per-gpu 128" "kaggleflat|DQRM_APPLY=flat|--config kaggle" \
         "kaggleranges|DQRM_APPLY=ranges|--config kaggle"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $A $args > gpurun_out/${T}_$lab.log 2>&1 || { tail -n 20 gpurun_out/${T}_$lab.log; exit 1; }
  tail -n 1 gpurun_out/${T}_$lab.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_$lab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'], d.get('launch_share'))"
done
for B in 2048 256; do
  timeout -k 10 300 python -u tools/prof_exchange.py terabyte_ref $B 200 > gpurun_out/${T}_host_$B.log 2>&1 || { tail -n 20 gpurun_out/${T}_host_$B.log; exit 1; }
  tail -n 1 gpurun_out/${T}_host_$B.log
done
