# Round-5: GPU tests (incl. the range-owned apply on every apply fixture), then the N>1 (RCCL
# forced) lines with the library-issued exchange: flat+finalize vs range-owned apply.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_stall.py tests/test_gpu_modules.py -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests0.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests0.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests0.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
A="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "tb2048flag|DQRM_APPLY=flat|" "tb2048noskip|DQRM_FIN_FLAGGED=0|" "tb2048ranges|DQRM_APPLY=ranges|" "tb256flag|DQRM_APPLY=flat|--batch-per-gpu 256" "tb256ranges|DQRM_APPLY=ranges|--batch-per-gpu 256" \
         "tb128flag|DQRM_APPLY=flat|--batch-per-gpu 128" "kaggleflag|DQRM_APPLY=flat|--config kaggle" \
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
EXTRA="--force-collectives --mlp-iters 0 --gather-batch 0" bash tools/prof_cfg.sh ${T}_tbforced terabyte || { tail -n 20 gpurun_out/prof_${T}_tbforced_trace.log; exit 1; }
cd $R && python3 tools/prof_summary.py gpurun_out/prof_${T}_tbforced gpurun_out/${T}_tbforced > gpurun_out/${T}_tbforced_prof.txt && head -n 12 gpurun_out/${T}_tbforced_prof.txt
timeout -k 10 300 python -u tools/diag_coalesce.py terabyte 2048 apply > gpurun_out/${T}_phase_tb_apply.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_tb_apply.txt; exit 1; }
head -n 4 gpurun_out/${T}_phase_tb_apply.txt
timeout -k 10 300 python -u tools/diag_sgd.py 128 > gpurun_out/${T}_phase_sgd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_sgd.txt; exit 1; }
head -n 4 gpurun_out/${T}_phase_sgd.txt
