# Round-5: the next batch's forward inside the one-launch update (dqrm_emb_bwd_apply_fwd_local):
# its parity tests first, then the whole GPU suite, then same-box A/B lines (fused next forward
# vs --separate-forward) on TB and Kaggle, and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_next" tests/test_gpu_stall.py -x -v --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests_new.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests_new.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
N1="--steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for round in 1 2; do
for v in "tbnext||$N1" "tbsep||$N1 --separate-forward" "kgnext||$N1 --config kaggle" "kgsep||$N1 --config kaggle --separate-forward"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'], d['roofline']['frac'])"
done
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver.log 2>&1 || { tail -n 20 gpurun_out/${T}_driver.log; exit 1; }
tail -n 1 gpurun_out/${T}_driver.log | cut -c1-400
timeout -k 10 300 python -u tools/diag_coalesce.py terabyte 2048 applyfwd > gpurun_out/${T}_phase_tb_applyfwd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_tb_applyfwd.txt; exit 1; }
head -n 3 gpurun_out/${T}_phase_tb_applyfwd.txt; tail -n 30 gpurun_out/${T}_phase_tb_applyfwd.txt
