# Round-5: config 3 with the next batch's forward inside k_sgd_small (dqrm_emb_bwd_sgd_fwd):
# parity tests, same-box A/B (eager and 32-step graphs), rocprof of the fused kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_sgd_next or sgd_small or fused_next" -x -v --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests_new.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests_new.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests_new.log
C3="--config kaggle --batch-per-gpu 128 --mode sgd --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 384 --warmup 32"
for round in 1 2; do
for v in "next|$C3" "sep|$C3 --separate-forward" "nextg|$C3 --graph --graph-steps 32" "sepg|$C3 --separate-forward --graph --graph-steps 32"; do
  lab=${v%%|*}; args=${v#*|}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c3 -o tb --output-format csv -- python3 $R/bench.py $C3 > $R/gpurun_out/prof_${T}_c3.log 2>&1) || { tail -n 20 gpurun_out/prof_${T}_c3.log; exit 1; }
python3 tools/kmedian.py gpurun_out/prof_${T}_c3 sgd_small
