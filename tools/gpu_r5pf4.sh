# Round-5: the k_sgd_small next-row prefetch as a variant (tools/sgd_fwd_prefetch.patch built as
# tools/variants/libdqrm_pf4.so, single exit, no scratch): its parity, same-box config-3 A/B
# against the in-tree library, then the whole GPU suite + smoke on the in-tree library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5pf4}
DQRM_LIB_PATH=tools/variants/libdqrm_pf4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "sgd or empty_update" -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
C3="--config kaggle --batch-per-gpu 128 --mode sgd --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 384 --warmup 32"
for round in 1 2; do
for v in "pf4|DQRM_LIB_PATH=tools/variants/libdqrm_pf4.so|$C3" "main||$C3" "pf4g|DQRM_LIB_PATH=tools/variants/libdqrm_pf4.so|$C3 --graph --graph-steps 32" "maing||$C3 --graph --graph-steps 32"; do
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
