# Round-5: k_sgd_small<LPR, true> with the next rows loaded up front and patched from LDS
# (DQRM_SG_FWD_PREFETCH) -- parity of the fused SGD forms, then same-box config-3 A/B against
# the variant built with -DDQRM_SG_FWD_PREFETCH=0 (tools/variants/libdqrm_nopf.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5pf}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "sgd or empty_update" -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 1 gpurun_out/${T}_tests.log
C3="--config kaggle --batch-per-gpu 128 --mode sgd --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 384 --warmup 32"
for round in 1 2; do
for v in "pf||$C3" "nopf|DQRM_LIB_PATH=tools/variants/libdqrm_nopf.so|$C3" "pfg||$C3 --graph --graph-steps 32" "nopfg|DQRM_LIB_PATH=tools/variants/libdqrm_nopf.so|$C3 --graph --graph-steps 32"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o c3 --output-format csv -- python3 $R/bench.py $C3 \
    > $R/gpurun_out/${T}_prof.log 2>&1 || { tail -n 20 $R/gpurun_out/${T}_prof.log; exit 1; }
cd $R && timeout -k 10 60 python3 tools/kmedian.py gpurun_out/${T}_prof "k_sgd_small" > gpurun_out/${T}_kmedian.txt 2>&1 && cat gpurun_out/${T}_kmedian.txt
