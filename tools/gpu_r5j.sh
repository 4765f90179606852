# Round-5: full GPU tests; same-box A/B of the dimension-major stage for dimension-split workgroups (DQRM_COAL_DSDM)
# on the N=1 headline and the forced N>1 path; phase clocks of the N>1 coalesce and the one-launch step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5j}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
N1="--steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
F="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for round in 1 2; do
for v in "n1dsdm||$N1" "n1dsrm|DQRM_LIB_PATH=tools/variants/libdqrm_dsrm.so|$N1" \
         "fdsdm||$F" "fdsrm|DQRM_LIB_PATH=tools/variants/libdqrm_dsrm.so|$F"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
done
timeout -k 10 300 python -u tools/diag_coalesce.py terabyte 2048 apply > gpurun_out/${T}_phase_tb_apply.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_tb_apply.txt; exit 1; }
head -n 30 gpurun_out/${T}_phase_tb_apply.txt
timeout -k 10 300 python -u tools/diag_coalesce.py terabyte 2048 > gpurun_out/${T}_phase_tb_coal.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_tb_coal.txt; exit 1; }
head -n 12 gpurun_out/${T}_phase_tb_coal.txt
