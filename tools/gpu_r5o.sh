# Round-5: fused next-batch forward v4 (final max published at the last arrival when nothing is finalized): parity tests, same-box A/B, phase clocks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5o}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_next" tests/test_gpu_stall.py -x -v --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests_new.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests_new.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests_new.log
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
timeout -k 10 300 python -u tools/diag_coalesce.py terabyte 2048 applyfwd > gpurun_out/${T}_phase_tb_applyfwd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_tb_applyfwd.txt; exit 1; }
head -n 3 gpurun_out/${T}_phase_tb_applyfwd.txt; tail -n 30 gpurun_out/${T}_phase_tb_applyfwd.txt
timeout -k 10 300 python -u tools/diag_coalesce.py kaggle 2048 applyfwd > gpurun_out/${T}_phase_kaggle_applyfwd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_kaggle_applyfwd.txt; exit 1; }
head -n 3 gpurun_out/${T}_phase_kaggle_applyfwd.txt; tail -n 30 gpurun_out/${T}_phase_kaggle_applyfwd.txt
