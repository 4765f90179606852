# Round-5: phase clocks of the fused next-batch forward with its sub-phase stamps (diagnostic build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5m}
for cfg in terabyte kaggle; do
timeout -k 10 300 python -u tools/diag_coalesce.py $cfg 2048 applyfwd > gpurun_out/${T}_phase_${cfg}_applyfwd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_${cfg}_applyfwd.txt; exit 1; }
tail -n 30 gpurun_out/${T}_phase_${cfg}_applyfwd.txt
done
# forced-collectives lines after the dimension-major N>1 coalesce (per-rank shares of configs 4/5, Kaggle)
F="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "ftb2048|$F" "ftb256|$F --batch-per-gpu 256" "ftb128|$F --batch-per-gpu 128" "fkg|$F --config kaggle"; do
  lab=${v%%|*}; args=${v#*|}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}.log >> gpurun_out/${T}_forced_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
