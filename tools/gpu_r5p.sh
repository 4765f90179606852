# Round-5: the driver's bench command (3 runs) after moving the event brackets out of the timed
# loop, next to a 200-step line and the --separate-forward form.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5p}
for k in 1 2 3; do
  bash tools/gpu_driver_bench.sh ${T}_$k > /dev/null || exit 1
  tail -n 1 gpurun_out/${T}_${k}_driver_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('driver', d['us_per_step'], d['value'], d['roofline']['frac'], d['roofline']['timed_launches'])"
done
N1="--steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "tb200|$N1" "tb200sep|$N1 --separate-forward" "tb20sep|--steps 20 --warmup 5 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --separate-forward"; do
  lab=${v%%|*}; args=${v#*|}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
