# One GPU call, any sequence of steps, each under its own time limit; stops at the first
# failure (no retries). Replaces the per-call one-off wrappers of earlier rounds.
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   tests[=<pytest -k expr>]        the -m gpu tests (all, or the -k selection)
#   smoke                           __graft_entry__.smoke()
#   bench=<label>=<bench.py args>   one bench line -> gpurun_out/<tag>_lines.jsonl
#   torchrun=<label>=<n>=<args>     bench.py under torch.distributed.run with n ranks
#   profiles                        rocprofv3 trace + traffic passes: TB, Kaggle, config 3 (gpu_profiles.sh)
#   prof=<label>=<config>=<args>    the same passes for one bench line (prof_cfg.sh + prof_summary.py)
#   driver                          the driver's exact round-end bench command, wall-timed
#   py=<label>=<script args>        python3 <script args> (a tools/ measurement script)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${T}_lines.jsonl
summ() {
  python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d.get('roofline') or {}
print('$1', d.get('value'), 'us/step', d.get('us_per_step'), 'frac', r.get('frac'), 'kms', d.get('kernels_ms'))"
}
for step in "$@"; do
  kind=${step%%=*}; rest=${step#*=}
  [ "$rest" = "$step" ] && rest=""
  case $kind in
    tests)
      K=(); [ -n "$rest" ] && K=(-k "$rest")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v "${K[@]}" --timeout 300 --timeout-method thread \
        > gpurun_out/${T}_tests.log 2>&1
      rc=$?; grep -E "passed|failed|error" gpurun_out/${T}_tests.log | tail -n 3
      [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_tests.log | head -n 20; tail -n 40 gpurun_out/${T}_tests.log; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
        || { tail -n 20 gpurun_out/${T}_smoke.log; exit 1; }
      tail -n 1 gpurun_out/${T}_smoke.log ;;
    bench)
      lab=${rest%%=*}; args=${rest#*=}
      timeout -k 10 600 python -u bench.py $args > gpurun_out/${T}_${lab}.log 2>&1 \
        || { echo "FAILED: $args"; tail -n 25 gpurun_out/${T}_${lab}.log; exit 1; }
      tail -n 1 gpurun_out/${T}_${lab}.log >> $OUT
      tail -n 1 gpurun_out/${T}_${lab}.log | summ $lab ;;
    torchrun)
      lab=${rest%%=*}; r2=${rest#*=}; n=${r2%%=*}; args=${r2#*=}
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus $n $args > gpurun_out/${T}_${lab}.log 2>&1 \
        || { echo "FAILED: $args"; tail -n 30 gpurun_out/${T}_${lab}.log; exit 1; }
      grep "^{" gpurun_out/${T}_${lab}.log | tail -n 1 >> $OUT
      grep "^{" gpurun_out/${T}_${lab}.log | tail -n 1 | summ $lab ;;
    profiles)
      bash tools/gpu_profiles.sh ${T} || exit 1 ;;
    prof)
      lab=${rest%%=*}; r2=${rest#*=}; cfg=${r2%%=*}; args=${r2#*=}
      EXTRA="$args" bash tools/prof_cfg.sh ${T}_${lab} $cfg || { tail -n 20 gpurun_out/prof_${T}_${lab}_trace.log; exit 1; }
      cd $R && python3 tools/prof_summary.py gpurun_out/prof_${T}_${lab} gpurun_out/${T}_${lab} \
        > gpurun_out/${T}_${lab}_prof.txt && head -n 8 gpurun_out/${T}_${lab}_prof.txt ;;
    driver)
      bash tools/gpu_driver_bench.sh ${T} || exit 1 ;;
    py)
      lab=${rest%%=*}; args=${rest#*=}
      timeout -k 10 600 python3 -u $args > gpurun_out/${T}_${lab}.log 2>&1 \
        || { echo "FAILED: $args"; tail -n 25 gpurun_out/${T}_${lab}.log; exit 1; }
      tail -n 12 gpurun_out/${T}_${lab}.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
