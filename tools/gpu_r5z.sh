# Round-5 final evidence on the final tree: full GPU suite + smoke, rocprofv3 summaries (kernel
# trace + FETCH_SIZE / WRITE_SIZE / read-request-size passes) of the TB, Kaggle and config-3
# lines and of the forced-collectives TB line, and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${T}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${T}_smoke.log
bash tools/gpu_profiles.sh ${T} || exit 1
EXTRA="--force-collectives" bash tools/prof_cfg.sh ${T}_tbforced terabyte || { tail -n 20 gpurun_out/prof_${T}_tbforced_trace.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_${T}_tbforced gpurun_out/${T}_tbforced > gpurun_out/${T}_tbforced_prof.txt && head -n 8 gpurun_out/${T}_tbforced_prof.txt
bash tools/gpu_driver_bench.sh ${T} || exit 1
# config 3 (B=128 fused SGD): eager and 32-step graphs; forced-collectives lines (configs 4/5 per-rank shares, Kaggle)
C3="--config kaggle --batch-per-gpu 128 --mode sgd --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
F="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "c3|$C3 --steps 384 --warmup 32" "c3g|$C3 --steps 384 --warmup 32 --graph --graph-steps 32" \
         "ftb2048|$F" "ftb256|$F --batch-per-gpu 256" "ftb128|$F --batch-per-gpu 128" "fkg|$F --config kaggle"; do
  lab=${v%%|*}; args=${v#*|}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'])"
done
