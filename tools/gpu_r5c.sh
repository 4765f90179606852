# Round-5: GPU tests + the library-issued exchange (dqrm_comm) lines and host profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_modules.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r5c_tests1.log 2>&1 || { tail -n 40 gpurun_out/r5c_tests1.log; exit 1; }
tail -n 2 gpurun_out/r5c_tests1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r5c_tests.log 2>&1 || { tail -n 40 gpurun_out/r5c_tests.log; exit 1; }
tail -n 2 gpurun_out/r5c_tests.log
A="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "tb2048|" "tb2048torch|DQRM_C_COMM=0" "tb256|--batch-per-gpu 256" "tb128|--batch-per-gpu 128" "kaggle|--config kaggle"; do
  lab=${v%%|*}; extra=${v#*|}
  envs=""; args="$extra"
  case "$extra" in DQRM_*) envs="$extra"; args="";; esac
  env $envs timeout -k 10 300 python -u bench.py $A $args > gpurun_out/r5c_$lab.log 2>&1 || { tail -n 20 gpurun_out/r5c_$lab.log; exit 1; }
  tail -n 1 gpurun_out/r5c_$lab.log >> gpurun_out/r5c_lines.jsonl
  tail -n 1 gpurun_out/r5c_$lab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'], d.get('launch_share'), d['collectives'].get('issued_by'))"
done
for B in 2048 256; do
  timeout -k 10 300 python -u tools/prof_exchange.py terabyte_ref $B 200 > gpurun_out/r5c_host_$B.log 2>&1 || { tail -n 20 gpurun_out/r5c_host_$B.log; exit 1; }
  tail -n 1 gpurun_out/r5c_host_$B.log
done
