# Round-5 probe of the N > 1 exchange step at world size 1 (RCCL forced): host issue cost per
# call, kernel timeline (rocprofv3 kernel trace), and the apply-kernel A/B switches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r5b_tests.log 2>&1 || { tail -n 30 gpurun_out/r5b_tests.log; exit 1; }
tail -n 2 gpurun_out/r5b_tests.log
for B in 2048 256; do
  timeout -k 10 300 python -u tools/prof_exchange.py terabyte_ref $B 200 > gpurun_out/r5b_host_$B.log 2>&1 || { tail -n 20 gpurun_out/r5b_host_$B.log; exit 1; }
  tail -n 1 gpurun_out/r5b_host_$B.log
done
A="--steps 200 --warmup 20 --force-collectives --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for v in "flat|" "qlegacy|DQRM_QPACK=legacy" "slot|DQRM_APPLY=slot" "inline|DQRM_FINALIZE=inline"; do
  lab=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 300 python -u bench.py $A > gpurun_out/r5b_ab_$lab.log 2>&1 || { tail -n 20 gpurun_out/r5b_ab_$lab.log; exit 1; }
  tail -n 1 gpurun_out/r5b_ab_$lab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d['kernels_ms'], d.get('launch_share'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b_trace -o run -- \
    python3 bench.py --steps 60 --warmup 10 $A --batch-per-gpu 256 > gpurun_out/r5b_trace.log 2>&1 || { tail -n 20 gpurun_out/r5b_trace.log; exit 1; }
echo trace done
