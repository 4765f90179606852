# Targeted check of the one-launch local step: its parity tests, then the TB / Kaggle bench
# lines one-launch vs two-launch.  usage: bash tools/gpu_fused_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "fused or simulated or criteo_form" > gpurun_out/${T}_fused_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_fused_tests.log; exit 1; }
tail -n 3 gpurun_out/${T}_fused_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "simulated" > gpurun_out/${T}_sim_tests.log 2>&1 || { tail -n 60 gpurun_out/${T}_sim_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_sim_tests.log
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 200 --warmup 20"
for cfg in terabyte kaggle; do
  for v in "" "--two-launch-local"; do
    timeout -k 10 300 python bench.py --config $cfg $Q $v > gpurun_out/${T}_${cfg}${v}.log 2>&1 || { tail -n 30 gpurun_out/${T}_${cfg}${v}.log; exit 1; }
    tail -n 1 gpurun_out/${T}_${cfg}${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $v', d['value'], d['us_per_step'], d['kernels_ms'], d['roofline']['frac'])"
  done
done
