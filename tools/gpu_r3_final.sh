# Round-3 evidence in one call: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of
# the TB and Kaggle bench lines (tools/prof_cfg.sh), the driver's exact bench command with
# its wall time, and the B=128 graph-replayed config-2 / config-3 lines.
# usage: bash tools/gpu_r3_final.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
bash tools/prof_cfg.sh ${T}_tb terabyte || { tail -n 20 gpurun_out/prof_${T}_tb_trace.log; exit 1; }
bash tools/prof_cfg.sh ${T}_kaggle kaggle || { tail -n 20 gpurun_out/prof_${T}_kaggle_trace.log; exit 1; }
cd $R
python3 tools/prof_summary.py gpurun_out/prof_${T}_tb gpurun_out/${T}_tb > gpurun_out/${T}_tb_prof.txt && head -n 8 gpurun_out/${T}_tb_prof.txt
python3 tools/prof_summary.py gpurun_out/prof_${T}_kaggle gpurun_out/${T}_kaggle > gpurun_out/${T}_kaggle_prof.txt && head -n 8 gpurun_out/${T}_kaggle_prof.txt
bash tools/gpu_driver_bench.sh $T || exit 1
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --config kaggle --batch-per-gpu 128 --graph --graph-steps 32 --steps 384 --warmup 32"
for m in fwd sgd dp; do
  timeout -k 10 300 python bench.py $Q --mode $m > gpurun_out/${T}_b128_$m.log 2>&1 || { tail -n 20 gpurun_out/${T}_b128_$m.log; exit 1; }
  tail -n 1 gpurun_out/${T}_b128_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('b128 $m', d['value'], d['us_per_step'], d['kernels_ms'])"
done
