# finalize A/B: inline (k_apply_*<, true>) vs launch (k_apply_*<, false> + k_table_finalize); TB, Kaggle,
# and the config-3 sgd line (k_sgd_small), all under rocprofv3 kernel traces.  usage: bash tools/gpu_ab_fin3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd /tmp && export TMPDIR=/tmp
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 50 --warmup 10"
for fin in inline launch; do
  export DQRM_FINALIZE=$fin
  for cfg in terabyte kaggle; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab3_${T}_${fin}_${cfg} -o k --output-format csv -- python3 $R/bench.py --config $cfg $Q > $R/gpurun_out/ab3_${T}_${fin}_${cfg}.log 2>&1 || { tail -n 20 $R/gpurun_out/ab3_${T}_${fin}_${cfg}.log; exit 1; }
    echo "$fin $cfg $(grep -o '"us_per_step": [0-9.]*' $R/gpurun_out/ab3_${T}_${fin}_${cfg}.log)"
    python3 $R/tools/kstats.py $(find $R/gpurun_out/ab3_${T}_${fin}_${cfg} -name "*kernel_stats.csv") | grep -E "apply|finalize|coalesce|emb_fwd"
  done
done
unset DQRM_FINALIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab3_${T}_c3 -o k --output-format csv -- python3 $R/bench.py --config kaggle --mode sgd --batch-per-gpu 128 --steps 200 --warmup 20 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > $R/gpurun_out/ab3_${T}_c3.log 2>&1 || { tail -n 20 $R/gpurun_out/ab3_${T}_c3.log; exit 1; }
echo "c3 $(grep -o '"us_per_step": [0-9.]*' $R/gpurun_out/ab3_${T}_c3.log)"
python3 $R/tools/kstats.py $(find $R/gpurun_out/ab3_${T}_c3 -name "*kernel_stats.csv") | grep -E "sgd|emb_fwd|finalize|bwd"
