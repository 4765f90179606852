# A/B of the hierarchy finalize for the fused N=1 apply: (inline, sc1) (launch, sc1) (launch, plain) (inline, plain: timing only)
# rocprof kernel trace per variant, TB and Kaggle.  usage: bash tools/gpu_ab_fin2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd /tmp && export TMPDIR=/tmp
Q="--cpu-baseline 0 --gather-batch 0 --mlp-iters 0 --steps 50 --warmup 10"
for v in inline:1 launch:1 launch:0 inline:0; do
  export DQRM_FINALIZE=${v%%:*} DQRM_WT=${v##*:}
  tag=${DQRM_FINALIZE}_wt${DQRM_WT}
  for cfg in terabyte kaggle; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab2_${T}_${tag}_${cfg} -o k --output-format csv -- python3 $R/bench.py --config $cfg $Q > $R/gpurun_out/ab2_${T}_${tag}_${cfg}.log 2>&1 || { tail -n 20 $R/gpurun_out/ab2_${T}_${tag}_${cfg}.log; exit 1; }
    tail -n 1 $R/gpurun_out/ab2_${T}_${tag}_${cfg}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag $cfg', d['us_per_step'], d['kernels_ms'])"
    python3 $R/tools/kstats.py $(find $R/gpurun_out/ab2_${T}_${tag}_${cfg} -name "*kernel_stats.csv") | grep -E "apply|finalize|coalesce|emb_fwd"
  done
done
