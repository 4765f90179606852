# rocprof kernel traces of the TB / Kaggle / config-3 lines (no tests), the config-3 SGD
# phase clocks, and the drop-in host profiles.  usage: bash tools/gpu_r3_prof.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
bash tools/gpu_prof3.sh $T 0 || exit 1
cd $R
timeout -k 10 120 python tools/diag_sgd.py 128 > gpurun_out/${T}_diag_sgd.log 2>&1 || { tail -n 20 gpurun_out/${T}_diag_sgd.log; exit 1; }
head -n 8 gpurun_out/${T}_diag_sgd.log
for k in coll-dp list-sgd; do
  timeout -k 10 300 python tools/prof_dropin.py $k 40 > gpurun_out/${T}_prof_dropin_$k.log 2>&1 || { tail -n 20 gpurun_out/${T}_prof_dropin_$k.log; exit 1; }
  head -n 1 gpurun_out/${T}_prof_dropin_$k.log
done
