# k_merge_pos phase costs at N ranks: rocprofv3 kernel trace of tools/bench_apply_ranks.py with
# DQRM_MERGE_DIAG phases skipped (4: after the header, 8: after the run counts, 1: after the LDS
# copy; results wrong, timing only). usage: NS=8 bash tools/prof_merge_diag.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
for d in 0 4 8 1; do
  DQRM_MERGE_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_${T}_d$d -o r --output-format csv -- python3 $R/tools/bench_apply_ranks.py terabyte merge 2048 ${NS:-8} > $R/gpurun_out/${T}_d$d.log 2>&1 || { tail -20 $R/gpurun_out/${T}_d$d.log; exit 1; }
  echo "diag $d"; python3 $R/tools/kmedian.py $R/gpurun_out/prof_${T}_d$d k_merge_pos; python3 $R/tools/kmedian.py $R/gpurun_out/prof_${T}_d$d k_apply_pos
done
