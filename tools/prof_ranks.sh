set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6g -o r --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_apply_ranks.py terabyte merge 2048 ${NS:-8} > $GRAFT_REPO_ROOT/gpurun_out/r6g_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r6g_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kmedian.py gpurun_out/prof_r6g > gpurun_out/r6g_kmedian.txt 2>&1; head -30 gpurun_out/r6g_kmedian.txt
