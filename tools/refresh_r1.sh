# rocprofv3 trace + PMC passes for the TB and Kaggle configs, then the default bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_tb_* $R/gpurun_out/prof_kaggle_*
bash $R/tools/prof_cfg.sh tb terabyte || { tail -n 20 $R/gpurun_out/prof_tb_*.log; exit 1; }
bash $R/tools/prof_cfg.sh kaggle kaggle || { tail -n 20 $R/gpurun_out/prof_kaggle_*.log; exit 1; }
cd $R
timeout -k 10 400 python bench.py > gpurun_out/s5_bench_tb.log 2>&1 || { tail -n 20 gpurun_out/s5_bench_tb.log; exit 1; }
timeout -k 10 400 python bench.py --config kaggle > gpurun_out/s5_bench_kaggle.log 2>&1 || { tail -n 20 gpurun_out/s5_bench_kaggle.log; exit 1; }
tail -n 1 gpurun_out/s5_bench_tb.log
tail -n 1 gpurun_out/s5_bench_kaggle.log
