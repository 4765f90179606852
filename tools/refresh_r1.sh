# rocprofv3 trace + PMC passes (tools/prof_r1.sh), then the default bench lines (TB, Kaggle)
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/prof_r1.sh || { tail -n 20 $R/gpurun_out/prof_r1_*.log; exit 1; }
cd $R
timeout -k 10 400 python bench.py > gpurun_out/s3_bench_tb.log 2>&1 || { tail -n 20 gpurun_out/s3_bench_tb.log; exit 1; }
timeout -k 10 400 python bench.py --config kaggle > gpurun_out/s3_bench_kaggle.log 2>&1 || { tail -n 20 gpurun_out/s3_bench_kaggle.log; exit 1; }
tail -n 1 gpurun_out/s3_bench_tb.log
tail -n 1 gpurun_out/s3_bench_kaggle.log
