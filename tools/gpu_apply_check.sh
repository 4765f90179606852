# GPU parity for both apply kernels + rank sweep of each (one gpurun call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_ranking.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_parity.log 2>&1 || { tail -n 40 gpurun_out/s3_parity.log; exit 1; }
tail -n 2 gpurun_out/s3_parity.log
timeout -k 10 300 python tools/bench_apply_ranks.py terabyte > gpurun_out/s3_ranks_tb.log 2>&1 && \
timeout -k 10 300 python tools/bench_apply_ranks.py kaggle > gpurun_out/s3_ranks_kaggle.log 2>&1 && \
grep -h apply gpurun_out/s3_ranks_tb.log gpurun_out/s3_ranks_kaggle.log
