# GPU round check: all GPU tests, smoke, the default bench line, a rocprofv3 kernel trace.
# usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-check}
K=${2:-}
cd $R && mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
fi
tail -n 2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -n 20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_bench.log
if [ -n "${TRACE:-}" ]; then
  bash tools/prof_trace.sh ${TAG} ${TRACE} || { tail -n 20 gpurun_out/prof_${TAG}.log; exit 1; }
  tail -n 1 gpurun_out/prof_${TAG}.log
fi
