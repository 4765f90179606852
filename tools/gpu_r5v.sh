# Round-5: the step-boundary parity tests (SGD and one-launch forms) and the stall tests on the final kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5v}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_sgd_next or fused_next" tests/test_gpu_stall.py -v --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/${T}_tests.log | cut -c1-150; tail -n 1 gpurun_out/${T}_tests.log
