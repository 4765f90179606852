# Round-5 closing check: the empty-update + next-forward test, the whole GPU suite, smoke, and the
# driver's default bench command on the same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5zz}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "empty_update" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${T}_empty.log 2>&1 || { tail -n 40 gpurun_out/${T}_empty.log; exit 1; }
tail -n 1 gpurun_out/${T}_empty.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_suite.log 2>&1 || { tail -n 40 gpurun_out/${T}_suite.log; exit 1; }
tail -n 1 gpurun_out/${T}_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${T}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -n 20 gpurun_out/${T}_bench.log; exit 1; }
tail -n 1 gpurun_out/${T}_bench.log
