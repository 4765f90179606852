# One GPU call: the -m gpu tests (optional), smoke(), and a list of bench.py lines, each under
# its own time limit; every JSON line lands in gpurun_out/<tag>_lines.jsonl and a one-line
# summary is printed. Stops at the first failure.
# usage: bash tools/gpu_suite.sh <tag> [tests|notests] ["<bench args>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
MODE=$1; shift
cd $R && mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_lines.jsonl
: > $OUT
if [ "$MODE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -n 15 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -n 20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_smoke.log
fi
i=0
for args in "$@"; do
  i=$((i + 1))
  timeout -k 10 600 python -u bench.py $args > gpurun_out/${TAG}_b$i.log 2>&1 || { echo "FAILED: $args"; tail -n 25 gpurun_out/${TAG}_b$i.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_b$i.log >> $OUT
  tail -n 1 gpurun_out/${TAG}_b$i.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d.get('roofline') or {}
print('$i', '[$args]', d.get('value'), 'us/step', d.get('us_per_step'), 'frac', r.get('frac'), 'kms', d.get('kernels_ms'),
      'ref', (d.get('torch_gpu_reference') or {}).get('us_per_step'), 'launches', d.get('launches_per_step'))"
done
