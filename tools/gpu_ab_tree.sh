# Same-box A/B of this tree against another built checkout (e.g. the previous round's, exported
# with `git archive <rev> deep_quantized_recommendation_model_dqrm_amd include bench.py oracle`
# into tools/<dir> and built there): the bench line alternately from each tree, <n> times per
# argument set; prints us/step and the per-kernel breakdown of each run.
# usage: bash tools/gpu_ab_tree.sh <other tree dir> <n> "<bench args>" ["<bench args>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/$1; N=$2; shift 2
cd $R && mkdir -p gpurun_out
line() {  # <label> <dir> <args>
  (cd $2 && timeout -k 10 300 python bench.py $3 2>/dev/null | tail -n 1) | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$1', d['us_per_step'], d.get('kernels_ms'))"
}
for args in "$@"; do
  echo "== $args"
  for i in $(seq $N); do
    line other $O "$args" || exit 1
    line this $R "$args" || exit 1
  done
done
