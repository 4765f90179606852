# Same-box A/B of several variants of the bench line, interleaved <n> rounds: each variant is
# "label|tree dir (relative to the repo, . = this tree)|env assignments" — e.g.
#   "r3|tools/r3tree|"  "early|.|DQRM_LIB_PATH=tools/variants/libdqrm_early.so"  "nosub|.|DQRM_SUBSLOTS=0"
# Prints us/step and the per-kernel breakdown of each run.
# usage: bash tools/gpu_ab_variants.sh <n> "<bench args>" "<variant>" ["<variant>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
N=$1; ARGS=$2; shift 2
cd $R && mkdir -p gpurun_out
echo "== $ARGS"
for i in $(seq $N); do
  for v in "$@"; do
    IFS='|' read -r label dir envs <<< "$v"
    envabs=""
    for e in $envs; do
      k=${e%%=*}; val=${e#*=}
      case $val in tools/*) val=$R/$val ;; esac
      envabs="$envabs $k=$val"
    done
    (cd $R/$dir && env $envabs timeout -k 10 300 python bench.py $ARGS 2>/dev/null | tail -n 1) | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$label', d['us_per_step'], d.get('kernels_ms'))" || exit 1
  done
done
