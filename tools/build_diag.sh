#!/bin/bash
# Diagnostic build of libdqrm with per-phase wall-clock stamps (-DDQRM_DIAG_CLOCK), read by
# tools/diag_clock.py / diag_coalesce.py / diag_sgd.py. Output: tools/diag_build/libdqrm_clock.so
# (git-ignored, not the product). Every translation unit of the package (_build.SOURCES).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/tools/diag_build
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DDQRM_DIAG_CLOCK $* -I $R/include"
SRCS=$(cd $R && python3 -c "from deep_quantized_recommendation_model_dqrm_amd._build import SOURCES; print(' '.join(SOURCES))")
OBJS=""
for s in $SRCS; do
  b=$(basename $s .hip)
  /opt/rocm/bin/hipcc $F -c $s -o $O/$b.o 2>/dev/null &
  OBJS="$OBJS $O/$b.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o $O/libdqrm_clock.so
echo built $O/libdqrm_clock.so
