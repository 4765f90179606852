#!/bin/bash
# Diagnostic build of libdqrm with per-phase wall-clock stamps (-DDQRM_DIAG_CLOCK), read by
# tools/diag_clock.py. Output: tools/diag_build/libdqrm_clock.so (git-ignored, not the product).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/tools/diag_build
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DDQRM_DIAG_CLOCK $* -I $R/include"
for s in dqrm_kernels dqrm_coalesce dqrm_dense dqrm_input dqrm_sync; do
  /opt/rocm/bin/hipcc $F -c $R/deep_quantized_recommendation_model_dqrm_amd/csrc/$s.hip -o $O/$s.o 2>/dev/null
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/dqrm_kernels.o $O/dqrm_coalesce.o $O/dqrm_dense.o $O/dqrm_input.o $O/dqrm_sync.o -o $O/libdqrm_clock.so
echo built $O/libdqrm_clock.so
