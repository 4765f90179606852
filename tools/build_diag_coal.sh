#!/bin/bash
# Diagnostic rebuild of the Criteo-form coalesce only (-DDQRM_DIAG_CLOCK), linked with the
# other objects of the last full diagnostic build (tools/build_diag.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/tools/diag_build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DDQRM_DIAG_CLOCK $* -I $R/include"
/opt/rocm/bin/hipcc $F -c $R/deep_quantized_recommendation_model_dqrm_amd/csrc/dqrm_coalesce.hip -o $O/dqrm_coalesce.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/*.o -o $O/libdqrm_clock.so
echo built $O/libdqrm_clock.so
