#!/bin/bash
# A/B libraries for the Criteo-form coalesce: "old" = dqrm_coalesce.hip at a git revision,
# "new" = the working tree; product and phase-clock builds, linked with the product's other
# objects into tools/diag_build/libdqrm_{old,new}[_clock].so.  usage: bash tools/build_ab.sh [rev]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/deep_quantized_recommendation_model_dqrm_amd/csrc; O=$R/tools/diag_build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I $R/include"
mkdir -p $O
git -C $R show ${1:-HEAD}:deep_quantized_recommendation_model_dqrm_amd/csrc/dqrm_coalesce.hip > $C/_coal_old.hip
one() {  # <src> <tag> <extra flags>
  /opt/rocm/bin/hipcc $F $3 -c $1 -o $O/c_$2.o 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/dqrm_kernels.o $O/c_$2.o $C/dqrm_dense.o $C/dqrm_input.o -o $O/libdqrm_$2.so
}
one $C/_coal_old.hip old "" & one $C/_coal_old.hip old_clock -DDQRM_DIAG_CLOCK &
one $C/dqrm_coalesce.hip new "" & one $C/dqrm_coalesce.hip new_clock -DDQRM_DIAG_CLOCK &
wait
rm -f $C/_coal_old.hip
ls $O/libdqrm_*.so
