#!/bin/bash
# A/B variant of libdqrm: dqrm_coalesce.hip rebuilt with extra flags (e.g. -DDQRM_COAL_WPF=4),
# linked with the in-tree objects of the other translation units (build the package first).
# Output tools/variants/libdqrm_<name>.so (git-ignored); bench.py / diag tools load it with
# DQRM_LIB_PATH=tools/variants/libdqrm_<name>.so.
# usage: bash tools/build_variant.sh <name> [hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
O=$R/tools/variants
C=$R/deep_quantized_recommendation_model_dqrm_amd/csrc
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" -I $R/include \
  -c $C/dqrm_coalesce.hip -o $O/coal_$N.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/dqrm_kernels.o $O/coal_$N.o $C/dqrm_dense.o \
  $C/dqrm_input.o $C/dqrm_sync.o -o $O/libdqrm_$N.so
echo built $O/libdqrm_$N.so
