#!/bin/bash
# A/B variant of libdqrm: one translation unit (default dqrm_coalesce.hip; VARIANT_SRC=<file>
# for another) rebuilt with extra flags (e.g. -DDQRM_COAL_WPF=4), linked with the in-tree
# objects of the other translation units (build the package first).
# Output tools/variants/libdqrm_<name>.so (git-ignored); bench.py / diag tools load it with
# DQRM_LIB_PATH=tools/variants/libdqrm_<name>.so.
# usage: [VARIANT_SRC=dqrm_kernels.hip] bash tools/build_variant.sh <name> [hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
O=$R/tools/variants
C=$R/deep_quantized_recommendation_model_dqrm_amd/csrc
V=${VARIANT_SRC:-dqrm_coalesce.hip}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "$@" -I $R/include \
  -c $C/$V -o $O/var_$N.o
OBJS=""
for o in $C/*.o; do
  [ "$(basename $o .o)" = "$(basename $V .hip)" ] || OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $O/var_$N.o -o $O/libdqrm_$N.so
echo built $O/libdqrm_$N.so
