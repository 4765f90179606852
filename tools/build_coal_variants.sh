#!/bin/bash
# Variant libraries of the Criteo-form coalesce (block size / prefetch depth), product and
# phase-clock builds, linked with the product's other objects: tools/diag_build/libdqrm_<v>.so
# and libdqrm_<v>_clock.so. usage: bash tools/build_coal_variants.sh "1024:6:4096 512:8:0"
# (block size : prefetched float4 per thread : largest row span sorted by counting)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/tools/diag_build; C=$R/deep_quantized_recommendation_model_dqrm_amd/csrc
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I $R/include"
for v in $1; do
  IFS=: read tpb pfr csp ch <<< "$v"; n=t${tpb}p${pfr}c${csp}h${ch}
  ( /opt/rocm/bin/hipcc $F -DDQRM_COAL_TPB=$tpb -DDQRM_COAL_PFR=$pfr -DDQRM_COAL_CSPAN=$csp -DDQRM_COAL_CH=$ch -c $C/dqrm_coalesce.hip -o $O/c_$n.o 2>/dev/null &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/dqrm_kernels.o $O/c_$n.o $C/dqrm_dense.o $C/dqrm_input.o -o $O/libdqrm_$n.so ) &
  ( /opt/rocm/bin/hipcc $F -DDQRM_DIAG_CLOCK -DDQRM_COAL_TPB=$tpb -DDQRM_COAL_PFR=$pfr -DDQRM_COAL_CSPAN=$csp -DDQRM_COAL_CH=$ch -c $C/dqrm_coalesce.hip -o $O/cc_$n.o 2>/dev/null &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/dqrm_kernels.o $O/cc_$n.o $C/dqrm_dense.o $C/dqrm_input.o -o $O/libdqrm_${n}_clock.so ) &
done
wait
ls $O/*.so
