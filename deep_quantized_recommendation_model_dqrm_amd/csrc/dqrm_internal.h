// dqrm_internal.h — launch interface between the translation units of libdqrm (not part of
// the C ABI; include/dqrm.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dqrm_internal {

// The coalesce backward of a Criteo-form batch (DQRM_BATCH_POOLING_ONE: table t's lookups
// are idx[t*B, (t+1)*B), bag b = lookup b), written into the caller's coalesced-gradient
// workspace (include/dqrm.h, dqrm_emb_bwd_coalesce).
struct CoalesceArgs {
    const int64_t* meta;        // [4][T] row_base, num_rows, blk_base, sblk_base
    int T;
    int D;
    int64_t B;                  // lookups (= bags) per table
    const int64_t* idx;         // [T][B]
    const float* dy;            // dy[t*dst_t + b*dst_b + d]
    int64_t dst_t, dst_b;
    const float* scale;         // [T] forward scale (STE)
    int ste;
    uint32_t* err;
    const int64_t* ws_cap_base; // [T*S+1]
    int32_t* ws_rows;
    float* ws_vals;
    int32_t* ws_ucount;
    float* ws_absmax;
};

// largest B the Criteo-form coalesce kernel takes (larger batches use the general kernel)
constexpr int64_t kCoalesceMaxB = 4096;

// launches k_coalesce_p1 (dqrm_coalesce.hip); returns the HIP error of the launch
hipError_t launch_coalesce_pool1(const CoalesceArgs& a, hipStream_t stream);

}  // namespace dqrm_internal
