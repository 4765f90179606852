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

// The single-rank update fused behind the coalesce (dqrm_emb_bwd_apply_local): quantize the
// coalesced rows with the table's scale, SGD into W and keep the |W| hierarchy exact
// (dqrm_apply_local's arithmetic), inside the same launch.
struct LocalApplyArgs {
    float* W;
    uint8_t* packed;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    float* tmax;
    const float* pscale;
    uint32_t* sync;             // [T * DQRM_SYNC_STRIDE]: arrival counters of the table's workgroups
    float* s_avg;               // [T] the table scale the update used
    int bits;
    float nlr;                  // -lr
    int repack;
    // sub-slots (host-planned, dqrm_coalesce.hip): spare group e serves table sub_table[e]
    // (-1: idle); bit t of sub_mask = table t's slots are halved between two workgroups
    uint32_t sub_mask;
    int8_t sub_table[32];
};
constexpr int kSubTables = 32;  // LocalApplyArgs::sub_table entries

// largest B the Criteo-form coalesce kernel takes (larger batches use the general kernel)
constexpr int64_t kCoalesceMaxB = 4096;
// largest table count the fused coalesce + update runs with: its (T+7)/8*64 workgroups of
// 1024 threads (one per CU: 156 KiB LDS) must all be resident at once, since a table's
// workgroups wait for each other's gradient maxima
constexpr int kCoalesceApplyMaxT = 32;

// Whether the fused form's grid of T tables can be resident at once on the current device
// from `stream`: workgroups per CU (occupancy query) x CUs >= the grid, and the stream's CU
// mask enables every CU. Device properties are queried once per device.
bool coalesce_apply_resident(int T, hipStream_t stream);

// Sub-slot plan of the fused form (la->sub_mask / sub_table) from the host row counts
// (nullable: no sub-slots). DQRM_SUBSLOTS=0 in the environment disables them (A/B).
void plan_sub_slots(const int64_t* num_rows_host, int T, LocalApplyArgs* la);

// launches k_coalesce_p1 (dqrm_coalesce.hip); la != nullptr: the fused update as well
// (hipErrorInvalidValue if !coalesce_apply_resident). Returns the HIP error of the launch.
hipError_t launch_coalesce_pool1(const CoalesceArgs& a, const LocalApplyArgs* la, hipStream_t stream);

}  // namespace dqrm_internal
