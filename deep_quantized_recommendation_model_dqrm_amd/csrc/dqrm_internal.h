// dqrm_internal.h — launch interface between the translation units of libdqrm (not part of
// the C ABI; include/dqrm.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqrm.h"

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
    // group g < T serves table table_of_group[g] when group_perm (host-planned, A/B
    // DQRM_TABLE_GROUPS=critical: the tables expected to end last on the XCDs dealt first)
    int8_t table_of_group[32];
    int group_perm;
    // rendezvous polls before a workgroup gives up (DQRM_ERRF_STALL; its rows are then applied
    // by the table's last-arriving workgroup); the host sets it (DQRM_STALL_SPIN, default 2^20)
    uint32_t spin_limit;
    // the next batch's forward behind the update (dqrm_emb_bwd_apply_fwd_local; fwd_idx null:
    // none): Criteo-form indices [T][B] (the same B), out[t*fwd_ost_t + b*fwd_ost_b + d],
    // dqrm_emb_fwd's bits and flags (DQRM_FWD_REFRESH_SCALE / DQRM_FWD_FULL_PRECISION)
    const int64_t* fwd_idx;
    float* fwd_out;
    int64_t fwd_ost_t, fwd_ost_b;
    float* fwd_scale;           // [T] the forward scale: written (refresh) or read (held)
    int fwd_bits;
    uint32_t fwd_flags;
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

// K5 quantize-pack of the N > 1 exchange (dqrm_exchange.hip): the rank's slot workspace ->
// its wire payload, the table scales averaged over the all-gathered per-slot maxima
// (dqrm_grad_quant_pack_strided's arguments, validated by the caller).
struct QuantPackArgs {
    int T;
    int D;
    const int64_t* ws_cap_base;  // [T*S+1]
    const int32_t* ws_rows;
    const float* ws_vals;
    const int32_t* ws_ucount;
    const float* absmax_all;     // [N][pitch], rank r's per-slot max|grad| at r*pitch + t*S + s
    int64_t am_pitch;
    int N;
    int bits;                    // 2..16 quantized, 32 = FP32 values
    const int64_t* cap_base;     // [T+1] payload capacity prefix
    int64_t cap_total;
    float* s_avg;                // [T]
    unsigned char* payload;
};
hipError_t launch_quant_pack(const QuantPackArgs& a, hipStream_t stream);

// The pre-summed per-lookup gradient (dqrm_lookup.hip, dqrm_emb_bwd_lookup_grad_presum):
// one workgroup per table of at most kPresumMaxL lookups.
constexpr int kPresumMaxL = DQRM_PRESUM_MAX_LOOKUPS;
struct PresumArgs {
    const int64_t* meta;
    const float* scale;
    uint32_t* err;
    const int64_t* idx;
    const int64_t* off;
    const int64_t* idx_base;
    const float* dy;
    int64_t dst_t, dst_b;
    int64_t B;
    int64_t* rows;
    float* vals;
    int T;
    int D;
    int ste;
    int pool1;
};
hipError_t launch_lookup_grad_presum(const PresumArgs& a, hipStream_t stream);

// K6 with row ranges owned per workgroup (dqrm_apply.hip, DQRM_APPLY_RANGES): the gathered
// payloads decoded, summed over ranks, applied, and the |W| hierarchy finalized in-launch.
struct RangeApplyArgs {
    float* W;
    uint8_t* packed;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    float* tmax;
    uint32_t* sync;
    const float* pscale;
    const int64_t* meta;
    uint32_t* err;
    const int64_t* cap_base;
    int64_t cap_total;
    const unsigned char* payloads;  // rank r's payload at payloads + r * rank_pitch
    int64_t rank_pitch;
    int N;
    int T;
    int D;
    int bits;
    const float* s_avg;
    float nlr;
    int mode;
    int repack;
    int K;                          // chunks per row-range slot
};
hipError_t launch_apply_ranges(const RangeApplyArgs& a, hipStream_t stream);

// K6 with the ranks' rows merged on chip (dqrm_apply_merge.hip, DQRM_APPLY_MERGE): k_merge_pos
// (workgroups own block-aligned row ranges, K_t chunks per row-range slot of table t, locate every
// entry's row in the other ranks' runs in LDS) writes the positions; k_apply_pos updates, finalizes
// the |W| hierarchy in-launch and (fwd_idx) runs the next batch's forward behind per-table gates.
constexpr int kMergeMaxRanks = 16;
constexpr int kMergeMaxTables = 64;
struct MergeApplyArgs {
    float* W;
    uint8_t* packed;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    float* tmax;
    uint32_t* sync;
    const float* pscale;
    const int64_t* meta;
    uint32_t* err;
    const int64_t* cap_base;
    int64_t cap_total;
    const unsigned char* payloads;  // rank r's payload at payloads + r * rank_pitch
    int64_t rank_pitch;
    int N;
    int T;
    int D;
    int bits;
    const float* s_avg;
    float nlr;
    int mode;
    int repack;
    int32_t* pos;                     // N > 1: [N][cap_total][N] workspace (apply_workspace_bytes)
    int gx;                           // k_apply_pos: entry chunks per (table, rank)
    int kt[kMergeMaxTables];          // k_merge_pos: chunks per row-range slot of table t
    int kbase[kMergeMaxTables + 1];   //   first workgroup of table t (SPLIT * kt prefix)
    // the next batch's forward in the same launch (fwd_idx null: none): Criteo-form indices
    // [T][fwd_B], out[t*fwd_ost_t + b*fwd_ost_b + d], dqrm_emb_fwd's bits / flags
    // (DQRM_FWD_REFRESH_SCALE, DQRM_FWD_FULL_PRECISION); fwd_gx workgroups per table
    const int64_t* fwd_idx;
    int64_t fwd_B;
    float* fwd_out;
    int64_t fwd_ost_t, fwd_ost_b;
    float* fwd_scale;
    int fwd_bits;
    uint32_t fwd_flags;
    int fwd_gx;
    uint32_t spin_limit;              // gate polls before a forward workgroup flags DQRM_ERRF_STALL
    int diag;                         // DQRM_MERGE_DIAG (timing experiments only; 0 in normal use)
};
hipError_t launch_apply_merge(const MergeApplyArgs& a, hipStream_t stream);
int merge_forward_gx(int64_t B);
size_t apply_workspace_bytes(int num_ranks, int64_t cap_total);

}  // namespace dqrm_internal
