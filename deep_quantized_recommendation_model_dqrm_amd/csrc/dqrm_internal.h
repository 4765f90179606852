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

// launches k_coalesce_p1 (dqrm_coalesce.hip); returns a DQRM_E_* code
int launch_coalesce_pool1(const CoalesceArgs& a, hipStream_t stream);

// STE backward g' = (g * s) / s (quant_utils.py:349-363) without the IEEE division
// sequence, bit-identical to it: y = RN(1/s) once per table; q0 = RN(x*y) lies within 2 ulp
// of x/s, one residual correction (fma: the product is exact) makes it faithful, and
// Markstein's step with the correctly rounded y then gives exactly RN(x/s). Valid while
// nothing under- or overflows: s in [2^-60, 2^60] (checked per table) and |x| in
// [2^-60, 2^60]; a zero keeps its sign through x*y; anything else (tiny, huge, non-finite
// values, s = 0) takes the IEEE division.
struct SteDiv {
    float s, y;
    bool ok;
    __device__ __forceinline__ explicit SteDiv(float s_) : s(s_) {
        const float as = fabsf(s_);
        ok = as >= 0x1p-60f && as <= 0x1p60f;
        y = ok ? 1.0f / s_ : 0.0f;
    }
    __device__ __forceinline__ float operator()(float g) const {
        const float x = g * s;
        const float ax = fabsf(x);
        if (!ok || !(ax <= 0x1p60f && (ax >= 0x1p-60f || ax == 0.0f))) return x / s;
        float q = x * y;
        float r = fmaf(-s, q, x);
        q = fmaf(r, y, q);
        r = fmaf(-s, q, x);
        q = fmaf(r, y, q);
        return ax == 0.0f ? x * y : q;
    }
    __device__ __forceinline__ float4 operator()(float4 g) const {
        return make_float4((*this)(g.x), (*this)(g.y), (*this)(g.z), (*this)(g.w));
    }
};

}  // namespace dqrm_internal
