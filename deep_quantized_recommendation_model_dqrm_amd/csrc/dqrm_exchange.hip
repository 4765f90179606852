// dqrm_exchange.hip — the N > 1 exchange step's quantize-pack (K5): the rank's coalesced
// gradient (slot workspace) -> its dense wire payload, with the table scales averaged over
// the ranks' all-gathered per-slot max|grad|.
//
// Reference: sgd_quantized_gradients_parallel_comm.py quantize_emb_grad :861-869
//   s_r = clamp(max|g|, 1e-8) / (2^(b-1) - 1)            (quant_utils.py:141-194)
//   dist.all_reduce(s, SUM); s.mul_(1/N)                  (:863-866; Gloo's one-element order)
//   q = clamp(round(1/s * g + 0), -2^(b-1), 2^(b-1) - 1)  (quant_utils.py:75-101, :322-346)
//
// Built for latency (the step is launch- and round-trip-bound, not HBM-bound: ~2.3 MB written
// per launch at TB): grid (T x SPLIT slots, CY chunks) of 256-thread workgroups, every wave
// derives the slot's payload offset and the table scale itself from lane-held loads (no LDS,
// no barrier), and each lane group keeps QU entries' loads in flight. Two dependent round
// trips per workgroup: the slot's uniform bases (scalar) with the counts and maxima, then the
// entries' rows and values.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dqrm_device.h"
#include "dqrm_internal.h"

namespace {

constexpr int SPLIT = DQRM_TABLE_SPLIT;
constexpr int QP_TPB = 256;
constexpr int QP_QU = 4;  // entries per lane group in flight

template <int LPR>
__global__ void __launch_bounds__(QP_TPB) k_qpack(dqrm_internal::QuantPackArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = QP_TPB / LPR;         // lane groups (entries per pass)
    constexpr int E = G * QP_QU;            // entries per workgroup round
    const int k = blockIdx.x, t = k / SPLIT, s = k % SPLIT;
    const int tid = threadIdx.x, lane = tid % WAVE;
    const int N = a.N, bits = a.bits;
    const bool quant = bits >= 2 && bits <= 16;
    // round trip 1: the slot counts (lanes 0..7), rank r's slot maxima (lane r: 8 loads), and
    // the uniform bases (scalar loads)
    const int c_l = lane < SPLIT ? a.ws_ucount[t * SPLIT + lane] : 0;
    float am_l = 0.0f;
    if (quant && lane < N) {
        const float* p = a.absmax_all + (int64_t)lane * a.am_pitch + t * SPLIT;
        float x[SPLIT];
#pragma unroll
        for (int q = 0; q < SPLIT; ++q) x[q] = p[q];
#pragma unroll
        for (int q = 0; q < SPLIT; ++q) am_l = fmaxf(am_l, x[q]);
    }
    const int64_t ws0 = a.ws_cap_base[k], ws1 = a.ws_cap_base[k + 1];
    const int64_t cb0 = a.cap_base[t], cb1 = a.cap_base[t + 1];
    const PayloadLayout pl = payload_layout(a.T, a.cap_total, D, bits);
    const int scap = (int)(ws1 - ws0);  // the slot's workspace capacity
    const int sub = tid % LPR, grp = tid / LPR;
    const int u0 = (int)blockIdx.y * E + grp;
    const int ustride = (int)gridDim.y * E;
    // the first round of entries, issued before the counts arrive (indices clamped into the
    // slot's capacity; entries past the count are dropped below)
    float4 v[QP_QU];
    int32_t row[QP_QU];
    const float4* vals4 = reinterpret_cast<const float4*>(a.ws_vals);
#pragma unroll
    for (int h = 0; h < QP_QU; ++h) {
        int u = u0 + h * G;
        u = u < scap ? u : (scap > 0 ? scap - 1 : 0);
        const int64_t e = ws0 + u;
        v[h] = scap > 0 ? vals4[e * LPR + sub] : make_float4(0.f, 0.f, 0.f, 0.f);
        row[h] = scap > 0 ? a.ws_rows[e] : 0;
    }
    // the table's slot counts in slot order, clamped against its payload capacity (overflow
    // truncates the table), uniform in every wave
    const int cap = (int)(cb1 - cb0);
    int run = 0, pre = 0, my = 0;
#pragma unroll
    for (int q = 0; q < SPLIT; ++q) {
        int c = __builtin_amdgcn_readlane(c_l, q);
        c = c < cap - run ? c : cap - run;
        c = c < 0 ? 0 : c;
        if (q == s) { pre = run; my = c; }
        if (s == 0 && blockIdx.y == 0 && tid == q)  // the table's header counts
            reinterpret_cast<int32_t*>(a.payload)[t * SPLIT + q] = c;
        run += c;
    }
    // ranks' scales, summed in Gloo's one-element all_reduce order (descending rank), * 1/N
    float sv = 1.0f;
    if (quant) {
        const float s_l = sym_scale(am_l, bits);
        float acc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s_l), N - 1));
        for (int r = N - 2; r >= 0; --r)
            acc = acc + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s_l), r));
        sv = acc * (float)(1.0 / (double)N);
        if (s == 0 && blockIdx.y == 0 && tid == 0) a.s_avg[t] = sv;
    }
    const float rr = 1.0f / sv;
    const float qlo = -(float)(1 << (bits - 1)), qhi = (float)((1 << (bits - 1)) - 1);
    int32_t* prow = reinterpret_cast<int32_t*>(a.payload + pl.rows_off) + cb0 + pre;
    unsigned char* pval = a.payload + pl.vals_off + (cb0 + pre) * (int64_t)D * pl.elem;
    auto emit = [&](int u, float4 x, int32_t r) {
        if (sub == 0) prow[u] = r;
        if (!quant) {
            reinterpret_cast<float4*>(pval + (int64_t)u * D * 4)[sub] = x;
            return;
        }
        const float q0 = fake_quant(x.x, rr, qlo, qhi), q1 = fake_quant(x.y, rr, qlo, qhi);
        const float q2 = fake_quant(x.z, rr, qlo, qhi), q3 = fake_quant(x.w, rr, qlo, qhi);
        if (pl.elem == 1) {
            const uint32_t pk = ((uint32_t)(uint8_t)(int8_t)(int)q0) | ((uint32_t)(uint8_t)(int8_t)(int)q1 << 8) |
                                ((uint32_t)(uint8_t)(int8_t)(int)q2 << 16) | ((uint32_t)(uint8_t)(int8_t)(int)q3 << 24);
            reinterpret_cast<uint32_t*>(pval + (int64_t)u * D)[sub] = pk;
        } else {
            uint2 pk;
            pk.x = ((uint32_t)(uint16_t)(int16_t)(int)q0) | ((uint32_t)(uint16_t)(int16_t)(int)q1 << 16);
            pk.y = ((uint32_t)(uint16_t)(int16_t)(int)q2) | ((uint32_t)(uint16_t)(int16_t)(int)q3 << 16);
            reinterpret_cast<uint2*>(pval + (int64_t)u * D * 2)[sub] = pk;
        }
    };
#pragma unroll
    for (int h = 0; h < QP_QU; ++h)
        if (u0 + h * G < my) emit(u0 + h * G, v[h], row[h]);
    // a slot beyond the grid's first round (crowded slot): the rest, grid-strided
    for (int ub = u0 + ustride; ub < my; ub += ustride) {
#pragma unroll
        for (int h = 0; h < QP_QU; ++h) {
            const int u = ub + h * G;
            if (u < my) {
                v[h] = vals4[(ws0 + u) * LPR + sub];
                row[h] = a.ws_rows[ws0 + u];
            }
        }
#pragma unroll
        for (int h = 0; h < QP_QU; ++h)
            if (ub + h * G < my) emit(ub + h * G, v[h], row[h]);
    }
}

}  // namespace

namespace dqrm_internal {

hipError_t launch_quant_pack(const QuantPackArgs& a, hipStream_t stream) {
    // chunks per slot: the payload capacity spread evenly over the slots (a Criteo batch's
    // rows land roughly evenly in a table's row ranges), at least 1, at most 16
    const int64_t slots = (int64_t)a.T * SPLIT;
    auto chunks = [&](int lpr) {
        const int64_t e = (int64_t)(QP_TPB / lpr) * QP_QU;
        int64_t cy = (a.cap_total + slots * e - 1) / (slots * e);
        return (unsigned)(cy < 1 ? 1 : (cy > 16 ? 16 : cy));
    };
    const dim3 grid((unsigned)slots, 1);
    switch (a.D) {
#define QP_CASE(Dd)                                                                               \
    case Dd: {                                                                                    \
        constexpr int LPR = Dd / 4;                                                               \
        hipLaunchKernelGGL(k_qpack<LPR>, dim3(grid.x, chunks(LPR)), dim3(QP_TPB), 0, stream, a); \
    } break;
        QP_CASE(4) QP_CASE(8) QP_CASE(16) QP_CASE(32) QP_CASE(64) QP_CASE(128) QP_CASE(256)
#undef QP_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dqrm_internal
