// dqrm_kernels.hip — CDNA4 (gfx950) kernels and the C ABI of libdqrm.
//
// Hot path: DQRM's data-parallel QAT step for embedding tables
// (reference YangZhou08/Deep_Quantized_Recommendation_Model_DQRM @ 2024-10-24):
//   fwd   QuantEmbeddingBagTwo.forward      quantization_supp/quant_modules_not_quantize_grad.py:317-398
//   bwd   SymmetricQuantFunction.backward   quantization_supp/quant_utils.py:349-363
//   sgd   torch.optim.SGD (sparse)          dlrm_s_pytorch_single_gpu.py:1736-1750,1943-1950
//   dp    quantize_emb_grad / grad_update_parallel_comm / weight_update_parallel_comm
//                                           sgd_quantized_gradients_parallel_comm.py:257-317,601-628,850-890
//
// Everything here is integer/byte/gather work: HBM- or latency-bound, no MFMA.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see build.py). fp-contract must
// stay off: the reference's `1/s*x + 0`, `(g*s)/s`, `W + (-lr*v)` are separately rounded;
// the one fused multiply-add the reference does perform (torch CPU's sparse SGD axpy) is
// written as an explicit fmaf.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "../../include/dqrm.h"
#include "dqrm_internal.h"
#include "dqrm_device.h"

namespace {

// Diagnostic build only (-DDQRM_DIAG_CLOCK, tools/diag_clock.py): thread 0 of every slot
// workgroup stamps the 100 MHz wall clock at phase boundaries.
#ifdef DQRM_DIAG_CLOCK
__device__ unsigned long long g_diag_clk[8192 * 16];
#define DIAG_T(k) \
    do { if (threadIdx.x == 0) g_diag_clk[blockIdx.x * 16 + (k)] = wall_clock64(); } while (0)
#else
#define DIAG_T(k) do { } while (0)
#endif
// diagnostic stamp after every outstanding memory operation of the thread has landed
#ifdef DQRM_DIAG_CLOCK
#define DIAG_W(k) do { __builtin_amdgcn_s_waitcnt(0); DIAG_T(k); } while (0)
#else
#define DIAG_W(k) do { } while (0)
#endif
// diagnostic shader-cycle stamp (s_memtime): with the wall stamps, the in-kernel clock
#ifdef DQRM_DIAG_CLOCK
#define DIAG_C(k) \
    do { if (threadIdx.x == 0) g_diag_clk[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define DIAG_C(k) do { } while (0)
#endif

// ------------------------------------------------------------------------------------
// error reporting (host)
// ------------------------------------------------------------------------------------
thread_local char g_last_error[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return set_error(DQRM_E_HIP, "HIP error: %s (%d)", hipGetErrorString(e_), (int)e_);                                           \
    } while (0)

#define LAUNCH_CHECK() HIP_TRY(hipGetLastError())

constexpr int MAX_TABLES = 256;
constexpr int DQRM_MAX_RANKS = 64;    // dqrm_apply_sparse_update: num_ranks <= 64


// ------------------------------------------------------------------------------------
// K0: synthetic init, U(-sqrt(1/n), sqrt(1/n)) per table (q_m_n_q_g.py:273-275 distribution)
// ------------------------------------------------------------------------------------
DQRM_INLINE uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_init_uniform(float* __restrict__ W, const int64_t* __restrict__ meta, int T,
                               int D, int64_t total_rows, uint64_t seed) {
    Meta m = make_meta(meta, T);
    const int64_t n4 = total_rows * (D / 4);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
         q += (int64_t)gridDim.x * blockDim.x) {
        int64_t row = q / (D / 4);
        int t = find_table(m.row_base, T, row);
        float bound = sqrtf(1.0f / (float)m.num_rows[t]);
        uint64_t h0 = splitmix64(seed ^ ((uint64_t)q * 2ull));
        uint64_t h1 = splitmix64(seed ^ ((uint64_t)q * 2ull + 1ull));
        float4 v;
        v.x = ((float)(uint32_t)(h0 >> 40) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
        v.y = ((float)(uint32_t)((h0 >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
        v.z = ((float)(uint32_t)(h1 >> 40) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
        v.w = ((float)(uint32_t)((h1 >> 16) & 0xFFFFFF) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
        v.x *= bound; v.y *= bound; v.z *= bound; v.w *= bound;
        reinterpret_cast<float4*>(W)[q] = v;
    }
}

// ------------------------------------------------------------------------------------
// K1: absolute-max hierarchy  rowmax -> blkmax -> sblkmax -> tmax
// (exact replacement of the full-table min/max, quant_utils.py:177-178)
// ------------------------------------------------------------------------------------
template <int LPR>  // lanes per row = D/4
__global__ void k_rowmax_all(const float* __restrict__ W, float* __restrict__ rowmax,
                             int64_t total_rows) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ngrp = (int64_t)gridDim.x * blockDim.x / LPR;
    const int lane = threadIdx.x % LPR;
    for (int64_t row = gid / LPR; row < total_rows; row += ngrp) {
        float4 v = reinterpret_cast<const float4*>(W + row * (LPR * 4))[lane];
        float m = group_max<LPR>(abs_max4(v));
        if (lane == 0) rowmax[row] = m;
    }
}

// one wave per output: out[ob_t + j] = max(in[ib_t + j*256 .. min(+256, nin_t)])
// level 1: in = rowmax (ib = row_base, nin = num_rows), out = blkmax (ob = blk_base)
// level 2: in = blkmax (ib = blk_base, nin = nblk),     out = sblkmax (ob = sblk_base)
__global__ void k_level_max(const float* __restrict__ in, float* __restrict__ out,
                            const int64_t* __restrict__ meta, int T, int level,
                            int64_t total_out) {
    Meta m = make_meta(meta, T);
    const int lane = threadIdx.x % WAVE;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const int64_t nw = (int64_t)gridDim.x * blockDim.x / WAVE;
    const int64_t* ob = level == 1 ? m.blk_base : m.sblk_base;
    for (int64_t o = wid; o < total_out; o += nw) {
        int t = find_table(ob, T, o);
        int64_t j = o - ob[t];
        int64_t ib = level == 1 ? m.row_base[t] : m.blk_base[t];
        int64_t nin = level == 1 ? m.num_rows[t] : ceil_div(m.num_rows[t], BLK);
        int64_t s0 = j * 256, s1 = s0 + 256 < nin ? s0 + 256 : nin;
        float v = 0.0f;
        for (int64_t k = s0 + lane; k < s1; k += WAVE) v = fmaxf(v, in[ib + k]);
        v = wave_max(v);
        if (lane == 0) out[o] = v;
    }
}

// one workgroup per table: tmax[t] = max(sblkmax of t)
__global__ void k_table_max(const float* __restrict__ sblkmax, float* __restrict__ tmax,
                            const int64_t* __restrict__ meta, int T) {
    Meta m = make_meta(meta, T);
    __shared__ float red[16];
    const int t = blockIdx.x;
    const int64_t ns = ceil_div(ceil_div(m.num_rows[t], BLK), SBLK_BLOCKS);
    float v = 0.0f;
    for (int64_t k = threadIdx.x; k < ns; k += blockDim.x) v = fmaxf(v, sblkmax[m.sblk_base[t] + k]);
    v = wave_max(v);
    if ((threadIdx.x % WAVE) == 0) red[threadIdx.x / WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = 0.0f;
        for (int w = 0; w < (int)(blockDim.x / WAVE); ++w) r = fmaxf(r, red[w]);
        tmax[t] = r;
    }
}

// ------------------------------------------------------------------------------------
// K2: periodic scale refresh + conditional INT4 repack
// ------------------------------------------------------------------------------------
__global__ void k_refresh_scale(const float* __restrict__ tmax, float* __restrict__ scale,
                                float* __restrict__ pscale, uint32_t* __restrict__ tflags,
                                int T, int bits, int has_packed) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    float s = sym_scale(tmax[t], bits);
    scale[t] = s;
    uint32_t need = 0;
    if (has_packed) {
        float ps = pscale[t];
        need = !(ps == s);  // NaN pscale (never packed) -> repack
        pscale[t] = s;
    }
    tflags[t] = need;
}


template <int LPR>
DQRM_INLINE void pack_row_int4(const float4 w, uint8_t* __restrict__ packed, int64_t grow,
                               int lane, float r) {
    pack4_row(w, packed + grow * (LPR * 2), lane, r);
}

template <int LPR>
__global__ void k_repack_flagged(const float* __restrict__ W, uint8_t* __restrict__ packed,
                                 const float* __restrict__ scale,
                                 const uint32_t* __restrict__ tflags,
                                 const int64_t* __restrict__ meta, int T, int64_t total_rows) {
    Meta m = make_meta(meta, T);
    const int lane = threadIdx.x % LPR;
    const int64_t ngrp = (int64_t)gridDim.x * blockDim.x / LPR;
    const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    for (int t = 0; t < T; ++t) {
        if (!tflags[t]) continue;  // scale unchanged since the last pack: rows still exact
        const float r = 1.0f / scale[t];
        const int64_t r0 = m.row_base[t], r1 = r0 + m.num_rows[t];
        for (int64_t row = r0 + g0; row < r1; row += ngrp) {
            float4 w = reinterpret_cast<const float4*>(W + row * (LPR * 4))[lane];
            pack_row_int4<LPR>(w, packed, row, lane, r);
        }
    }
    (void)total_rows;
}

// ------------------------------------------------------------------------------------
// K3: fused multi-table fake-quant EmbeddingBag forward
// One group of LPR = D/4 lanes per bag, float4 per lane; UNR bags in flight per group.
// Per-table scale / reciprocal / bounds staged in LDS once per workgroup.
// ------------------------------------------------------------------------------------
struct FwdArgs {
    const float* W;
    const uint8_t* packed;
    const float* tmax;
    float* scale;
    const int64_t* meta;
    uint32_t* err;
    const int64_t* idx;
    const int64_t* off;
    const int64_t* idx_base;
    float* out;
    int64_t B;
    int64_t ost_t, ost_b;
    int T;
    int bits;
    uint32_t flags;
    int pool1;  // DQRM_BATCH_POOLING_ONE: bag b of every table is lookup b (offsets unread)
    uint32_t* sync;     // k_finalize_fwd: the tables' sync words (gate, arrivals)
    uint32_t spin;      //   gate polls before a forward workgroup flags a stall
};

// k_finalize_fwd's per-table sync words (apart from the merge apply's 8/9 and the one-launch
// step's 3-5 / 32+): the gate (1 = the table's |W| maxima are final) and its forward arrivals
constexpr int FINFWD_GATE_WORD = 10;
constexpr int FINFWD_CNT_WORD = 11;

// wave-uniform bounded wait for a table's gate (a gate that never opens is flagged, not a hang)
DQRM_INLINE void wait_gate(const uint32_t* gate, uint32_t spin, uint32_t* err) {
    uint32_t n = 0;
    while (ld_wt(gate) == 0u) {
        if (++n > spin) {
            flag_error(err, DQRM_ERRF_STALL);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Table t's bags, workgroup bx of gx (the body of k_emb_fwd; WT: the table max was just
// written by this workgroup -- k_fwd_after_update -- and is read write-through). GATE
// (k_finalize_fwd): the table max is final only once the table's finalize workgroup opened its
// gate, so the scale is taken after the first pass's index and row loads are in flight (W
// itself is final at launch start), and every workgroup passes the gate once.
template <int LPR, int UNR, bool WT, bool GATE = false, int TPB = 256>
__device__ __forceinline__ void emb_fwd_table(const FwdArgs& a, int t, int64_t bx, int64_t gx) {
    const bool full_precision = (a.flags & DQRM_FWD_FULL_PRECISION) != 0;
    const bool refresh = (a.flags & DQRM_FWD_REFRESH_SCALE) != 0;
    const bool use_packed = (a.flags & DQRM_FWD_USE_PACKED) != 0 && !full_precision;
    float s = 1.0f, r = 1.0f;
    const bool gated = GATE && refresh && !full_precision;  // a frozen scale needs no final max
    bool waited = !gated;   // the scale is taken
    bool passed = false;    // GATE: this workgroup passed the gate
    uint32_t* gate = GATE ? a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FINFWD_GATE_WORD : nullptr;
    auto take_scale = [&]() {
        if (!full_precision) s = refresh ? sym_scale((WT || GATE) ? ld_wt(a.tmax + t) : a.tmax[t], a.bits) : a.scale[t];
        r = 1.0f / s;
        if (refresh && !full_precision && bx == 0 && threadIdx.x == 0) a.scale[t] = s;
    };
    if (!gated) take_scale();
    const int64_t rowbase = a.meta[t], nrows = a.meta[a.T + t];
    // Criteo form: table t's lookups are idx[t*B, (t+1)*B) -- no idx_base round trip in front of the index loads
    const int64_t ibase = a.pool1 ? (int64_t)t * a.B : a.idx_base[t];
    const int64_t L = a.pool1 ? a.B : a.idx_base[t + 1] - ibase;
    const int64_t B = a.B;
    const int64_t* __restrict__ off = a.off + (int64_t)t * B;
    const int64_t* __restrict__ idx = a.idx + ibase;
    float* __restrict__ out = a.out + (int64_t)t * a.ost_t;

    const float qlo = -(float)(1 << (a.bits - 1));
    const float qhi = (float)((1 << (a.bits - 1)) - 1);
    constexpr int G = TPB / LPR;  // bags per workgroup pass
    const int lane = threadIdx.x % LPR;
    const int grp = threadIdx.x / LPR;
    const int D = LPR * 4;

    // Every global load of a phase is issued unconditionally (addresses clamped into the
    // arrays, the values of invalid bags / lookups dropped afterwards), so the UNR bags' index
    // loads and then their row loads are in flight together: a per-bag branch around a load
    // made the compiler wait for each one before the next (one round trip per bag).
    const bool p1 = a.pool1 && L == B;
    for (int64_t b0 = bx * (G * UNR); b0 < B; b0 += gx * (G * UNR)) {
        int64_t beg[UNR], len[UNR], row[UNR];
        // phase 1: offsets
        int64_t s0v[UNR], s1v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            const int64_t b = b0 + k * G + grp;
            const int64_t bb = b < B ? b : 0;
            if (p1) {
                s0v[k] = bb;
                s1v[k] = bb + 1;
            } else {
                s0v[k] = off[bb];
                s1v[k] = off[bb + 1 < B ? bb + 1 : bb];
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            const int64_t b = b0 + k * G + grp;
            const bool valid = b < B;
            int64_t s0 = s0v[k];
            int64_t s1 = (p1 || b + 1 < B) ? s1v[k] : L;
            if (s0 < 0 || s1 > L || s1 < s0) {
                if (valid && lane == 0) flag_error(a.err, DQRM_ERRF_OFFSET);
                s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
                s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
            }
            beg[k] = s0;
            len[k] = valid ? s1 - s0 : -1;  // -1: no such bag
        }
        // phase 2: single-lookup indices
        int64_t rv[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) rv[k] = L > 0 ? idx[beg[k] < L ? beg[k] : L - 1] : -1;
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            row[k] = -1;
            if (len[k] == 1) {
                if (rv[k] < 0 || rv[k] >= nrows) {
                    if (lane == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                } else {
                    row[k] = rv[k];
                }
            }
        }
        // phase 3: row loads for single-lookup bags (row 0 of the table for the others, dropped)
        float4 acc[UNR];
        uint32_t pk[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            pk[k] = 0x8888u;  // q = 0
        }
        if (nrows > 0) {
            if (use_packed) {
#pragma unroll
                for (int k = 0; k < UNR; ++k)
                    pk[k] = reinterpret_cast<const uint16_t*>(a.packed + (rowbase + (row[k] >= 0 ? row[k] : 0)) * (D / 2))[lane];
            } else {
#pragma unroll
                for (int k = 0; k < UNR; ++k)
                    acc[k] = reinterpret_cast<const float4*>(a.W + (rowbase + (row[k] >= 0 ? row[k] : 0)) * D)[lane];
            }
#pragma unroll
            for (int k = 0; k < UNR; ++k)
                if (row[k] < 0) {
                    acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                    pk[k] = 0x8888u;
                }
        }
        if (!waited) {  // GATE: the first pass's loads are in flight; now the table's final max
            wait_gate(gate, a.spin, a.err);
            waited = passed = true;
            take_scale();
        }
        // phase 4: pooled sums for multi-lookup bags (bag order, FP32), quantize, store
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            if (len[k] < 0) continue;
            float4 y;
            if (len[k] == 1 && use_packed) {
                const uint32_t p = pk[k];
                y.x = (float)((int)(p & 15u) - 8) * s;
                y.y = (float)((int)((p >> 4) & 15u) - 8) * s;
                y.z = (float)((int)((p >> 8) & 15u) - 8) * s;
                y.w = (float)((int)((p >> 12) & 15u) - 8) * s;
            } else {
                float4 v = acc[k];
                if (len[k] > 1) {
                    v = make_float4(0.f, 0.f, 0.f, 0.f);
                    for (int64_t i = 0; i < len[k]; ++i) {
                        const int64_t rr = idx[beg[k] + i];
                        if (rr < 0 || rr >= nrows) {
                            if (lane == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                            continue;
                        }
                        const float4 w = reinterpret_cast<const float4*>(a.W + (rowbase + rr) * D)[lane];
                        v.x = v.x + w.x; v.y = v.y + w.y; v.z = v.z + w.z; v.w = v.w + w.w;
                    }
                }
                if (full_precision) {
                    y = v;
                } else {
                    y.x = fake_quant(v.x, r, qlo, qhi) * s;
                    y.y = fake_quant(v.y, r, qlo, qhi) * s;
                    y.z = fake_quant(v.z, r, qlo, qhi) * s;
                    y.w = fake_quant(v.w, r, qlo, qhi) * s;
                }
            }
            const int64_t b = b0 + k * G + grp;
            reinterpret_cast<float4*>(out + b * a.ost_b)[lane] = y;
        }
    }
    if constexpr (GATE) {
        // every forward workgroup of the table passes the gate once (also one without bags), so
        // when the last one arrives here none still polls: it re-arms the gate for the next launch
        if (!passed) wait_gate(gate, a.spin, a.err);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t* cnt = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FINFWD_CNT_WORD;
            if (atomicAdd(cnt, 1u) + 1u == (uint32_t)gx) {
                __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gate, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

template <int LPR, int UNR>
__global__ void __launch_bounds__(256) k_emb_fwd(FwdArgs a) {
    // grid = (bag chunks, tables): the table index is blockIdx.y, so every per-table value
    // is wave-uniform (scalar registers) and no 64-bit division is needed per bag.
    emb_fwd_table<LPR, UNR, false>(a, blockIdx.y, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------
// K3p: INT4 packed forward, one bag per thread, three lane-parallel phases per 256 bags:
//   (1) offsets + single-lookup index for 256 consecutive bags (coalesced),
//   (2) 256 independent packed-row loads (D/2 bytes, lane per bag) staged in LDS,
//   (3) dequantize + store: LPR lanes x float4 per output row (full-line, coalesced).
// Bags that do not hold exactly one valid lookup take the exact FP32 fake-quant path in
// phase 3. The row loads no longer sit behind a per-group dependent chain, so the kernel
// runs at the output-write stream rate.
// ------------------------------------------------------------------------------------
template <int LPR, bool NT>
__global__ void __launch_bounds__(256) k_emb_fwd_packed(FwdArgs a) {
    constexpr int D = LPR * 4;
    constexpr int PB = D / 2;                 // packed bytes per row
    constexpr int PW = PB / 4 > 0 ? PB / 4 : 1;  // dwords per packed row (D >= 8)
    __shared__ __attribute__((aligned(16))) uint32_t s_pk[256 * PW + 4];
    __shared__ int64_t s_beg[256];
    __shared__ int s_len[256];
    const int t = blockIdx.y;
    const float s = a.scale[t];               // frozen scale the rows were packed with
    const float r = 1.0f / s;
    const float qlo = -(float)(1 << (a.bits - 1)), qhi = (float)((1 << (a.bits - 1)) - 1);
    const int64_t rowbase = a.meta[t], nrows = a.meta[a.T + t];
    // Criteo form: table t's lookups are idx[t*B, (t+1)*B) -- no idx_base round trip in front of the index loads
    const int64_t ibase = a.pool1 ? (int64_t)t * a.B : a.idx_base[t];
    const int64_t L = a.pool1 ? a.B : a.idx_base[t + 1] - ibase;
    const int64_t B = a.B;
    const int64_t* __restrict__ off = a.off + (int64_t)t * B;
    const int64_t* __restrict__ idx = a.idx + ibase;
    float* __restrict__ out = a.out + (int64_t)t * a.ost_t;
    const int tid = threadIdx.x;

    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < B; b0 += (int64_t)gridDim.x * 256) {
        // phase 1: one bag per thread
        const int64_t b = b0 + tid;
        int64_t s0 = 0, s1 = 0;
        int len = -1;
        int64_t row = -1;
        if (b < B) {
            const bool p1 = a.pool1 && L == B;
            s0 = p1 ? b : off[b];
            s1 = p1 ? b + 1 : ((b + 1 < B) ? off[b + 1] : L);
            if (s0 < 0 || s1 > L || s1 < s0) {
                flag_error(a.err, DQRM_ERRF_OFFSET);
                s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
                s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
            }
            len = (int)(s1 - s0 > 0x7fffffff ? 0x7fffffff : s1 - s0);
            if (len == 1) {
                row = idx[s0];
                if (row < 0 || row >= nrows) {
                    flag_error(a.err, DQRM_ERRF_INDEX);
                    row = -1;
                    len = 0;  // an invalid lookup contributes nothing (zero row)
                }
            }
        }
        // phase 2: packed row -> LDS
        uint32_t pk[PW];
        if (len == 1) {
            const uint8_t* src = a.packed + (rowbase + row) * PB;
            if constexpr (PB >= 16) {
#pragma unroll
                for (int q = 0; q < PB / 16; ++q) {
                    const uint4 v = reinterpret_cast<const uint4*>(src)[q];
                    pk[4 * q] = v.x; pk[4 * q + 1] = v.y; pk[4 * q + 2] = v.z; pk[4 * q + 3] = v.w;
                }
            } else if constexpr (PB == 8) {
                const uint2 v = *reinterpret_cast<const uint2*>(src);
                pk[0] = v.x; pk[1] = v.y;
            } else {
                pk[0] = *reinterpret_cast<const uint32_t*>(src);
            }
        } else {
#pragma unroll
            for (int q = 0; q < PW; ++q) pk[q] = 0x88888888u;
        }
        __syncthreads();  // previous pass's phase 3 is done with the LDS
#pragma unroll
        for (int q = 0; q < PW; ++q) s_pk[tid * PW + q] = pk[q];
        s_len[tid] = len;
        s_beg[tid] = s0;
        __syncthreads();
        // phase 3: LPR lanes per bag, float4 each
        constexpr int G = 256 / LPR;
        const int lane = tid % LPR, grp = tid / LPR;
        for (int j = grp; j < 256; j += G) {
            const int64_t bb = b0 + j;
            const int ln = s_len[j];
            if (ln < 0) break;  // past the last bag (uniform per group: bags are in order)
            float4 y;
            if (ln == 1 || ln == 0) {
                const uint32_t w = reinterpret_cast<const uint16_t*>(s_pk + j * PW)[lane];
                y.x = (float)((int)(w & 15u) - 8) * s;
                y.y = (float)((int)((w >> 4) & 15u) - 8) * s;
                y.z = (float)((int)((w >> 8) & 15u) - 8) * s;
                y.w = (float)((int)((w >> 12) & 15u) - 8) * s;
            } else {  // multi-lookup bag: exact FP32 sum in bag order, then fake-quant
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                const int64_t sb = s_beg[j];
                for (int i = 0; i < ln; ++i) {
                    const int64_t rr = idx[sb + i];
                    if (rr < 0 || rr >= nrows) {
                        if (lane == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                        continue;
                    }
                    const float4 w = reinterpret_cast<const float4*>(a.W + (rowbase + rr) * D)[lane];
                    v.x = v.x + w.x; v.y = v.y + w.y; v.z = v.z + w.z; v.w = v.w + w.w;
                }
                y.x = fake_quant(v.x, r, qlo, qhi) * s;
                y.y = fake_quant(v.y, r, qlo, qhi) * s;
                y.z = fake_quant(v.z, r, qlo, qhi) * s;
                y.w = fake_quant(v.w, r, qlo, qhi) * s;
            }
            float4* dst = reinterpret_cast<float4*>(out + bb * a.ost_b) + lane;
            if (NT) {
                typedef float v4f __attribute__((ext_vector_type(4)));
                v4f yv = {y.x, y.y, y.z, y.w};
                __builtin_nontemporal_store(yv, reinterpret_cast<v4f*>(dst));
            } else {
                *dst = y;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Per-table workgroup machinery (backward / coalesce / apply).
// Each table is split into DQRM_TABLE_SPLIT row-range slots (block-aligned); one
// 512-thread workgroup per (table, slot) gathers the lookups (or payload entries) of its
// rows as keys (row << 32 | tag) in LDS, sorts them (stable radix), compacts the segment heads
// (= unique rows) and processes every segment in exact sequential order.
// ------------------------------------------------------------------------------------
constexpr int SPLIT = DQRM_TABLE_SPLIT;
constexpr int TWG = 512;                       // threads per (table, slot) workgroup
constexpr int SLOT_KEYS = DQRM_SLOT_KEYS;      // keys one slot sorts on chip (64 KiB)

constexpr int LONG_SEG = 8;   // longer segments are combined block-cooperatively
constexpr int LONG_SEGS_MAX = SLOT_KEYS / (LONG_SEG + 1) + 1;
constexpr int STAGE_FLOATS = 16384;                        // 64 KiB
constexpr int STAGE_PAD = 1024;                            // dim-major stage: +4 floats per dim row
constexpr int STAGE_F4 = STAGE_FLOATS / 4 / TWG;           // 8 float4 per thread per chunk
constexpr int CARRY_FLOATS = 2 * 256;                      // two rows of max D
constexpr int LPRE_INTS = (LONG_SEGS_MAX + 1 + 3) / 4 * 4;
// dynamic LDS of a slot workgroup: keys u64 | heads u16 | stage | carry | long prefix
constexpr int SLOT_LDS =
    SLOT_KEYS * 8 + SLOT_KEYS * 2 + (STAGE_FLOATS + STAGE_PAD) * 4 + CARRY_FLOATS * 4 + LPRE_INTS * 4;
static_assert(SLOT_LDS + 3072 <= 160 * 1024, "slot LDS budget (dynamic + static)");

struct SlotLds {
    uint64_t* keys;
    uint16_t* heads;
    float* stage;
    float* carry;
    int* lpre;
    DQRM_INLINE explicit SlotLds(unsigned char* lds)
        : keys(reinterpret_cast<uint64_t*>(lds)),
          heads(reinterpret_cast<uint16_t*>(lds + SLOT_KEYS * 8)),
          stage(reinterpret_cast<float*>(lds + SLOT_KEYS * 10)),
          carry(reinterpret_cast<float*>(lds + SLOT_KEYS * 10 + (STAGE_FLOATS + STAGE_PAD) * 4)),
          lpre(reinterpret_cast<int*>(lds + SLOT_KEYS * 10 + (STAGE_FLOATS + STAGE_PAD) * 4 + CARRY_FLOATS * 4)) {}
};

DQRM_INLINE uint32_t key_row(uint64_t k) { return (uint32_t)(k >> 32); }
DQRM_INLINE uint32_t key_lo(uint64_t k) { return (uint32_t)k; }
DQRM_INLINE uint64_t with_lo(uint64_t k, uint32_t lo) { return (k & 0xFFFFFFFF00000000ull) | lo; }

// rows [r0, r1) of slot s of a table with nrows rows (block-aligned split)
DQRM_INLINE void slot_rows(int64_t nrows, int s, int64_t& r0, int64_t& r1) {
    const int64_t nblk = ceil_div(nrows, BLK);
    const int64_t b0 = nblk * s / SPLIT, b1 = nblk * (s + 1) / SPLIT;
    r0 = b0 * BLK;
    r1 = b1 * BLK < nrows ? b1 * BLK : nrows;
}

// exclusive block-wide prefix of one int per thread; *total = the sum (s_wsum: TWG/WAVE+1)
DQRM_INLINE int block_excl_scan(int cnt, int* s_wsum, int* total) {
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    int v = cnt;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        int y = __shfl_up(v, o, WAVE);
        if (lane >= o) v += y;
    }
    if (lane == WAVE - 1) s_wsum[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int k = 0; k < TWG / WAVE; ++k) { int x = s_wsum[k]; s_wsum[k] = run; run += x; }
        s_wsum[TWG / WAVE] = run;
    }
    __syncthreads();
    *total = s_wsum[TWG / WAVE];
    return s_wsum[w] + v - cnt;
}

// Sorting a slot's keys. The keys arrive in ascending tag order (lookup position, or
// (rank, entry)), so what is needed is a STABLE sort by row: an LSD radix sort on
// (row - r0), 4-bit digits, wave-parallel. Wave w owns keys [w*64*KPL, (w+1)*64*KPL),
// held in registers (KPL per lane). Per pass: every wave counts its digits with four
// bit-sliced ballots per 64 keys, one wave scans the 16x8 (digit, wave) counts, and every
// lane places its key at base[digit] + (earlier lanes with that digit), the per-digit
// bases living in lanes 0..15 and read with one bpermute. 3 barriers per pass, no
// serial per-thread loops. Heads are then compacted with ballots as well.
DQRM_INLINE uint64_t lanemask_lt() { return (1ull << (threadIdx.x % WAVE)) - 1ull; }

// lanes whose digit equals v, from the four bit-slice ballots
DQRM_INLINE uint64_t digit_mask(uint32_t v, uint64_t b0, uint64_t b1, uint64_t b2, uint64_t b3) {
    return ((v & 1) ? b0 : ~b0) & ((v & 2) ? b1 : ~b1) & ((v & 4) ? b2 : ~b2) & ((v & 8) ? b3 : ~b3);
}

// sort the slot's n keys (rows in [r0, r0 + span)) stably by row, then compact segment
// heads: heads[u] = index of the first key of the u-th distinct row. Returns U.
// Wave w owns keys [w*64*kpl, (w+1)*64*kpl), kpl = ceil(n / TWG), 64 at a time.
DQRM_INLINE int sort_and_heads(const SlotLds& L, int n, uint32_t r0, uint32_t span, int* s_wsum,
                               bool presorted = false) {
    const int bits = span <= 1 ? 0 : 32 - __builtin_clz(span - 1);
    uint64_t* keys = L.keys;
    uint64_t* tmp = reinterpret_cast<uint64_t*>(L.heads);  // scratch over heads + stage until heads exist
    int* s_hist = reinterpret_cast<int*>(reinterpret_cast<unsigned char*>(keys) + SLOT_KEYS * 16);
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    const int kpl = (n + TWG - 1) / TWG;
    const int i0 = w * WAVE * kpl + lane;  // this lane's keys: i0 + k * WAVE, k < kpl
    const uint64_t lt = lanemask_lt();
    if (!presorted && bits > 0) {
        uint64_t* src = keys;
        uint64_t* dst = tmp;
        for (int sh = 0; sh < bits; sh += 4) {
            uint32_t cnt = 0;  // lane d < 16: this wave's keys with digit d
#pragma unroll 4
            for (int k = 0; k < kpl; ++k) {
                const int i = i0 + k * WAVE;
                const bool v = i < n;
                const uint32_t d = v ? ((key_row(src[i]) - r0) >> sh) & 15u : 0u;
                const uint64_t b0 = __ballot(d & 1), b1 = __ballot(d & 2), b2 = __ballot(d & 4), b3 = __ballot(d & 8);
                cnt += __popcll(digit_mask(lane, b0, b1, b2, b3) & __ballot(v));
            }
            if (lane < 16) s_hist[lane * 8 + w] = (int)cnt;
            __syncthreads();
            if (w == 0) {  // exclusive scan of the 128 (digit-major, wave-minor) counts
                const int v0 = s_hist[2 * lane], v1 = s_hist[2 * lane + 1];
                int v = v0 + v1;
#pragma unroll
                for (int o = 1; o < WAVE; o <<= 1) {
                    const int y = __shfl_up(v, o, WAVE);
                    if (lane >= o) v += y;
                }
                const int ex = v - v0 - v1;
                s_hist[2 * lane] = ex;
                s_hist[2 * lane + 1] = ex + v0;
            }
            __syncthreads();
            uint32_t base = lane < 16 ? (uint32_t)s_hist[lane * 8 + w] : 0u;
#pragma unroll 4
            for (int k = 0; k < kpl; ++k) {
                const int i = i0 + k * WAVE;
                const bool v = i < n;
                const uint64_t x = v ? src[i] : 0ull;
                const uint64_t vmask = __ballot(v);
                const uint32_t d = ((key_row(x) - r0) >> sh) & 15u;
                const uint64_t b0 = __ballot(d & 1), b1 = __ballot(d & 2), b2 = __ballot(d & 4), b3 = __ballot(d & 8);
                const uint64_t mine = digit_mask(d, b0, b1, b2, b3) & vmask;
                const uint32_t pos = (uint32_t)__shfl((int)base, (int)d, WAVE) + (uint32_t)__popcll(mine & lt);
                if (v) dst[pos] = x;
                base += (uint32_t)__popcll(digit_mask(lane, b0, b1, b2, b3) & vmask);
            }
            __syncthreads();
            uint64_t* t = src; src = dst; dst = t;
        }
        if (src != keys) {  // the sorted keys sit in tmp: bring them home (the heads reuse tmp)
            for (int i = threadIdx.x; i < n; i += TWG) keys[i] = src[i];
            __syncthreads();
        }
    }
    DIAG_T(6);
    // heads: first key of every distinct row, by ballots over the same ownership
    auto is_head = [&](int k) {
        const int i = i0 + k * WAVE;
        return i < n && (i == 0 || key_row(keys[i]) != key_row(keys[i - 1]));
    };
    int hc = 0;
#pragma unroll 4
    for (int k = 0; k < kpl; ++k) hc += __popcll(__ballot(is_head(k)));
    if (lane == 0) s_wsum[w] = hc;
    __syncthreads();
    int run = 0, U = 0;
    for (int k = 0; k < TWG / WAVE; ++k) { const int c = s_wsum[k]; run += k < w ? c : 0; U += c; }
#pragma unroll 4
    for (int k = 0; k < kpl; ++k) {
        const bool h = is_head(k);
        const uint64_t hm = __ballot(h);
        if (h) L.heads[run + __popcll(hm & lt)] = (uint16_t)(i0 + k * WAVE);
        run += __popcll(hm);
    }
    __syncthreads();
    return U;
}

DQRM_INLINE int seg_end(const uint16_t* heads, int U, int n, int u) {
    return u + 1 < U ? (int)heads[u + 1] : n;
}

// ------------------------------------------------------------------------------------
// Segment reduction in exact sequential order.
// A segment = the sorted keys of one row; its entries are combined strictly in key order
// (ascending lookup position, or ascending rank) to reproduce the reference's rounding:
//   OP_FMA  acc = fma(v, -lr, acc) per entry          (torch CPU sparse SGD axpy)
//   OP_SUM  acc = v0; acc = acc + v_k                  (coalesce / sparse all_reduce)
//   OP_AXPY acc = acc + (v * -lr), product rounded     (W.add_(-lr * grad), s_q_g_p_c.py:616)
// Short segments: one lane group (LPR lanes x float4), 4 entries in flight per chunk.
// Long segments (> LONG_SEG entries, tiny hot tables): a whole wave loads 4*WAVE/LPR
// entries per chunk (the next chunk prefetched) and combines them in order via shuffles.
// Masked entries re-load the head's own entry, so they never address out of bounds.
// ------------------------------------------------------------------------------------
constexpr int OP_FMA = 0;
constexpr int OP_SUM = 1;
constexpr int OP_AXPY = 2;

template <int OP>
DQRM_INLINE float4 combine(float4 acc, float4 v, bool& first, float nlr) {
    if (OP == OP_FMA) {
        acc.x = fmaf(v.x, nlr, acc.x); acc.y = fmaf(v.y, nlr, acc.y);
        acc.z = fmaf(v.z, nlr, acc.z); acc.w = fmaf(v.w, nlr, acc.w);
    } else if (OP == OP_AXPY) {
        acc.x = acc.x + v.x * nlr; acc.y = acc.y + v.y * nlr;
        acc.z = acc.z + v.z * nlr; acc.w = acc.w + v.w * nlr;
    } else if (first) {
        acc = v;
        first = false;
    } else {
        acc.x = acc.x + v.x; acc.y = acc.y + v.y; acc.z = acc.z + v.z; acc.w = acc.w + v.w;
    }
    return acc;
}

template <int LPR, int OP, class Src>
DQRM_INLINE float4 seg_reduce_group(const uint64_t* keys, int i, int len, float4 acc, const Src& src,
                                    float nlr, int sub) {
    const uint32_t head_lo = key_lo(keys[i]);
    bool first = true;
    for (int j = 0; j < len; j += 4) {
        float4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int jj = j + c;
            v[c] = src.load(jj < len ? key_lo(keys[i + jj]) : head_lo, sub);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (j + c < len) acc = combine<OP>(acc, v[c], first, nlr);
    }
    return acc;
}

// Long segments (> LONG_SEG entries: tiny hot tables, Zipf-hot rows) are combined by
// "dim-lane" groups of GD = min(D, 64) lanes, each lane owning NDL = D/GD dimensions, so the
// strictly ordered chain is one add (or fma) per entry per lane. Their entries are fed
// block-cooperatively (staged_long_segments below).
template <int LPR>
struct DimLane {
    static constexpr int D = LPR * 4;
    static constexpr int GD = D < WAVE ? D : WAVE;
    static constexpr int NDL = D / GD;
};

template <int OP>
DQRM_INLINE float combine1(float acc, float v, bool first, float nlr) {
    if (OP == OP_FMA) return fmaf(v, nlr, acc);
    if (OP == OP_AXPY) return acc + v * nlr;
    return first ? v : acc + v;
}

template <int LPR>
DQRM_INLINE float dl_absmax(const float (&v)[DimLane<LPR>::NDL]) {
    float m = 0.0f;
#pragma unroll
    for (int d = 0; d < DimLane<LPR>::NDL; ++d) m = fmaxf(m, fabsf(v[d]));
    return group_max<DimLane<LPR>::GD>(m);
}

// repack a dim-lane row: even lanes combine their nibble with the odd neighbour's.
// prow = the row's packed bytes, dim0 = first dim this group owns.
template <int LPR>
DQRM_INLINE void dl_pack_int4(const float (&v)[DimLane<LPR>::NDL], uint8_t* prow, int dim0, int lig, float rcp) {
    using DL = DimLane<LPR>;
#pragma unroll
    for (int d = 0; d < DL::NDL; ++d) {
        const int q = (int)fake_quant(v[d], rcp, -8.0f, 7.0f) + 8;
        const int qn = __shfl_xor(q, 1, WAVE);
        const int dim = dim0 + lig + DL::GD * d;
        if ((dim & 1) == 0) prow[dim / 2] = (uint8_t)(q | (qn << 4));
    }
}

// Short segments (<= LONG_SEG entries): one float4 lane group (LPRS lanes) per segment, SB
// segments of a group in flight together: heads, the first entry's row of all SB segments
// and their initial values are loaded before anything is combined (one HBM round trip per
// SB segments instead of per segment); further entries follow 4 at a time. finit(u, i, sub, st) loads the
// initial state, ffin(u, i, sub, st) stores the result; combination is strictly in key order.
struct SegState {
    float4 acc;   // running value (W row for SGD, sum otherwise)
    float4 w;     // apply: the W row being updated
    float blk;    // old max of the row's 256-row block
};

// After a wide-table row is updated its head key's low word holds the row's new max |W|
// (a non-negative float) with bit 31 set iff the row held its block's max and shrank;
// maintain_blocks reads only these (no rowmax loads; rowmax is store-only on the hot path).
DQRM_INLINE uint32_t row_record(float new_rm, float old_rm, float old_blk) {
    return __float_as_uint(new_rm) | ((old_rm == old_blk && new_rm < old_rm) ? 0x80000000u : 0u);
}

template <int LPRS, int OP, int SB, class Src, class FI, class FF>
DQRM_INLINE void short_segments(const uint64_t* keys, const uint16_t* heads, int U, int n, const Src& src,
                                float nlr, FI&& finit, FF&& ffin, int ubeg = 0, int uend = -1) {
    const int sub = threadIdx.x % LPRS, grp = threadIdx.x / LPRS;
    constexpr int NGRP = TWG / LPRS;
    if (uend < 0) uend = U;
    for (int u0 = ubeg + grp; u0 < uend; u0 += NGRP * SB) {
        int ii[SB], ll[SB];
#pragma unroll
        for (int b = 0; b < SB; ++b) {
            const int u = u0 + b * NGRP;
            int i = 0, len = 0;
            if (u < uend) {
                i = heads[u];
                len = seg_end(heads, U, n, u) - i;
                if (len > LONG_SEG) len = 0;  // long: block-cooperative path
            }
            ii[b] = i;
            ll[b] = len;
        }
        SegState st[SB];
        typename Src::Raw r[SB];
#pragma unroll
        for (int b = 0; b < SB; ++b) {  // initial values + the first entry of all SB segments
            if (ll[b]) {
                finit(u0 + b * NGRP, ii[b], sub, st[b]);
                r[b] = src.fetch(key_lo(keys[ii[b]]), sub);
            }
        }
        if (u0 == ubeg + grp) DIAG_T(11);  // first batch: loads issued
#pragma unroll
        for (int b = 0; b < SB; ++b) {
            if (!ll[b]) continue;
            bool first = true;
            st[b].acc = combine<OP>(st[b].acc, src.finish(r[b]), first, nlr);
            for (int j = 1; j < ll[b]; j += 4) {  // the rest (most segments of wide tables have one entry)
                typename Src::Raw q[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (j + c < ll[b]) q[c] = src.fetch(key_lo(keys[ii[b] + j + c]), sub);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (j + c < ll[b]) st[b].acc = combine<OP>(st[b].acc, src.finish(q[c]), first, nlr);
            }
        }
        if (u0 == ubeg + grp) DIAG_T(12);  // first batch combined (its loads have landed)
#pragma unroll
        for (int b = 0; b < SB; ++b)
            if (ll[b]) ffin(u0 + b * NGRP, ii[b], sub, st[b]);
        if (u0 == ubeg + grp) DIAG_T(13);  // first batch's stores issued
    }
    DIAG_T(14);
}

// ordered compaction of the long segments' indices u into s_long (ballots); returns their number
DQRM_INLINE int compact_long(const uint16_t* heads, int U, int n, uint16_t* s_long, int* s_wsum) {
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    const int kpl = (U + TWG - 1) / TWG;
    const int u0 = w * WAVE * kpl + lane;
    const uint64_t lt = lanemask_lt();
    auto is_long = [&](int u) { return u < U && seg_end(heads, U, n, u) - (int)heads[u] > LONG_SEG; };
    int c = 0;
    for (int k = 0; k < kpl; ++k) c += __popcll(__ballot(is_long(u0 + k * WAVE)));
    if (lane == 0) s_wsum[w] = c;
    __syncthreads();
    DIAG_T(15);  // every thread's short work done and its stores drained
    int run = 0, total = 0;
    for (int k = 0; k < TWG / WAVE; ++k) { const int x = s_wsum[k]; run += k < w ? x : 0; total += x; }
    for (int k = 0; k < kpl; ++k) {
        const int u = u0 + k * WAVE;
        const bool lg = is_long(u);
        const uint64_t m = __ballot(lg);
        if (lg) s_long[run + __popcll(m & lt)] = (uint16_t)u;
        run += __popcll(m);
    }
    __syncthreads();
    return total;
}

// Long segments, block-cooperatively. Their entries, concatenated in key order, stream
// through an LDS stage CE = STAGE_FLOATS / D entries at a time: all TWG threads fetch the
// rows (STAGE_F4 float4 per thread; the next chunk's fetch is in flight while the current
// chunk is combined), then every piece (segment part) of the chunk is combined in entry
// order by one dim-lane group straight from LDS. A segment crossing a chunk boundary
// hands its partial row on through a carry row (two, alternating by chunk parity).
//   fbegin(i, lig, acc)      initial value of a segment (head key index i)
//   fend(u, i, lig, acc)     the finished row
template <int LPR, int OP, class Src, class FB, class FE>
DQRM_INLINE void staged_long_segments(const SlotLds& L, int U, int n, const uint16_t* s_long, int nlong,
                                      int* s_wsum, const Src& src, float nlr, FB&& fbegin, FE&& fend) {
    if (nlong == 0) return;  // uniform
    constexpr int D = LPR * 4;
    using DL = DimLane<LPR>;
    constexpr int GD = DL::GD, NDL = DL::NDL;
    constexpr int CE = STAGE_FLOATS / D;          // entries per chunk
    constexpr int SP = CE + 4;                    // stage row pitch (floats) of one dim
    static_assert(D * SP <= STAGE_FLOATS + STAGE_PAD, "dim-major stage");
    static_assert(STAGE_F4 <= LONG_SEG + 1, "forward walk: at most one segment boundary per lane group");
    const uint64_t* keys = L.keys;
    const uint16_t* heads = L.heads;
    int* lpre = L.lpre;
    // exclusive prefix of the long segments' lengths
    {
        constexpr int PER = (LONG_SEGS_MAX + TWG - 1) / TWG;
        int len[PER], cnt = 0;
#pragma unroll
        for (int c = 0; c < PER; ++c) {
            const int k = threadIdx.x * PER + c;
            len[c] = 0;
            if (k < nlong) { const int u = s_long[k]; len[c] = seg_end(heads, U, n, u) - (int)heads[u]; }
            cnt += len[c];
        }
        int total;
        int run = block_excl_scan(cnt, s_wsum, &total);
#pragma unroll
        for (int c = 0; c < PER; ++c) {
            const int k = threadIdx.x * PER + c;
            if (k < nlong) lpre[k] = run;
            run += len[c];
        }
        if (threadIdx.x == 0) lpre[nlong] = total;
        __syncthreads();
    }
    const int E = lpre[nlong];
    DIAG_T(8);
    // largest k in [lo, hi] with lpre[k] <= e
    auto seg_of = [&](int e, int lo, int hi) {
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (lpre[mid] <= e) lo = mid; else hi = mid - 1;
        }
        return lo;
    };
    const int sub = threadIdx.x % LPR;
    typename Src::Raw raw[STAGE_F4];
    // lane group g stages entries [c0 + g*STAGE_F4, +STAGE_F4): one segment search, then a
    // forward walk (segments are > LONG_SEG >= STAGE_F4 entries long)
    auto fetch = [&](int c0) {
        const int e0 = c0 + (threadIdx.x / LPR) * STAGE_F4;
        if (e0 >= E) return;
        int k = seg_of(e0, 0, nlong - 1);
        int kstart = lpre[k], kend = lpre[k + 1];
        int hk = heads[s_long[k]];
#pragma unroll
        for (int f = 0; f < STAGE_F4; ++f) {
            const int e = e0 + f;
            if (e < E) {
                if (e >= kend) {
                    ++k;
                    kstart = kend;
                    kend = lpre[k + 1];
                    hk = heads[s_long[k]];
                }
                raw[f] = src.fetch(key_lo(keys[hk + (e - kstart)]), sub);
            }
        }
    };
    const int dg = threadIdx.x / GD, ndg = TWG / GD, lig = threadIdx.x % GD;
    fetch(0);
    int par = 0;
    for (int c0 = 0; c0 < E; c0 += CE, par ^= 1) {
        {  // dim-major stage[dim * SP + entry]: the lane group's 8 consecutive entries of each
           // of its 4 dims go out as two 16-B writes per dim (transposed in registers)
            static_assert(STAGE_F4 == 8, "two float4 per dim row");
            const int el0 = (threadIdx.x / LPR) * STAGE_F4;
            float4 v[STAGE_F4];
#pragma unroll
            for (int f = 0; f < STAGE_F4; ++f)
                v[f] = c0 + el0 + f < E ? src.finish(raw[f]) : make_float4(0.f, 0.f, 0.f, 0.f);
            if (c0 + el0 < E) {
                float* base = L.stage + (4 * sub) * SP + el0;
                *reinterpret_cast<float4*>(base) = make_float4(v[0].x, v[1].x, v[2].x, v[3].x);
                *reinterpret_cast<float4*>(base + 4) = make_float4(v[4].x, v[5].x, v[6].x, v[7].x);
                *reinterpret_cast<float4*>(base + SP) = make_float4(v[0].y, v[1].y, v[2].y, v[3].y);
                *reinterpret_cast<float4*>(base + SP + 4) = make_float4(v[4].y, v[5].y, v[6].y, v[7].y);
                *reinterpret_cast<float4*>(base + 2 * SP) = make_float4(v[0].z, v[1].z, v[2].z, v[3].z);
                *reinterpret_cast<float4*>(base + 2 * SP + 4) = make_float4(v[4].z, v[5].z, v[6].z, v[7].z);
                *reinterpret_cast<float4*>(base + 3 * SP) = make_float4(v[0].w, v[1].w, v[2].w, v[3].w);
                *reinterpret_cast<float4*>(base + 3 * SP + 4) = make_float4(v[4].w, v[5].w, v[6].w, v[7].w);
            }
        }
        __syncthreads();
        if (c0 == 0) DIAG_T(9);
        if (c0 + CE < E) fetch(c0 + CE);
        const int ce = min(CE, E - c0);
        const int kf = seg_of(c0, 0, nlong - 1), kl = seg_of(c0 + ce - 1, kf, nlong - 1);
        for (int k = kf + dg; k <= kl; k += ndg) {
            const int sb = lpre[k], se = lpre[k + 1];
            const int a0 = max(sb, c0), a1 = min(se, c0 + ce);
            const int u = s_long[k], i = heads[u];
            float acc[NDL];
            bool first = sb >= c0;
            if (first) {
                fbegin(i, lig, acc);
            } else {
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = L.carry[(par ^ 1) * 256 + lig + GD * d];
            }
            // the piece's entries of this lane's dims: col[d][e0 + j], j < len
            const int e0 = a0 - c0, len = a1 - a0;
            const float* col[NDL];
#pragma unroll
            for (int d = 0; d < NDL; ++d) col[d] = L.stage + (lig + GD * d) * SP + e0;
            auto op = [&](float x, float y) {
                return OP == OP_FMA ? fmaf(y, nlr, x) : (OP == OP_AXPY ? x + y * nlr : x + y);
            };
            int j = 0;
            if (OP == OP_SUM && first && len > 0) {  // peel: the chain below is adds only
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = col[d][0];
                j = 1;
            }
            for (; j < len && ((e0 + j) & 3); ++j)  // up to a 16-B boundary
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = op(acc[d], col[d][j]);
            // strictly ordered chain over 4-entry float4 reads; the next VB float4s per dim
            // are in flight while the current ones are added (ping-pong, no copies)
            constexpr int VB = NDL >= 4 ? 1 : 4 / NDL;
            constexpr int BE = 4 * VB;  // entries per batch
            float4 xa[VB][NDL], xb[VB][NDL];
            auto loadb = [&](float4 (&x)[VB][NDL], int jj) {
#pragma unroll
                for (int v = 0; v < VB; ++v)
#pragma unroll
                    for (int d = 0; d < NDL; ++d) x[v][d] = *reinterpret_cast<const float4*>(col[d] + jj + 4 * v);
            };
            auto addb = [&](const float4 (&x)[VB][NDL]) {
#pragma unroll
                for (int v = 0; v < VB; ++v)
#pragma unroll
                    for (int d = 0; d < NDL; ++d)
                        acc[d] = op(op(op(op(acc[d], x[v][d].x), x[v][d].y), x[v][d].z), x[v][d].w);
            };
            if (j + BE <= len) {
                loadb(xa, j);
                while (true) {
                    const bool m1 = j + 2 * BE <= len;
                    if (m1) loadb(xb, j + BE);
                    addb(xa);
                    j += BE;
                    if (!m1) break;
                    const bool m2 = j + 2 * BE <= len;
                    if (m2) loadb(xa, j + BE);
                    addb(xb);
                    j += BE;
                    if (!m2) break;
                }
            }
            for (; j + 4 <= len; j += 4) {
#pragma unroll
                for (int d = 0; d < NDL; ++d) {
                    const float4 x = *reinterpret_cast<const float4*>(col[d] + j);
                    acc[d] = op(op(op(op(acc[d], x.x), x.y), x.z), x.w);
                }
            }
            for (; j < len; ++j)
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = op(acc[d], col[d][j]);
            if (se <= c0 + ce) {
                fend(u, i, lig, acc);
            } else {
#pragma unroll
                for (int d = 0; d < NDL; ++d) L.carry[par * 256 + lig + GD * d] = acc[d];
            }
        }
        if (c0 == 0) DIAG_T(10);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------
// Incremental |W| hierarchy maintenance (exact), per slot.
// Before it runs, every head key carries its row's record (row_record: new max |W| and a
// "held the block max and shrank" bit). A block's new max is max(old blkmax, new maxima of
// its touched rows) unless a flagged row is among them (then the block's 256 rowmax, which
// the segment phase keeps current, are re-read). The slot owns its
// blocks; superblocks can be shared between slots: increases go in with an order-free
// atomicMax on the (non-negative) float bits, a holder that shrank flags the superblock,
// and the table's last workgroup (finalize_table) re-reduces flagged superblocks and tmax.
// ------------------------------------------------------------------------------------
DQRM_INLINE void update_superblock(float* sblkmax, uint8_t* sdirty, int64_t sb, float old_blk, float nb) {
    const float old_sb = sblkmax[sb];
    if (old_blk == old_sb && nb < old_blk) flag_set(sdirty, sb);
    if (nb > old_sb) atomicMax(reinterpret_cast<unsigned int*>(sblkmax) + sb, __float_as_uint(nb));
}

// Blocks whose max may have dropped are queued in LDS (the stage region, free by now) and
// re-reduced by whole waves (64 lanes x 4 rows = one 256-row block per round trip).
DQRM_INLINE void maintain_blocks(const Meta& m, int t, const SlotLds& sl, int U, const float* rowmax,
                                 float* blkmax, float* sblkmax, uint8_t* sdirty, int* s_cnt) {
    const uint64_t* keys = sl.keys;
    const uint16_t* heads = sl.heads;
    uint32_t* queue = reinterpret_cast<uint32_t*>(sl.stage);
    const int64_t nrows = m.num_rows[t];
    const int64_t rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    if (threadIdx.x == 0) *s_cnt = 0;
    __syncthreads();
    for (int u = threadIdx.x; u < U; u += blockDim.x) {
        const uint32_t blk = key_row(keys[heads[u]]) >> 8;
        if (u > 0 && (key_row(keys[heads[u - 1]]) >> 8) == blk) continue;  // not a block start
        // end of the block's heads: first head whose row is in a later block
        int lo = u + 1, hi = U;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((key_row(keys[heads[mid]]) >> 8) == blk) lo = mid + 1; else hi = mid;
        }
        const float old_blk = blkmax[bb + blk];
        bool dec = lo - u > 32;  // crowded block: one wave re-reducing it beats a serial walk
        float cand = 0.0f;
        for (int k = u; k < lo && !dec; ++k) {  // the block's row records (LDS)
            const uint32_t rec = key_lo(keys[heads[k]]);
            dec |= (rec >> 31) != 0u;
            cand = fmaxf(cand, __uint_as_float(rec & 0x7FFFFFFFu));
        }
        if (dec) {  // re-reduce the block's rowmax (kept current by the segment phase)
            queue[atomicAdd(s_cnt, 1)] = blk;
            continue;
        }
        const float nb = fmaxf(old_blk, cand);
        st_wt(blkmax + bb + blk, nb);
        update_superblock(sblkmax, sdirty, sbb + (blk >> 8), old_blk, nb);
    }
    __syncthreads();
    const int nq = *s_cnt;
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    for (int k = w; k < nq; k += TWG / WAVE) {
        const uint32_t blk = queue[k];
        const int64_t r0 = (int64_t)blk * BLK;
        float v = 0.0f;
#pragma unroll
        for (int j = 0; j < BLK / WAVE; ++j) {
            const int64_t r = r0 + lane + j * WAVE;
            if (r < nrows) v = fmaxf(v, rowmax[rb + r]);
        }
        v = wave_max(v);
        if (lane == 0) {
            const float old_blk = blkmax[bb + blk];
            st_wt(blkmax + bb + blk, v);
            update_superblock(sblkmax, sdirty, sbb + (blk >> 8), old_blk, v);
        }
    }
}


// One workgroup per table after the slot kernels (a kernel boundary is the cheap way to
// make the slots' writes visible here: an agent-scope fence inside the slot kernel, e.g. a
// "last workgroup finalizes" counter, writes back the XCD's L2 and measured 2x slower).
// flagged (after the flat apply kernels, which keep every table's maxima -- narrow ones
// included -- exact but for the blocks / superblocks they flagged, and mark such tables in
// FLAG_WORD): a table that flagged nothing is skipped after one load.
__global__ void __launch_bounds__(1024) k_table_finalize(const float* __restrict__ W, float* __restrict__ rowmax,
                                                         float* __restrict__ blkmax, float* __restrict__ sblkmax,
                                                         uint8_t* __restrict__ sdirty, uint8_t* __restrict__ bdirty,
                                                         float* __restrict__ tmax,
                                                         const int64_t* __restrict__ meta, int T, int D,
                                                         int tracked, uint32_t* __restrict__ sync, int flagged) {
    const Meta m = make_meta(meta, T);
    const int t = blockIdx.x;
    if (flagged) {
        uint32_t* fw = sync + (int64_t)t * DQRM_SYNC_STRIDE + FLAG_WORD;
        if (*fw == 0u) return;  // uniform
        __syncthreads();  // every thread has read the word before it is cleared
        if (threadIdx.x == 0) *fw = 0u;
    }
    finalize_table<false, false, 4, 4>(m, t, W, rowmax, blkmax, sblkmax, sdirty, bdirty, tmax, D, tracked != 0,
                                       flagged == 0);
}

// The flat apply's finalize and the next batch's forward in ONE launch (dqrm_apply_sparse_update_fwd
// / dqrm_exchange_apply_fwd with the flat apply kernel: weight_update_parallel_comm, s_q_g_p_c.py:601-628,
// then the next apply_emb, single_gpu.py:609-674). Workgroups 0..T-1 finalize one table each as
// k_table_finalize does (1024 threads), store the table max
// write-through and open the table's gate; the forward workgroups behind them (k_emb_fwd's grid, table
// by table) issue their index and row loads at once -- W is final at launch start, only the
// maxima may still move -- and take the scale from the table max once the gate is open. The gates
// are opened by lower-numbered workgroups, which are dispatched first, so they are resident before
// any forward workgroup polls (bounded polls: DQRM_ERRF_STALL, no hang).
struct FinArgs {
    const float* W;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    float* tmax;
    int D;
    int tracked, flagged;
};

constexpr int FINFWD_TPB = 1024;  // the finalize's 16 waves (as k_table_finalize); the forward's bag passes alike

template <int LPR, int UNR>
__global__ void __launch_bounds__(FINFWD_TPB) k_finalize_fwd(FwdArgs a, FinArgs f, int gx) {
    const int T = a.T;
    if ((int)blockIdx.x < T) {
        const int t = blockIdx.x;
        bool fin = true;
        if (f.flagged) {
            uint32_t* fw = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FLAG_WORD;
            fin = *fw != 0u;  // uniform
            __syncthreads();  // every thread has read the word before it is cleared
            if (fin && threadIdx.x == 0) *fw = 0u;
        }
        uint32_t* gate = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FINFWD_GATE_WORD;
        auto open_gate = [gate]() {  // the table max is final (and, if it moved, stored write-through)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(gate, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        if (fin)  // the gate opens as soon as the table max is known final, the lower levels after it
            finalize_table<false, true, 4, 1>(make_meta(a.meta, T), t, f.W, f.rowmax, f.blkmax, f.sblkmax, f.sdirty,
                                              f.bdirty, f.tmax, f.D, f.tracked != 0, f.flagged == 0, open_gate);
        else
            open_gate();
        return;
    }
    const int id = (int)blockIdx.x - T;
    const int t = id / gx;
    emb_fwd_table<LPR, UNR, false, true, FINFWD_TPB>(a, t, id - t * gx, gx);
}

// gather the lookups of table t whose row falls in [r0, r1) as keys (row << 32 | bag);
// deterministic placement (count, block-scan, write; keys end up in bag order); returns
// the key count, or -1 (uniform) when the slot overflows SLOT_KEYS. Each thread owns a
// contiguous run of bags, processed GB at a time with every offset / first-index load of
// the batch in flight together.
template <class Visit>
DQRM_INLINE void visit_slot_lookups(const int64_t* off, const int64_t* idx, int64_t B, int64_t L,
                                    int64_t nrows, int64_t b0, int64_t b1, bool report, uint32_t* err,
                                    bool pool1, Visit&& visit) {
    constexpr int GB = 8;
    if (pool1 && L == B) {  // Criteo form: bag b = lookup b, no offsets round trip
        for (int64_t bs = b0; bs < b1; bs += GB) {
            int64_t r[GB];
#pragma unroll
            for (int k = 0; k < GB; ++k) r[k] = bs + k < b1 ? idx[bs + k] : -1;
#pragma unroll
            for (int k = 0; k < GB; ++k) {
                if (bs + k >= b1) continue;
                if (r[k] < 0 || r[k] >= nrows) {
                    if (report) flag_error(err, DQRM_ERRF_INDEX);
                    continue;
                }
                visit(r[k], bs + k);
            }
        }
        return;
    }
    for (int64_t bs = b0; bs < b1; bs += GB) {
        int64_t o[GB + 1];
#pragma unroll
        for (int k = 0; k <= GB; ++k) {  // GB+1 offsets in flight
            const int64_t b = bs + k;
            o[k] = b < B ? off[b] : L;
        }
        int64_t beg[GB], end[GB], first[GB];
#pragma unroll
        for (int k = 0; k < GB; ++k) {  // validate, then the first index of every bag in flight
            const int64_t b = bs + k;
            int64_t s0 = o[k], s1 = o[k + 1];
            if (b < b1 && (s0 < 0 || s1 > L || s1 < s0 || (b == 0 && s0 != 0))) {  // off[0] must be 0
                if (report) flag_error(err, DQRM_ERRF_OFFSET);
                s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
                s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
            }
            beg[k] = s0;
            end[k] = b < b1 ? s1 : s0;
            first[k] = end[k] > s0 ? idx[s0] : -1;
        }
#pragma unroll
        for (int k = 0; k < GB; ++k) {
            const int64_t b = bs + k;
            for (int64_t p = beg[k]; p < end[k]; ++p) {
                const int64_t r = p == beg[k] ? first[k] : idx[p];
                if (r < 0 || r >= nrows) {
                    if (report) flag_error(err, DQRM_ERRF_INDEX);
                    continue;
                }
                visit(r, b);
            }
        }
    }
}

// dy row of bag `lo` for the STE backward: g' = (g * s) / s  (quant_utils.py:349-363);
// off4 = first float4 of the row this slot owns (dimension-split tables)
struct DySource {
    const float* base;  // dy + t * dst_t
    int64_t st_b;
    float s;
    int ste;
    int off4;
    float div = 1.0f;   // dqrm_emb_bwd_coalesce_scaled: g' / div (simulated DP's grad / N)
    using Raw = float4;
    DQRM_INLINE float4 fetch(uint32_t bag, int sub) const {
        return reinterpret_cast<const float4*>(base + (int64_t)bag * st_b)[off4 + sub];
    }
    DQRM_INLINE float4 finish(float4 g) const {
        if (ste) {
            g.x = (g.x * s) / s; g.y = (g.y * s) / s; g.z = (g.z * s) / s; g.w = (g.w * s) / s;
        }
        if (div != 1.0f) {
            g.x = g.x / div; g.y = g.y / div; g.z = g.z / div; g.w = g.w / div;
        }
        return g;
    }
    DQRM_INLINE float4 load(uint32_t bag, int sub) const { return finish(fetch(bag, sub)); }
};

// Narrow tables (at most one 256-row block, i.e. every row would fall into one slot) are
// split across the SPLIT slots by DIMENSION instead: slot s owns float4s
// [s*LPRS, (s+1)*LPRS) of every row. All slots gather and sort the same keys, each streams
// only its slice of the rows, so the long ordered segments of tiny hot tables run on 8
// CUs at once. Per-row maxima of such tables are rebuilt by finalize_table; in the
// coalesced workspace / payload the table's entries sit in slot SPLIT-1 (which owns the
// table's single block in the row split).
template <int LPR>
struct DimSplit {
    static constexpr int LPRS = LPR / SPLIT > 0 ? LPR / SPLIT : 1;
    static constexpr int ACTIVE = LPR / LPRS;  // slots with a slice
};

DQRM_INLINE bool narrow_table(int64_t nrows) { return nrows <= BLK; }

// ------------------------------------------------------------------------------------
// K5: scale average + quantize-pack (slot workspace -> dense wire payload)
// ------------------------------------------------------------------------------------
// (the wire payload layout, PayloadLayout / payload_layout: dqrm_device.h)

// rank r's local scale from its slots' max |grad| (quant_utils.py:141-194 on the coalesced
// values), then dist.all_reduce(SUM) + mul_(1./N) (s_q_g_p_c.py:861-866). Gloo's allreduce
// of a one-element tensor accumulates in descending rank order
// (((s_{N-1} + s_{N-2}) + ...) + s_0) — measured for N = 2..8 with torch 2.10's Gloo;
// every rank evaluates the same order on the all-gathered values, so the average is
// bit-identical across ranks and equal to the reference's.
DQRM_INLINE float rank_scale(const float* absmax_all, int T, int r, int t, int bits) {
    float a = 0.0f;
    for (int s = 0; s < SPLIT; ++s) a = fmaxf(a, absmax_all[((int64_t)r * T + t) * SPLIT + s]);
    return sym_scale(a, bits);
}

DQRM_INLINE float average_scale(const float* absmax_all, int T, int N, int t, int bits) {
    const float inv_n = (float)(1.0 / (double)N);
    float acc = rank_scale(absmax_all, T, N - 1, t, bits);
    for (int r = N - 2; r >= 0; --r) acc = acc + rank_scale(absmax_all, T, r, t, bits);
    return acc * inv_n;
}

// One workgroup per (table, slot): the table's 8 slot counts are clamped in slot order
// against the table's payload capacity (overflow truncates the table), the N ranks'
// per-slot max|grad| are staged in LDS and averaged in Gloo's order, then LPR lanes per
// entry quantize and store the slot's entries at their dense payload position. Workgroup
// (t, 0) also writes the table's header counts and s_avg[t].
template <int LPR>
__global__ void __launch_bounds__(512) k_quant_pack(int T, const int64_t* __restrict__ ws_cap_base,
                                                    int64_t ws_cap_total, const int32_t* __restrict__ ws_rows,
                                                    const float* __restrict__ ws_vals,
                                                    const int32_t* __restrict__ ws_ucount,
                                                    const float* __restrict__ absmax_all, int64_t am_pitch,
                                                    int N, int bits,
                                                    const int64_t* __restrict__ cap_base, int64_t cap_total,
                                                    float* __restrict__ s_avg, unsigned char* __restrict__ payload,
                                                    const int32_t* __restrict__ tbits,
                                                    const float* __restrict__ tscale) {
    __shared__ int s_cnt[SPLIT];
    __shared__ float s_am[64 * SPLIT];
    __shared__ int s_pre, s_my;
    __shared__ float s_sc;
    (void)ws_cap_total;
    const int k = blockIdx.x, t = k / SPLIT, s = k % SPLIT;
    const int D = LPR * 4;
    const PayloadLayout pl = payload_layout(T, cap_total, D, bits);
    // ranking range (tbits != NULL): per-table bit width and scale; 0 / 32-bit tables send
    // nothing (grad_update_parallel_comm skips them, s_q_g_p_c.py:280-289)
    const int tb = tbits ? tbits[t] : bits;
    const bool ranked = tbits != nullptr;
    const bool send = !ranked || (tb >= 2 && tb <= 8);
    const bool quant = !ranked && bits >= 2 && bits <= 16;
    if (threadIdx.x < SPLIT) s_cnt[threadIdx.x] = send ? ws_ucount[t * SPLIT + threadIdx.x] : 0;
    if (quant)
        for (int j = threadIdx.x; j < N * SPLIT; j += blockDim.x)
            s_am[j] = absmax_all[(int64_t)(j / SPLIT) * am_pitch + t * SPLIT + (j % SPLIT)];
    __syncthreads();
    if (threadIdx.x == 0) {
        const int cap = (int)(cap_base[t + 1] - cap_base[t]);
        int run = 0;
        for (int ss = 0; ss < SPLIT; ++ss) {
            int c = s_cnt[ss];
            c = c < cap - run ? c : cap - run;  // overflow: the table's payload is truncated
            c = c < 0 ? 0 : c;
            if (ss == s) { s_pre = run; s_my = c; }
            if (s == 0) reinterpret_cast<int32_t*>(payload)[t * SPLIT + ss] = c;
            run += c;
        }
        if (quant) {  // rank scales, then Gloo's one-element all_reduce order
            const float inv_n = (float)(1.0 / (double)N);
            float acc = 0.0f;
            for (int r = N - 1; r >= 0; --r) {
                float am = 0.0f;
                for (int ss = 0; ss < SPLIT; ++ss) am = fmaxf(am, s_am[r * SPLIT + ss]);
                const float sr = sym_scale(am, bits);
                acc = r == N - 1 ? sr : acc + sr;
            }
            const float sv = acc * inv_n;
            s_sc = sv;
            if (s == 0) s_avg[t] = sv;
        }
    }
    __syncthreads();
    const int cnt = s_my;
    const int64_t src0 = ws_cap_base[k], dst0 = cap_base[t] + s_pre;
    const bool qv = quant || (ranked && send);  // values are quantized
    const float rr = quant ? 1.0f / s_sc : (qv ? 1.0f / tscale[t] : 0.0f);
    const int lane = threadIdx.x % LPR;
    constexpr int QU = 4;                 // entries in flight per lane group
    constexpr int EPI = 512 / LPR;        // lane groups per workgroup
    const int qb = ranked ? (send ? tb : 2) : bits;
    const float qlo = -(float)(1 << (qb - 1)), qhi = (float)((1 << (qb - 1)) - 1);
    for (int u0 = threadIdx.x / LPR; u0 < cnt; u0 += QU * EPI) {
        float4 v[QU];
        int32_t row[QU];
#pragma unroll
        for (int h = 0; h < QU; ++h) {  // QU entries' loads in flight
            const int u = u0 + h * EPI;
            if (u < cnt) {
                v[h] = reinterpret_cast<const float4*>(ws_vals + (src0 + u) * D)[lane];
                row[h] = ws_rows[src0 + u];
            }
        }
#pragma unroll
        for (int h = 0; h < QU; ++h) {
            const int u = u0 + h * EPI;
            if (u >= cnt) continue;
            const int64_t q = dst0 + u;  // dense payload entry
            if (lane == 0) reinterpret_cast<int32_t*>(payload + pl.rows_off)[q] = row[h];
            if (!qv) {
                reinterpret_cast<float4*>(payload + pl.vals_off + q * D * 4)[lane] = v[h];
                continue;
            }
            const float q0 = fake_quant(v[h].x, rr, qlo, qhi), q1 = fake_quant(v[h].y, rr, qlo, qhi);
            const float q2 = fake_quant(v[h].z, rr, qlo, qhi), q3 = fake_quant(v[h].w, rr, qlo, qhi);
            if (pl.elem == 1) {
                uint32_t pk = ((uint32_t)(uint8_t)(int8_t)(int)q0) | ((uint32_t)(uint8_t)(int8_t)(int)q1 << 8) |
                              ((uint32_t)(uint8_t)(int8_t)(int)q2 << 16) | ((uint32_t)(uint8_t)(int8_t)(int)q3 << 24);
                reinterpret_cast<uint32_t*>(payload + pl.vals_off + q * D)[lane] = pk;
            } else {
                uint2 pk;
                pk.x = ((uint32_t)(uint16_t)(int16_t)(int)q0) | ((uint32_t)(uint16_t)(int16_t)(int)q1 << 16);
                pk.y = ((uint32_t)(uint16_t)(int16_t)(int)q2) | ((uint32_t)(uint16_t)(int16_t)(int)q3 << 16);
                reinterpret_cast<uint2*>(payload + pl.vals_off + q * D * 2)[lane] = pk;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// K6: decode N payloads, union rows, sum, dequantize, SGD update + maintenance.
// Slot (t, s) binary-searches each rank's sorted row list for its row range;
// keys = (row << 32) | (rank << 24) | entry.
// ------------------------------------------------------------------------------------
struct ApplyArgs {
    float* W;
    uint8_t* packed;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    float* tmax;
    uint32_t* sync;
    int fin_launch;    // 1: the |W| hierarchy is finalized by a separate k_table_finalize launch
    int wt;            // rowmax / narrow-table W stores write-through (needed by the in-launch finalize)
    const float* pscale;
    const int64_t* meta;
    uint32_t* err;
    const int64_t* cap_base;
    int64_t cap_total;
    const unsigned char* payloads;
    int64_t payload_bytes;
    int N;
    int T;
    int bits;
    const float* s_avg;
    float nlr;
    int mode;
    int repack;
};

// one payload entry (rank = lo >> 24, entry = lo & 0xFFFFFF) widened to f32
template <int LPR>
struct PayloadSource {
    const unsigned char* payloads;
    int64_t payload_bytes;
    PayloadLayout pl;
    int64_t cap_base_t;
    int off4;  // first float4 of the row this slot owns (dimension-split tables)
    using Raw = uint4;
    DQRM_INLINE uint4 fetch(uint32_t lo, int sub) const {
        constexpr int D = LPR * 4;
        const unsigned char* p = payloads + (int64_t)(lo >> 24) * payload_bytes + pl.vals_off;
        const int64_t e = cap_base_t + (int64_t)(lo & 0xFFFFFF);
        uint4 x = make_uint4(0u, 0u, 0u, 0u);
        if (pl.elem == 1) {
            x.x = reinterpret_cast<const uint32_t*>(p + e * D)[off4 + sub];
        } else if (pl.elem == 2) {
            const uint2 y = reinterpret_cast<const uint2*>(p + e * D * 2)[off4 + sub];
            x.x = y.x; x.y = y.y;
        } else {
            x = reinterpret_cast<const uint4*>(p + e * D * 4)[off4 + sub];
        }
        return x;
    }
    DQRM_INLINE float4 finish(uint4 x) const {
        float4 v;
        if (pl.elem == 1) {
            v.x = (float)(int8_t)(x.x & 0xFF); v.y = (float)(int8_t)((x.x >> 8) & 0xFF);
            v.z = (float)(int8_t)((x.x >> 16) & 0xFF); v.w = (float)(int8_t)(x.x >> 24);
        } else if (pl.elem == 2) {
            v.x = (float)(int16_t)(x.x & 0xFFFF); v.y = (float)(int16_t)(x.x >> 16);
            v.z = (float)(int16_t)(x.y & 0xFFFF); v.w = (float)(int16_t)(x.y >> 16);
        } else {
            v = __builtin_bit_cast(float4, x);
        }
        return v;
    }
    DQRM_INLINE float4 load(uint32_t lo, int sub) const { return finish(fetch(lo, sub)); }
};


template <int LPR, int LPRS>
DQRM_INLINE void apply_segments(const ApplyArgs& a, const SlotLds& sl, uint16_t* s_long, int* s_wsum, const Meta& m,
                                int t, int U, int n, int off4, bool dsplit, const PayloadLayout& pl) {
    constexpr int D = LPR * 4;
    uint64_t* keys = sl.keys;
    const uint16_t* heads = sl.heads;
    const int64_t rb = m.row_base[t];
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate update{a.mode, (float)(1.0 / (double)a.N), sc, (float)((double)sc / (double)a.N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    PayloadSource<LPR> src{a.payloads, a.payload_bytes, pl, a.cap_base[t], off4};

    auto finit = [&](int, int i, int sub, SegState& st) {
        const int64_t grow = rb + key_row(keys[i]);
        st.w = reinterpret_cast<const float4*>(a.W + grow * D)[off4 + sub];
        if (!dsplit) st.blk = a.blkmax[m.blk_base[t] + (key_row(keys[i]) >> 8)];
        st.acc = make_float4(0.f, 0.f, 0.f, 0.f);
    };
    // integer-valued sums are exact in f32 (|sum| <= 2^15 * N << 2^24);
    // FP32 path: rank-ordered sum, as Gloo's sparse allreduce + coalesce
    auto ffin = [&](int, int i, int sub, SegState& st) {
        const int64_t grow = rb + key_row(keys[i]);
        float4 w = st.w;
        w.x = update(w.x, st.acc.x); w.y = update(w.y, st.acc.y);
        w.z = update(w.z, st.acc.z); w.w = update(w.w, st.acc.w);
        st4_w(reinterpret_cast<float4*>(a.W + grow * D) + off4 + sub, w, dsplit);
        if (a.repack) pack4_row(w, a.packed + grow * (D / 2), off4 + sub, r_pack);
        if (!dsplit) {
            const float old_rm = group_max<LPRS>(abs_max4(st.w));
            const float rm = group_max<LPRS>(abs_max4(w));
            if (sub == 0) {
                st_wt(a.rowmax + grow, rm);
                keys[i] = with_lo(keys[i], row_record(rm, old_rm, st.blk));
            }
        }
    };
    short_segments<LPRS, OP_SUM, 8>(keys, heads, U, n, src, 0.0f, finit, ffin);

    using DL = DimLane<LPRS>;
    auto fbegin = [&](int, int, float (&acc)[DL::NDL]) {
#pragma unroll
        for (int d = 0; d < DL::NDL; ++d) acc[d] = 0.0f;
    };
    auto fend = [&](int, int i, int lig, float (&acc)[DL::NDL]) {
        const int64_t grow = rb + key_row(keys[i]);
        float w[DL::NDL];
#pragma unroll
        for (int d = 0; d < DL::NDL; ++d) w[d] = a.W[grow * D + off4 * 4 + lig + DL::GD * d];
        const float old_rm = dsplit ? 0.0f : dl_absmax<LPRS>(w);
        const float old_blk = dsplit ? 0.0f : a.blkmax[m.blk_base[t] + (key_row(keys[i]) >> 8)];
#pragma unroll
        for (int d = 0; d < DL::NDL; ++d) w[d] = update(w[d], acc[d]);
#pragma unroll
        for (int d = 0; d < DL::NDL; ++d) st_w(a.W + grow * D + off4 * 4 + lig + DL::GD * d, w[d], dsplit);
        if (a.repack) dl_pack_int4<LPRS>(w, a.packed + grow * (D / 2), off4 * 4, lig, r_pack);
        if (!dsplit) {
            const float rm = dl_absmax<LPRS>(w);
            if (lig == 0) {
                st_wt(a.rowmax + grow, rm);
                keys[i] = with_lo(keys[i], row_record(rm, old_rm, old_blk));
            }
        }
    };
    const int nlong = compact_long(heads, U, n, s_long, s_wsum);
    DIAG_T(3);
    staged_long_segments<LPRS, OP_SUM>(sl, U, n, s_long, nlong, s_wsum, src, 0.0f, fbegin, fend);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // rowmax stores land before maintain_blocks reads them
    __syncthreads();
    DIAG_T(4);
    if (!dsplit) maintain_blocks(m, t, sl, U, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, s_wsum + TWG / WAVE + 2);
}

DQRM_INLINE int find_row(const int32_t* rows, int n, int32_t x);
// a workgroup's queue of shrunk block-max holders whose blocks it owns (k_apply_local)
struct OwnQueue {
    int* cnt;
    uint32_t* blk;
    float* old;
};
constexpr int OWN_QCAP = 64;
template <int LPR>
DQRM_INLINE void flat_row_update(const ApplyArgs& a, const ApplyUpdate& update, int t, int64_t grow, int64_t x,
                                 int64_t nrows, int64_t bb, int64_t sbb, float4 acc, float r_pack, int sub,
                                 bool owned = false, const OwnQueue* oq = nullptr);

// A slot whose merged entries exceed SLOT_KEYS (LDS sort capacity): k_apply_flat's method
// restricted to the slot. Every rank's slot rows are ascending, so the entry of row x in
// rank j is a binary search of rank j's slot range; the lowest rank holding x owns the row
// and sums the ranks' values in ascending rank order (= the sorted path's order).
template <int LPR>
DQRM_INLINE void apply_slot_flat(const ApplyArgs& a, const Meta& m, int t, const PayloadLayout& pl, const int* s_e0,
                                 const int* s_start, int* pos_lds) {
    constexpr int NG = TWG / LPR;
    const int N = a.N;
    const int64_t cb = a.cap_base[t];
    const int64_t nrows = m.num_rows[t], rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate update{a.mode, (float)(1.0 / (double)N), sc, (float)((double)sc / (double)N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const PayloadSource<LPR> src{a.payloads, a.payload_bytes, pl, cb, 0};
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int gbase = (threadIdx.x % WAVE) - sub;
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    int* pos = pos_lds + grp * DQRM_MAX_RANKS;  // LDS, written and read back by the same wave
    auto rows_of = [&](int j) {
        return reinterpret_cast<const int32_t*>(a.payloads + (int64_t)j * a.payload_bytes + pl.rows_off) + cb;
    };
    const int M = s_start[N];
    for (int i = grp; i < M; i += NG) {
        int r = 0;
        while (i >= s_start[r + 1]) ++r;
        const int e = s_e0[r] + (i - s_start[r]);
        const int32_t x = rows_of(r)[e];
        if (x < 0 || x >= nrows) {  // cannot happen for payloads this library packed
            if (sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
            continue;
        }
        bool lower = false;
        for (int j = sub; j < N; j += LPR) {
            int p = e;
            if (j != r) {
                const int q = find_row(rows_of(j) + s_e0[j], s_start[j + 1] - s_start[j], x);
                p = q >= 0 ? s_e0[j] + q : -1;
                lower |= (j < r) && p >= 0;
            }
            pos[j] = p;
        }
        if (__ballot(lower) & gmask) continue;  // a lower rank owns this row (group-uniform)
        bool first = true;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = r; j < N; ++j) {
            const int p = pos[j];
            if (p >= 0) acc = combine<OP_SUM>(acc, src.load(((uint32_t)j << 24) | (uint32_t)p, sub), first, 0.0f);
        }
        flat_row_update<LPR>(a, update, t, rb + x, x, nrows, bb, sbb, acc, r_pack, sub);
    }
}

template <int LPR>
__global__ void __launch_bounds__(TWG) k_table_apply(ApplyArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const SlotLds sl(lds);
    uint64_t* keys = sl.keys;
    __shared__ int s_wsum[TWG / WAVE + 8];
    __shared__ int s_e0[68];
    __shared__ int s_start[68];
    __shared__ uint16_t s_long[(LONG_SEGS_MAX + 7) / 8 * 8];

    const int t = blockIdx.x / SPLIT, s = blockIdx.x % SPLIT;
    const int T = a.T;
    const int D = LPR * 4;
    Meta m = make_meta(a.meta, T);
    // the slot's work; then all SPLIT workgroups of the table arrive and the last one
    // finalizes the table's |W| hierarchy (untracked: block-level maintenance, tmax rescan)
    [&]() {
    const PayloadLayout pl = payload_layout(T, a.cap_total, D, a.bits);
    DIAG_T(0);
    const int64_t cap = a.cap_base[t + 1] - a.cap_base[t];
    const int64_t nrows = m.num_rows[t];
    const bool dsplit = narrow_table(nrows);
    using DS = DimSplit<LPR>;
    int64_t r0, r1;
    int off4 = 0, ps = s;  // ps: the payload slot holding this workgroup's rows
    if (dsplit) {
        if (s >= DS::ACTIVE) return;
        r0 = 0;
        r1 = nrows;
        off4 = s * DS::LPRS;
        ps = SPLIT - 1;
    } else {
        slot_rows(nrows, s, r0, r1);
    }
    if (threadIdx.x < a.N) {  // this slot's entries in rank r's payload: header counts, no search
        const int32_t* cnt = reinterpret_cast<const int32_t*>(a.payloads + (int64_t)threadIdx.x * a.payload_bytes);
        int pre = 0, c = 0;
        for (int k = 0; k < SPLIT; ++k) {
            int x = cnt[t * SPLIT + k];
            x = x < 0 ? 0 : x;
            if (k < ps) pre += x; else if (k == ps) c = x;
        }
        if (pre + c > cap) {  // cannot happen for payloads this library packed
            if (s == 0) flag_error(a.err, DQRM_ERRF_OVERFLOW);
            pre = pre < cap ? pre : (int)cap;
            c = (int)cap - pre;
        }
        s_e0[threadIdx.x] = pre;
        s_start[threadIdx.x] = c;  // count, prefix-summed below
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int r = 0; r < a.N; ++r) { int c = s_start[r]; s_start[r] = run; run += c; }
        s_start[a.N] = run;
    }
    __syncthreads();
    const int M = s_start[a.N];
    if (M > SLOT_KEYS) {  // crowded slot (uniform): the flat method over its entries, full rows
        if (off4 == 0) apply_slot_flat<LPR>(a, m, t, pl, s_e0, s_start, reinterpret_cast<int*>(lds));
        return;
    }
    for (int i = threadIdx.x; i < M; i += blockDim.x) {
        int r = 0;
        while (i >= s_start[r + 1]) ++r;
        const int e = s_e0[r] + (i - s_start[r]);
        const unsigned char* p = a.payloads + (int64_t)r * a.payload_bytes;
        int64_t row = reinterpret_cast<const int32_t*>(p + pl.rows_off)[a.cap_base[t] + e];
        if (row < r0 || row >= r1) {  // cannot happen for payloads this library packed
            flag_error(a.err, DQRM_ERRF_INDEX);
            row = r0;
        }
        keys[i] = ((uint64_t)row << 32) | ((uint64_t)r << 24) | (uint64_t)e;
    }
    __syncthreads();
    const int n = M;
    DIAG_T(1);
    // one rank's rows arrive ascending and unique: already sorted
    const int U = sort_and_heads(sl, n, (uint32_t)r0, (uint32_t)(r1 - r0), s_wsum, a.N == 1);
    DIAG_T(2);
    if (dsplit)
        apply_segments<LPR, DS::LPRS>(a, sl, s_long, s_wsum, m, t, U, n, off4, true, pl);
    else
        apply_segments<LPR, LPR>(a, sl, s_long, s_wsum, m, t, U, n, 0, false, pl);
    DIAG_T(5);
    }();
    if (!a.fin_launch && arrive_last(a.sync + (int64_t)t * DQRM_SYNC_STRIDE, SPLIT))
        finalize_table<true>(m, t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax, D, false);
}

// ------------------------------------------------------------------------------------
// K6 (flat): one lane group (LPR lanes x float4) per payload entry, thousands of
// workgroups, no per-slot sort. Rank r's rows of a table arrive ascending and unique, so
// the entry of row x in rank j is found by a binary search of rank j's row list (lane k of
// the group searches ranks k, k+LPR, ...). The entry of the LOWEST rank holding x owns the
// row: it sums the rank-ordered values (integers: exact in any order; FP32: ascending rank,
// as the slot kernel and Gloo's sparse all_reduce), applies the SGD update, writes rowmax
// and keeps the |W| hierarchy exact without a per-block pass: growth goes in with an
// order-free atomicMax on the non-negative float bits; a row that held its block's max and
// shrank flags the block (bdirty) and its superblock (sdirty) for finalize, which
// re-reduces exactly those. Random 256-B row RMWs from the whole chip at once: the
// translation / HBM latency of the 198 GB slab is overlapped across all CUs instead of
// queueing behind 8 workgroups per table.
// ------------------------------------------------------------------------------------
DQRM_INLINE int table_entry_count(const unsigned char* payload, int t, int64_t cap) {
    const int32_t* cnt = reinterpret_cast<const int32_t*>(payload) + t * SPLIT;
    int c = 0;
#pragma unroll
    for (int k = 0; k < SPLIT; ++k) c += cnt[k] > 0 ? cnt[k] : 0;
    return c < cap ? c : (int)cap;
}

// position of row x in an ascending list of n distinct rows, or -1. A present row is probed on
// the way (the lower bound ends where a probe set hi = its position), so no load after the loop
DQRM_INLINE int find_row(const int32_t* rows, int n, int32_t x) {
    int lo = 0, hi = n, found = -1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int32_t v = rows[mid];
        if (v == x) found = mid;
        if (v < x) lo = mid + 1; else hi = mid;
    }
    return found;
}

constexpr int FLAT_TPB = 256;
constexpr int FLAT_HDR_RANKS = 32;  // k_apply_flat: ranks whose slot bounds it keeps in LDS
#ifndef DQRM_FLAT_PRELOAD
#define DQRM_FLAT_PRELOAD 1  // 0: an A/B build reading the superblock / table max only on growth
#endif

// SGD of row x (global row grow) by one LPR-lane group with the summed value acc, rowmax,
// and the exact |W| hierarchy without a per-block pass: growth goes in with an order-free
// atomicMax on the non-negative float bits; a row that held its block's max and shrank
// flags the block (bdirty) and its superblock (sdirty) for finalize's re-reduction. Rows
// of one call are distinct, so a concurrent grower either raised old_blk before this row
// read it (then the block max is that grower's current value) or the holder is flagged.
// the row and its maxima, loaded before the update's value is known (so they share its round trip)
struct FlatPre {
    float4 w0;
    float old_blk, old_sb, old_tm;
};
template <int LPR>
DQRM_INLINE FlatPre flat_row_preload(const ApplyArgs& a, int t, int64_t grow, int64_t x, int64_t bb, int64_t sbb,
                                     int sub) {
    constexpr int D = LPR * 4;
    const int64_t blk = x >> 8;
    FlatPre p;
    p.w0 = reinterpret_cast<const float4*>(a.W + grow * D)[sub];
    p.old_blk = a.blkmax[bb + blk];
    // the superblock and table maxima with the row (DQRM_FLAT_PRELOAD): no dependent round trips
    // on growth, which early in training is every row of a big table; a stale-low value only
    // costs a redundant atomicMax (within the launch they only grow)
    p.old_sb = DQRM_FLAT_PRELOAD ? a.sblkmax[sbb + (blk >> 8)] : 0.0f;
    p.old_tm = DQRM_FLAT_PRELOAD ? a.tmax[t] : 0.0f;
    return p;
}

template <int LPR>
DQRM_INLINE void flat_row_apply(const ApplyArgs& a, const ApplyUpdate& update, int t, int64_t grow, int64_t x,
                                int64_t nrows, int64_t bb, int64_t sbb, const FlatPre& pre, float4 acc, float r_pack,
                                int sub, bool owned, const OwnQueue* oq) {
    constexpr int D = LPR * 4;
    const int64_t blk = x >> 8;
    const float4 w0 = pre.w0;
    const float old_blk = pre.old_blk, old_sb = pre.old_sb, old_tm = pre.old_tm;
    float4 w;
    w.x = update(w0.x, acc.x); w.y = update(w0.y, acc.y);
    w.z = update(w0.z, acc.z); w.w = update(w0.w, acc.w);
    // narrow tables are rebuilt from W by finalize (write-through: it may run in this launch)
    st4_w(reinterpret_cast<float4*>(a.W + grow * D) + sub, w, nrows <= BLK && a.wt);
    if (a.repack) pack4_row(w, a.packed + grow * (D / 2), sub, r_pack);
    const float old_rm = group_max<LPR>(abs_max4(w0));
    const float rm = group_max<LPR>(abs_max4(w));
    if (sub == 0) {
        // every table, narrow ones (<= 256 rows: one block, one superblock) included: growth by
        // atomicMax, a shrunk block-max holder re-reduced by its owner or flagged
        st_w(a.rowmax + grow, rm, a.wt);
        const int64_t sb = sbb + (blk >> 8);
        if (rm > old_blk) {
            atomicMax(reinterpret_cast<unsigned int*>(a.blkmax) + bb + blk, __float_as_uint(rm));
            if (rm > (DQRM_FLAT_PRELOAD ? old_sb : a.sblkmax[sb])) {
                atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sb, __float_as_uint(rm));
                if (rm > (DQRM_FLAT_PRELOAD ? old_tm : a.tmax[t]))
                    atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(rm));
            }
        }
        if (old_rm == old_blk && rm < old_rm) {
            int p = OWN_QCAP;
            if (owned && oq) {  // the workgroup holds every touched row of this block: it re-reduces it
                p = atomicAdd(oq->cnt, 1);
                if (p < OWN_QCAP) { oq->blk[p] = (uint32_t)blk; oq->old[p] = old_blk; }
            }
            if (p >= OWN_QCAP) {  // the finalize re-reduces the block
                flag_set(a.bdirty, bb + blk);
                flag_set(a.sdirty, sb);
                mark_table_flagged(a.sync, t);
            }
        }
    }
}

template <int LPR>
DQRM_INLINE void flat_row_update(const ApplyArgs& a, const ApplyUpdate& update, int t, int64_t grow, int64_t x,
                                 int64_t nrows, int64_t bb, int64_t sbb, float4 acc, float r_pack, int sub,
                                 bool owned, const OwnQueue* oq) {
    flat_row_apply<LPR>(a, update, t, grow, x, nrows, bb, sbb, flat_row_preload<LPR>(a, t, grow, x, bb, sbb, sub), acc,
                        r_pack, sub, owned, oq);
}

// Single-rank DP step, quantize-pack and apply fused (dqrm_apply_local): grid (entry
// chunks, T * SPLIT workspace slots). Every workgroup derives table t's scale from the
// slots' max|grad| exactly as k_quant_pack does for N = 1 (s = sym_scale(max) * 1.0f),
// quantizes its coalesced entries with k_quant_pack's rounding and applies them with
// k_apply_flat's update: the same values the payload round trip produces, without
// writing and re-reading the payload.
template <int LPR, bool FIN>  // FIN: the table's last working workgroup finalizes its |W| hierarchy
__global__ void __launch_bounds__(FLAT_TPB) k_apply_local(ApplyArgs a, const int64_t* __restrict__ ws_cap_base,
                                                          const int32_t* __restrict__ ws_rows,
                                                          const float* __restrict__ ws_vals,
                                                          const int32_t* __restrict__ ws_ucount,
                                                          const float* __restrict__ ws_absmax,
                                                          float* __restrict__ s_avg) {
    constexpr int D = LPR * 4;
    constexpr int G = FLAT_TPB / LPR;
    const int k = blockIdx.y, t = k / SPLIT;
    // the table's slot counts: this slot's work, and how many workgroups of the table work
    // (each arrives once; the last one finalizes the table's |W| hierarchy)
    int cnt = 0;
    uint32_t expected = 0;
    if constexpr (FIN) {
#pragma unroll
        for (int ss = 0; ss < SPLIT; ++ss) {
            const int kk = t * SPLIT + ss;
            const int64_t cp = ws_cap_base[kk + 1] - ws_cap_base[kk];
            int c = ws_ucount[kk];
            c = c < 0 ? 0 : (c > cp ? (int)cp : c);
            if (kk == k) cnt = c;
            const uint32_t wgs = (uint32_t)((c + G - 1) / G);
            expected += wgs < gridDim.x ? wgs : gridDim.x;
        }
    } else {
        const int64_t cp = ws_cap_base[k + 1] - ws_cap_base[k];
        cnt = ws_ucount[k];
        cnt = cnt < 0 ? 0 : (cnt > cp ? (int)cp : cnt);
    }
    const bool writer = blockIdx.x == 0 && k % SPLIT == 0;  // s_avg[t], even for an empty slot
    if ((int64_t)blockIdx.x * G >= cnt && !writer) return;
    float am = 0.0f;
    for (int ss = 0; ss < SPLIT; ++ss) am = fmaxf(am, ws_absmax[t * SPLIT + ss]);
    const float sv = sym_scale(am, a.bits) * (float)(1.0 / 1.0);
    if (writer && threadIdx.x == 0) s_avg[t] = sv;
    if ((int64_t)blockIdx.x * G >= cnt) return;
    const Meta m = make_meta(a.meta, a.T);
    const float rr = 1.0f / sv;
    const float qlo = -(float)(1 << (a.bits - 1)), qhi = (float)((1 << (a.bits - 1)) - 1);
    const ApplyUpdate update{DQRM_UPD_DP, 1.0f, sv, sv, a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const int64_t nrows = m.num_rows[t], rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    const int64_t src0 = ws_cap_base[k];
    const int sub = threadIdx.x % LPR;
    // FIN = false: a block whose entries all fall in this workgroup's chunk is OWNED here (the
    // slot's rows are ascending, so another entry of the block would be the chunk's neighbour
    // entry): a shrunk holder of such a block is re-reduced below instead of being flagged
    __shared__ int s_oq_n;
    __shared__ uint32_t s_oq_blk[OWN_QCAP];
    __shared__ float s_oq_old[OWN_QCAP];
    const OwnQueue oq{&s_oq_n, s_oq_blk, s_oq_old};
    if (!FIN) {
        if (threadIdx.x == 0) s_oq_n = 0;
        __syncthreads();
    }
    for (int e = blockIdx.x * G + threadIdx.x / LPR; e < cnt; e += gridDim.x * G) {
        const int32_t x = ws_rows[src0 + e];
        const float4 v = reinterpret_cast<const float4*>(ws_vals + (src0 + e) * D)[sub];
        const int c0 = e - (int)(threadIdx.x / LPR);  // the chunk's first entry
        const int32_t xlo = (!FIN && c0 > 0) ? ws_rows[src0 + c0 - 1] : -1;
        const int32_t xhi = (!FIN && c0 + G < cnt) ? ws_rows[src0 + c0 + G] : -1;
        if (x < 0 || x >= nrows) {  // cannot happen for a workspace this library coalesced
            if (sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
            continue;
        }
        float4 acc;  // + 0.0f: the payload's integer round trip turns -0 into +0
        acc.x = fake_quant(v.x, rr, qlo, qhi) + 0.0f; acc.y = fake_quant(v.y, rr, qlo, qhi) + 0.0f;
        acc.z = fake_quant(v.z, rr, qlo, qhi) + 0.0f; acc.w = fake_quant(v.w, rr, qlo, qhi) + 0.0f;
        const bool owned = !FIN && (xlo < 0 || (xlo >> 8) != (x >> 8)) && (xhi < 0 || (xhi >> 8) != (x >> 8));
        flat_row_update<LPR>(a, update, t, rb + x, x, nrows, bb, sbb, acc, r_pack, sub, owned, FIN ? nullptr : &oq);
    }
    if constexpr (!FIN) {  // owned blocks whose max holder shrank: re-reduce their 256 row maxima
        __syncthreads();
        const int nq = s_oq_n < OWN_QCAP ? s_oq_n : OWN_QCAP;
        if (nq > 0) {  // uniform; rare
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's row maxima have landed
            __syncthreads();
            const int lane = threadIdx.x % WAVE;
            for (int q = threadIdx.x / WAVE; q < nq; q += FLAT_TPB / WAVE) {
                const int64_t blk = s_oq_blk[q];
                float mv = 0.0f;
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) {
                    const int64_t r = blk * BLK + lane + i * WAVE;
                    if (r < nrows) mv = fmaxf(mv, ld_wt(a.rowmax + rb + r));  // sc1: past any stale L1 line
                }
                mv = wave_max(mv);
                if (lane == 0) {
                    a.blkmax[bb + blk] = mv;
                    const int64_t sb = sbb + (blk >> 8);
                    if (mv < s_oq_old[q] && s_oq_old[q] == a.sblkmax[sb]) {  // held the superblock max
                        flag_set(a.sdirty, sb);
                        mark_table_flagged(a.sync, t);
                    }
                }
            }
        }
    }
    if constexpr (FIN) {
        if (arrive_last(a.sync + (int64_t)t * DQRM_SYNC_STRIDE, expected))
            finalize_table<true>(m, t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax, D, true);
    }
}

template <int LPR, bool FIN>
__global__ void __launch_bounds__(FLAT_TPB) k_apply_flat(ApplyArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = FLAT_TPB / LPR;               // entries per workgroup pass
    __shared__ int s_pos[G][DQRM_MAX_RANKS];       // per entry: its row's position in each rank
    const int t = blockIdx.y, r = blockIdx.z;
    const int T = a.T, N = a.N;
    const Meta m = make_meta(a.meta, T);
    const PayloadLayout pl = payload_layout(T, a.cap_total, D, a.bits);
    const int64_t cb = a.cap_base[t];
    const int64_t cap = a.cap_base[t + 1] - cb;
    const unsigned char* pr = a.payloads + (int64_t)r * a.payload_bytes;
    // N > 1: every rank's slot bounds of table t in LDS, ONE round trip (thread j*8+q loads rank
    // j's slot-q count; clamped prefix sums in slot order): a row's entry in rank j is then
    // searched within its slot's run only (~3 fewer dependent steps than the whole table's list)
    __shared__ int s_sb[FLAT_HDR_RANKS][SPLIT + 1];
    const bool slot_search = N > 1 && N <= FLAT_HDR_RANKS;
    if (slot_search) {
        if ((int)threadIdx.x < N * SPLIT) {
            const int j = threadIdx.x / SPLIT, q = threadIdx.x % SPLIT;
            int c = reinterpret_cast<const int32_t*>(a.payloads + (int64_t)j * a.payload_bytes)[t * SPLIT + q];
            c = c > 0 ? c : 0;
            int inc = c;  // inclusive prefix over the rank's 8 slots (8 aligned lanes of a wave)
#pragma unroll
            for (int o = 1; o < SPLIT; o <<= 1) {
                const int y = __shfl_up(inc, o, SPLIT);
                if (q >= o) inc += y;
            }
            s_sb[j][q + 1] = inc < cap ? inc : (int)cap;
            if (q == 0) s_sb[j][0] = 0;
        }
        __syncthreads();
    }
    const int cnt_r = slot_search ? s_sb[r][SPLIT] : table_entry_count(pr, t, cap);
    if ((int64_t)blockIdx.x * G >= cnt_r) return;
    // workgroups of table t that work, over all ranks' payloads (each arrives once)
    uint32_t expected = 0;
    if (FIN)
    for (int j = 0; j < N; ++j) {
        const uint32_t wgs =
            (uint32_t)((table_entry_count(a.payloads + (int64_t)j * a.payload_bytes, t, cap) + G - 1) / G);
        expected += wgs < gridDim.x ? wgs : gridDim.x;
    }
    const int64_t nrows = m.num_rows[t], rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate update{a.mode, (float)(1.0 / (double)N), sc, (float)((double)sc / (double)N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const PayloadSource<LPR> src{a.payloads, a.payload_bytes, pl, cb, 0};
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int gbase = (threadIdx.x % WAVE) - sub;   // first lane of this group in the wave
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    int* pos = s_pos[grp];
    const int32_t* rows_r = reinterpret_cast<const int32_t*>(pr + pl.rows_off) + cb;
    // one rank (N == 1, finalize launch after): a block whose entries all fall in this
    // workgroup's chunk is OWNED here (the table's rows are ascending, so another entry of the
    // block would be a neighbour of the chunk): a shrunk holder of it is re-reduced below, as
    // k_apply_local does, instead of flagging the table for the finalize launch
    const bool own_mode = !FIN && N == 1;
    __shared__ int s_oq_n;
    __shared__ uint32_t s_oq_blk[OWN_QCAP];
    __shared__ float s_oq_old[OWN_QCAP];
    OwnQueue oq;  // (filled at run time: a constant aggregate of LDS addresses cannot be a static initializer)
    oq.cnt = &s_oq_n;
    oq.blk = s_oq_blk;
    oq.old = s_oq_old;
    if (own_mode) {
        if (threadIdx.x == 0) s_oq_n = 0;
        __syncthreads();
    }
    for (int e = blockIdx.x * G + grp; e < cnt_r; e += gridDim.x * G) {
        const int32_t x = rows_r[e];
        const int c0 = e - grp;  // the chunk's first entry
        const int32_t xlo = (own_mode && c0 > 0) ? rows_r[c0 - 1] : -1;
        const int32_t xhi = (own_mode && c0 + G < cnt_r) ? rows_r[c0 + G] : -1;
        if (x < 0 || x >= nrows) {  // cannot happen for payloads this library packed
            if (sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
            continue;
        }
        float4 acc;
        if (N == 1) {
            acc = src.load((uint32_t)e, sub);
        } else {  // where the other ranks hold row x (lane k searches ranks k, k+LPR, ...)
            bool lower = false;
            // the slot of row x (slot s holds blocks [nblk*s/8, nblk*(s+1)/8)): its run in each rank
            const int64_t nblk = (nrows + BLK - 1) / BLK;
            const int xs = slot_search ? (int)((8 * ((int64_t)(x >> 8) + 1) + nblk - 1) / nblk) - 1 : 0;
            for (int j = sub; j < N; j += LPR) {
                int p = e;
                if (j != r) {
                    const unsigned char* pj = a.payloads + (int64_t)j * a.payload_bytes;
                    const int32_t* rows_j = reinterpret_cast<const int32_t*>(pj + pl.rows_off) + cb;
                    if (slot_search) {
                        const int lo = s_sb[j][xs], hi = s_sb[j][xs + 1];
                        const int q = find_row(rows_j + lo, hi - lo, x);
                        p = q >= 0 ? lo + q : -1;
                    } else {
                        p = find_row(rows_j, table_entry_count(pj, t, cap), x);
                    }
                    lower |= (j < r) && p >= 0;
                }
                pos[j] = p;  // LDS, read back by the same wave below (in-order LDS within a wave)
            }
            if (__ballot(lower) & gmask) continue;  // a lower rank owns this row (group-uniform)
            // owner: rank-ordered sum of the row's entries (ranks >= r)
            acc = make_float4(0.f, 0.f, 0.f, 0.f);
            if (pl.elem == 1 && N <= 8) {
                // int8 values: every rank's loaded in one round trip (absent ranks read entry 0 and
                // add +0 to the integer sum), then summed in ascending rank order (exact)
                uint32_t raw[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = j < N ? pos[j] : -1;
                    const bool ok = j >= r && p >= 0;
                    raw[j] = reinterpret_cast<const uint32_t*>(a.payloads + (int64_t)(j < N ? j : 0) * a.payload_bytes +
                                                               pl.vals_off + (cb + (ok ? p : 0)) * D)[sub];
                    if (!ok) raw[j] = 0u;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t v = raw[j];
                    acc.x += (float)(int8_t)(v & 0xFF); acc.y += (float)(int8_t)((v >> 8) & 0xFF);
                    acc.z += (float)(int8_t)((v >> 16) & 0xFF); acc.w += (float)(int8_t)(v >> 24);
                }
            } else {
                bool first = true;
                for (int j = r; j < N; ++j) {
                    const int p = pos[j];
                    if (p >= 0) acc = combine<OP_SUM>(acc, src.load(((uint32_t)j << 24) | (uint32_t)p, sub), first, 0.0f);
                }
            }
        }
        const bool owned = own_mode && (xlo < 0 || (xlo >> 8) != (x >> 8)) && (xhi < 0 || (xhi >> 8) != (x >> 8));
        flat_row_update<LPR>(a, update, t, rb + x, x, nrows, bb, sbb, acc, r_pack, sub, owned, own_mode ? &oq : nullptr);
    }
    if (own_mode) {  // owned blocks whose max holder shrank: re-reduce their 256 row maxima
        __syncthreads();
        const int nq = s_oq_n < OWN_QCAP ? s_oq_n : OWN_QCAP;
        if (nq > 0) {  // uniform
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's row maxima have landed
            __syncthreads();
            const int lane = threadIdx.x % WAVE;
            for (int q = threadIdx.x / WAVE; q < nq; q += FLAT_TPB / WAVE) {
                const int64_t blk = s_oq_blk[q];
                float mv = 0.0f;
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) {
                    const int64_t rr = blk * BLK + lane + i * WAVE;
                    if (rr < nrows) mv = fmaxf(mv, ld_wt(a.rowmax + rb + rr));  // sc1: past any stale L1 line
                }
                mv = wave_max(mv);
                if (lane == 0) {
                    a.blkmax[bb + blk] = mv;
                    const int64_t sb = sbb + (blk >> 8);
                    if (mv < s_oq_old[q] && s_oq_old[q] == a.sblkmax[sb]) {  // held the superblock max
                        flag_set(a.sdirty, sb);
                        mark_table_flagged(a.sync, t);
                    }
                }
            }
        }
    }
    if constexpr (FIN) {
        if (arrive_last(a.sync + (int64_t)t * DQRM_SYNC_STRIDE, expected))
            finalize_table<true>(m, t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax, D, true);
    }
}

// E binary searches (find_row's) interleaved: their dependent loads share round trips
template <int E>
DQRM_INLINE void find_rows(const int32_t* const* rs, const int* ns, const int32_t* xs, int* found) {
    int lo[E], hi[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        lo[k] = 0;
        hi[k] = ns[k];
        found[k] = -1;
    }
    for (;;) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < E; ++k) any |= lo[k] < hi[k];
        if (!any) break;
        int32_t v[E];
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] = lo[k] < hi[k] ? rs[k][(lo[k] + hi[k]) >> 1] : 0;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            if (lo[k] >= hi[k]) continue;
            const int mid = (lo[k] + hi[k]) >> 1;
            if (v[k] == xs[k]) found[k] = mid;
            if (v[k] < xs[k]) lo[k] = mid + 1; else hi[k] = mid;
        }
    }
}

// k_apply_flat for 1 < N <= FLAT_HDR_RANKS ranks with the finalize launch after it (the default):
// each lane group takes TWO entries of rank r's payload (e and e + G), whose searches in the other
// ranks' slot runs, value loads and row loads share their round trips -- twice the entries in
// flight per wave at nearly the same registers. Same arithmetic, ownership and |W| upkeep.
// Taken when the tables average >= 512 entries (apply_update_ex); DQRM_FLAT_DUAL=0/1 forces it.
template <int LPR, int E>
__global__ void __launch_bounds__(FLAT_TPB) k_apply_flat2(ApplyArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = FLAT_TPB / LPR;
    __shared__ int s_pos[E][G][DQRM_MAX_RANKS];
    __shared__ int s_sb[FLAT_HDR_RANKS][SPLIT + 1];
    const int t = blockIdx.y, r = blockIdx.z;
    const int T = a.T, N = a.N;
    const Meta m = make_meta(a.meta, T);
    const PayloadLayout pl = payload_layout(T, a.cap_total, D, a.bits);
    const int64_t cb = a.cap_base[t];
    const int64_t cap = a.cap_base[t + 1] - cb;
    const unsigned char* pr = a.payloads + (int64_t)r * a.payload_bytes;
    if ((int)threadIdx.x < N * SPLIT) {  // every rank's slot bounds of table t (as k_apply_flat)
        const int j = threadIdx.x / SPLIT, q = threadIdx.x % SPLIT;
        int c = reinterpret_cast<const int32_t*>(a.payloads + (int64_t)j * a.payload_bytes)[t * SPLIT + q];
        c = c > 0 ? c : 0;
        int inc = c;
#pragma unroll
        for (int o = 1; o < SPLIT; o <<= 1) {
            const int y = __shfl_up(inc, o, SPLIT);
            if (q >= o) inc += y;
        }
        s_sb[j][q + 1] = inc < cap ? inc : (int)cap;
        if (q == 0) s_sb[j][0] = 0;
    }
    __syncthreads();
    const int cnt_r = s_sb[r][SPLIT];
    if ((int64_t)blockIdx.x * E * G >= cnt_r) return;
    const int64_t nrows = m.num_rows[t], rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    const int64_t nblk = (nrows + BLK - 1) / BLK;
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate update{a.mode, (float)(1.0 / (double)N), sc, (float)((double)sc / (double)N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const PayloadSource<LPR> src{a.payloads, a.payload_bytes, pl, cb, 0};
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int gbase = (threadIdx.x % WAVE) - sub;
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    const int32_t* rows_r = reinterpret_cast<const int32_t*>(pr + pl.rows_off) + cb;
    for (int e0 = blockIdx.x * E * G + grp; e0 < cnt_r; e0 += gridDim.x * E * G) {
        int ee[E], xs[E];
        int32_t xx[E];
        bool ok[E];
#pragma unroll
        for (int k = 0; k < E; ++k) {
            ee[k] = e0 + k * G;
            const bool has = ee[k] < cnt_r;
            xx[k] = has ? rows_r[ee[k]] : -1;
        }
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const bool has = ee[k] < cnt_r;
            ok[k] = has && xx[k] >= 0 && xx[k] < nrows;
            if (has && !ok[k] && sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);  // (never for packed payloads)
            xs[k] = ok[k] ? (int)((8 * ((int64_t)(xx[k] >> 8) + 1) + nblk - 1) / nblk) - 1 : 0;
        }
        bool lower[E];
#pragma unroll
        for (int k = 0; k < E; ++k) lower[k] = false;
        for (int j = sub; j < N; j += LPR) {  // lane k searches ranks k, k+LPR, ... for all E entries
            int p[E];
            if (j != r) {
                const int32_t* rows_j =
                    reinterpret_cast<const int32_t*>(a.payloads + (int64_t)j * a.payload_bytes + pl.rows_off) + cb;
                const int32_t* rs[E];
                int lo[E], nn[E], q[E];
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    lo[k] = s_sb[j][xs[k]];
                    nn[k] = ok[k] ? s_sb[j][xs[k] + 1] - lo[k] : 0;
                    rs[k] = rows_j + lo[k];
                }
                find_rows<E>(rs, nn, xx, q);
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    p[k] = q[k] >= 0 ? lo[k] + q[k] : -1;
                    lower[k] |= (j < r) && p[k] >= 0;
                }
            } else {
#pragma unroll
                for (int k = 0; k < E; ++k) p[k] = ee[k];
            }
#pragma unroll
            for (int k = 0; k < E; ++k) s_pos[k][grp][j] = p[k];  // LDS, read back by the same wave below
        }
        bool own[E];
#pragma unroll
        for (int k = 0; k < E; ++k) own[k] = ok[k] && !(__ballot(lower[k]) & gmask);  // lowest holding rank owns it
        FlatPre pre[E];
        float4 acc[E];
#pragma unroll
        for (int k = 0; k < E; ++k) {
            acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (own[k]) pre[k] = flat_row_preload<LPR>(a, t, rb + xx[k], xx[k], bb, sbb, sub);
        }
        if (pl.elem == 1 && N <= 8) {  // int8: both entries' values of every rank in one round trip
            uint32_t raw[E][8];
#pragma unroll
            for (int k = 0; k < E; ++k)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = j < N ? s_pos[k][grp][j] : -1;
                    const bool v = own[k] && j >= r && p >= 0;
                    raw[k][j] = reinterpret_cast<const uint32_t*>(a.payloads + (int64_t)(j < N ? j : 0) * a.payload_bytes +
                                                                  pl.vals_off + (cb + (v ? p : 0)) * D)[sub];
                    if (!v) raw[k][j] = 0u;
                }
#pragma unroll
            for (int k = 0; k < E; ++k)
#pragma unroll
                for (int j = 0; j < 8; ++j) {  // ascending rank order (integers: exact)
                    const uint32_t v = raw[k][j];
                    acc[k].x += (float)(int8_t)(v & 0xFF); acc[k].y += (float)(int8_t)((v >> 8) & 0xFF);
                    acc[k].z += (float)(int8_t)((v >> 16) & 0xFF); acc[k].w += (float)(int8_t)(v >> 24);
                }
        } else {
#pragma unroll
            for (int k = 0; k < E; ++k) {
                if (!own[k]) continue;
                bool first = true;
                for (int j = r; j < N; ++j) {
                    const int p = s_pos[k][grp][j];
                    if (p >= 0) acc[k] = combine<OP_SUM>(acc[k], src.load(((uint32_t)j << 24) | (uint32_t)p, sub), first, 0.0f);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < E; ++k)
            if (own[k])
                flat_row_apply<LPR>(a, update, t, rb + xx[k], xx[k], nrows, bb, sbb, pre[k], acc[k], r_pack, sub, false,
                                    nullptr);
    }
}

// ------------------------------------------------------------------------------------
// Sort and gather helpers of the fused backward (K4, below): a workgroup of SORT_TPB threads
// sorts one slot's (row << 32 | position) keys in LDS or in the caller's workspace.
// ------------------------------------------------------------------------------------
constexpr int SORT_TPB = 512;
constexpr int SORT_WAVES = SORT_TPB / WAVE;
constexpr int SORT_LDS_KEYS = 4096;                 // keys a slot sorts in LDS (32 KiB + 32 KiB)
constexpr int SORT_KC = SORT_LDS_KEYS / SORT_TPB;   // key batches per lane cached in registers
constexpr int RADIX = 256;
constexpr int HP = SORT_WAVES + 1;                  // [digit][wave] counter pitch (odd: no bank conflicts)
// exclusive prefix of one int per thread over NT threads; *total = the sum.
// s_w: NT/WAVE + 1 ints. Two barriers.
template <int NT>
DQRM_INLINE int block_scan_excl(int cnt, int* s_w, int* total) {
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    int v = cnt;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const int y = __shfl_up(v, o, WAVE);
        if (lane >= o) v += y;
    }
    if (lane == WAVE - 1) s_w[w] = v;
    __syncthreads();
    if (w == 0) {  // wave 0 scans the NT/WAVE wave totals
        constexpr int NW = NT / WAVE;
        const int x = lane < NW ? s_w[lane] : 0;
        int y = x;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            const int z = __shfl_up(y, o, WAVE);
            if (lane >= o) y += z;
        }
        if (lane < NW) s_w[lane] = y - x;
        if (lane == NW - 1) s_w[NW] = y;
    }
    __syncthreads();
    *total = s_w[NT / WAVE];
    return s_w[w] + v - cnt;
}

// lanes of the wave whose 8-bit digit equals v, from the eight bit-slice ballots
DQRM_INLINE uint64_t digit_lanes8(uint32_t v, const uint64_t (&b)[8]) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int k = 0; k < 8; ++k) m &= ((v >> k) & 1u) ? b[k] : ~b[k];
    return m;
}

// one wave-batch of 64 keys: the key, its digit, and the lanes sharing it (incl. itself)
DQRM_INLINE void radix_batch(const uint64_t* src, int i, int n, uint32_t r0, int sh, uint64_t& x, uint32_t& d,
                             uint64_t& mine) {
    const bool v = i < n;
    x = v ? src[i] : 0ull;
    d = ((key_row(x) - r0) >> sh) & 255u;
    uint64_t b[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) b[q] = __ballot((d >> q) & 1u);
    mine = digit_lanes8(d, b) & __ballot(v);
}

// Stable LSD radix sort of keys[0, n) by row - r0 (bits [0, nbits)), 8-bit digits. Wave w
// owns keys [w*64*kpl, (w+1)*64*kpl), 64 at a time. Per pass: each batch's same-digit lanes
// come from eight bit-slice ballots; the last lane of a digit adds the batch's count to the
// wave's [digit][wave] counter (its own LDS column: no barrier); one block scan turns the
// counters into bases, and every lane places its key at its base plus the earlier same-digit
// lanes, the last one advancing the base. Up to SORT_KC batches per lane stay in registers
// between the count and the scatter. keys / tmp: LDS or global.
DQRM_INLINE void radix_sort_rows(uint64_t* keys, uint64_t* tmp, int n, uint32_t r0, int nbits, int* hist,
                                 int* s_scan) {
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    const int kpl = (n + SORT_TPB - 1) / SORT_TPB;
    const int i0 = w * WAVE * kpl + lane;
    const uint64_t lt = lanemask_lt();
    const bool cached = kpl <= SORT_KC;
    uint64_t* src = keys;
    uint64_t* dst = tmp;
    for (int sh = 0; sh < nbits; sh += 8) {
        for (int j = threadIdx.x; j < RADIX * HP; j += SORT_TPB) hist[j] = 0;
        __syncthreads();
        uint64_t cx[SORT_KC], cm[SORT_KC];
        uint32_t cd[SORT_KC];
        auto count = [&](int i, uint32_t d, uint64_t mine) {
            if (i < n && (mine >> lane) == 1ull) hist[d * HP + w] += (int)__popcll(mine);
        };
        if (cached) {
#pragma unroll
            for (int k = 0; k < SORT_KC; ++k)
                if (k < kpl) {
                    radix_batch(src, i0 + k * WAVE, n, r0, sh, cx[k], cd[k], cm[k]);
                    count(i0 + k * WAVE, cd[k], cm[k]);
                }
        } else {
            for (int k = 0; k < kpl; ++k) {
                uint64_t x, mine;
                uint32_t d;
                radix_batch(src, i0 + k * WAVE, n, r0, sh, x, d, mine);
                count(i0 + k * WAVE, d, mine);
            }
        }
        __syncthreads();
        {  // exclusive scan of the (digit-major, wave-minor) counters, 4 per thread
            static_assert(SORT_TPB * 4 == RADIX * SORT_WAVES, "4 counters per thread");
            int* h = hist + (threadIdx.x / 2) * HP + (threadIdx.x % 2) * 4;
            const int h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3];
            int tot;
            const int ex = block_scan_excl<SORT_TPB>(h0 + h1 + h2 + h3, s_scan, &tot);
            h[0] = ex; h[1] = ex + h0; h[2] = ex + h0 + h1; h[3] = ex + h0 + h1 + h2;
        }
        __syncthreads();
        auto place = [&](int i, uint64_t x, uint32_t d, uint64_t mine) {
            if (i < n) {
                int* hp = hist + d * HP + w;
                const int pos = *hp + (int)__popcll(mine & lt);
                dst[pos] = x;
                if ((mine >> lane) == 1ull) *hp = pos + 1;
            }
        };
        if (cached) {
#pragma unroll
            for (int k = 0; k < SORT_KC; ++k)
                if (k < kpl) place(i0 + k * WAVE, cx[k], cd[k], cm[k]);
        } else {
            for (int k = 0; k < kpl; ++k) {
                uint64_t x, mine;
                uint32_t d;
                radix_batch(src, i0 + k * WAVE, n, r0, sh, x, d, mine);
                place(i0 + k * WAVE, x, d, mine);
            }
        }
        __syncthreads();
        uint64_t* tt = src;
        src = dst;
        dst = tt;
    }
    if (src != keys) {
        for (int i = threadIdx.x; i < n; i += SORT_TPB) keys[i] = src[i];
        __syncthreads();
    }
}

// Sort of a slot whose keys are few for their row span (a wide table's slot): ONE stable
// 8-bit radix pass on the TOP digit of (row - r0) puts the keys into 256 row-ordered buckets
// of ~n/256 keys, and one thread per bucket finishes it by insertion sort on the full
// (unique) key. A bucket above FIX_MAX keys (power-law rows) falls back to the full LSD radix
// from the untouched input. keys -> keys; tmp, hist as for radix_sort_rows.
constexpr int FIX_MAX = 32;
DQRM_INLINE void msd_sort_rows(uint64_t* keys, uint64_t* tmp, int n, uint32_t r0, int nbits, int* hist, int* s_scan,
                               int* s_flag) {
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    const int kpl = (n + SORT_TPB - 1) / SORT_TPB;
    const int i0 = w * WAVE * kpl + lane;
    const uint64_t lt = lanemask_lt();
    const int sh = nbits - 8;
    int* start = hist + RADIX * HP;  // bucket starts [RADIX + 1]
    for (int j = threadIdx.x; j < RADIX * HP; j += SORT_TPB) hist[j] = 0;
    if (threadIdx.x == 0) *s_flag = 0;
    __syncthreads();
    uint64_t cx[SORT_KC], cm[SORT_KC];
    uint32_t cd[SORT_KC];
#pragma unroll
    for (int k = 0; k < SORT_KC; ++k)
        if (k < kpl) {
            radix_batch(keys, i0 + k * WAVE, n, r0, sh, cx[k], cd[k], cm[k]);
            if (i0 + k * WAVE < n && (cm[k] >> lane) == 1ull) hist[cd[k] * HP + w] += (int)__popcll(cm[k]);
        }
    __syncthreads();
    {
        int* h = hist + (threadIdx.x / 2) * HP + (threadIdx.x % 2) * 4;
        const int h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3];
        int tot;
        const int ex = block_scan_excl<SORT_TPB>(h0 + h1 + h2 + h3, s_scan, &tot);
        h[0] = ex; h[1] = ex + h0; h[2] = ex + h0 + h1; h[3] = ex + h0 + h1 + h2;
        if (threadIdx.x % 2 == 0) start[threadIdx.x / 2] = ex;
        if (threadIdx.x == 0) start[RADIX] = tot;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SORT_KC; ++k)
        if (k < kpl && i0 + k * WAVE < n) {
            int* hp = hist + cd[k] * HP + w;
            const int pos = *hp + (int)__popcll(cm[k] & lt);
            tmp[pos] = cx[k];
            if ((cm[k] >> lane) == 1ull) *hp = pos + 1;
        }
    if (threadIdx.x < RADIX && start[threadIdx.x + 1] - start[threadIdx.x] > FIX_MAX) *s_flag = 1;
    __syncthreads();
    if (*s_flag) {  // crowded bucket: the full LSD sort of the original keys
        radix_sort_rows(keys, tmp, n, r0, nbits, hist, s_scan);
        return;
    }
    if (threadIdx.x < RADIX) {  // insertion sort of bucket d, written back to keys
        const int b0 = start[threadIdx.x], b1 = start[threadIdx.x + 1];
        for (int i = b0; i < b1; ++i) {
            const uint64_t x = tmp[i];
            int j = i;
            while (j > b0 && keys[j - 1] > x) { keys[j] = keys[j - 1]; --j; }
            keys[j] = x;
        }
    }
    __syncthreads();
}

// gather_slot_keys for a Criteo-form batch whose indices the caller already loaded: the
// thread's bags [tid*per, +per) (per <= 8) are pre[0..per)
DQRM_INLINE int gather_slot_keys_pre(uint64_t* lds_keys, uint64_t* ws_keys, bool* in_lds, int* s_scan,
                                     const int64_t (&pre)[8], int per, int64_t B, int64_t nrows, int64_t r0,
                                     int64_t r1, bool report, uint32_t* err) {
    const int64_t b0 = (int64_t)threadIdx.x * per;
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t r = pre[j];
        if (j < per && b0 + j < B) {
            if (r < 0 || r >= nrows) {
                if (report) flag_error(err, DQRM_ERRF_INDEX);
            } else if (r >= r0 && r < r1) {
                ++cnt;
            }
        }
    }
    int total;
    int pos = block_scan_excl<SORT_TPB>(cnt, s_scan, &total);
    *in_lds = total <= SORT_LDS_KEYS;
    uint64_t* keys = *in_lds ? lds_keys : ws_keys;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t r = pre[j];
        if (j < per && b0 + j < B && r >= r0 && r < r1 && r < nrows)
            keys[pos++] = ((uint64_t)r << 32) | (uint64_t)(b0 + j);
    }
    __syncthreads();
    return total;
}

// the slot's keys (row in [r0, r1)) in lookup order into LDS (n <= SORT_LDS_KEYS) or the
// workspace: each thread owns a contiguous run of bags (count, block scan, write; RC keys
// per thread kept in registers). Returns n; *in_lds tells where they went.
DQRM_INLINE int gather_slot_keys(uint64_t* lds_keys, uint64_t* ws_keys, bool* in_lds, int* s_scan,
                                 const int64_t* off, const int64_t* idx, int64_t B, int64_t L, int64_t nrows,
                                 int64_t r0, int64_t r1, bool report, uint32_t* err, bool pool1) {
    const int64_t per = (B + SORT_TPB - 1) / SORT_TPB;
    int64_t b0 = (int64_t)threadIdx.x * per;
    b0 = b0 < B ? b0 : B;
    const int64_t b1 = b0 + per < B ? b0 + per : B;
    constexpr int RC = 8;
    uint64_t cache[RC];
    int cnt = 0;
    visit_slot_lookups(off, idx, B, L, nrows, b0, b1, report, err, pool1, [&](int64_t r, int64_t b) {
        if (r >= r0 && r < r1) {
            const uint64_t key = ((uint64_t)r << 32) | (uint64_t)b;
#pragma unroll
            for (int c = 0; c < RC; ++c)
                if (c == cnt) cache[c] = key;
            ++cnt;
        }
    });
    int total;
    int pos = block_scan_excl<SORT_TPB>(cnt, s_scan, &total);
    *in_lds = total <= SORT_LDS_KEYS;
    uint64_t* keys = *in_lds ? lds_keys : ws_keys;
    if (cnt <= RC) {
#pragma unroll
        for (int c = 0; c < RC; ++c)
            if (c < cnt) keys[pos + c] = cache[c];
    } else {
        visit_slot_lookups(off, idx, B, L, nrows, b0, b1, false, err, pool1, [&](int64_t r, int64_t b) {
            if (r >= r0 && r < r1) keys[pos++] = ((uint64_t)r << 32) | (uint64_t)b;
        });
    }
    __syncthreads();
    return total;
}

template <int OP>
DQRM_INLINE float seg_op(float acc, float v, float nlr) {
    if (OP == OP_FMA) return fmaf(v, nlr, acc);
    if (OP == OP_AXPY) return acc + v * nlr;
    return acc + v;
}

// ------------------------------------------------------------------------------------
// K4 (fused): the backward of one (table, row-range slot) per 512-thread workgroup.
//   STE (quant_utils.py:349-363) + EmbeddingBag sparse backward, then one of
//     MODE 0  torch.optim.SGD on the uncoalesced grad        (dlrm_s_pytorch_single_gpu.py:1736-1750)
//     MODE 1  grad.coalesce() + per-slot max|grad|           (s_q_g_p_c.py:859-861)
//     MODE 2  W.add_(-lr * grad), product rounded            (s_q_g_p_c.py:615-616, ranking range)
//  1. gather: the slot's valid lookups in lookup order (a stable count / scan / write over
//     the table's lookups; keys become (row << 32 | gather position), bags kept aside);
//  2. prefetch: every gathered lookup's dy row (this workgroup's dimensions, STE applied)
//     is loaded into registers BEFORE the sort, so the HBM round trip overlaps it;
//  3. sort by row: a sparse wide slot takes one MSD 8-bit pass + per-bucket insertion sort,
//     everything else a stable 8-bit LSD radix (narrow spans: one pass); the keys are
//     unique, so both give the reference's order (rows ascending, duplicates in lookup order);
//  4. every distinct row (segment) by one float4 lane group, its lookups combined strictly
//     in lookup order from LDS, FB_SB segments per group in flight; outputs written once,
//     the slot's max|grad| reduced in LDS and stored (no atomics).
// Tables with fewer than 8 row blocks (coalesce) or <= 256 rows (SGD: finalize rebuilds
// their maxima) are split by DIMENSION instead: all 8 workgroups see all the table's
// lookups and each owns D/8 dims (>= 4), so the long ordered chains of tiny hot tables run
// on 8 CUs. A slot whose rows do not fit in LDS streams its sorted lookups through a stage
// (segments carried across chunks by the same lane group); one with more than 4096 keys
// sorts in the caller's workspace. There is no per-batch limit.
// Wide-table SGD keeps the |W| hierarchy with the flat protocol (atomicMax growth, dirty
// flags for shrunk holders, tracked finalize).
// ------------------------------------------------------------------------------------
constexpr int FB_TPB = 512;
constexpr int FB_LDS = 156 * 1024;   // dynamic LDS of a workgroup (+ ~1.5 KiB static: 160 KiB)
constexpr int FB_STAGE = 8192;       // floats of the streaming stage
constexpr int FB_PFR = 12;           // prefetched float4 per thread held across the sort
constexpr int FB_SB = 4;             // segments in flight per lane group
static_assert(FB_TPB == SORT_TPB, "the sort helpers assume the workgroup size");

template <int LPR>
struct FGeom {
    static constexpr int D = LPR * 4;
    static constexpr int DSPLIT = LPR < SPLIT ? LPR : SPLIT;  // dim slices (>= 4 dims each)
};

struct FArgs {
    float* W;
    uint8_t* packed;
    float* rowmax;
    float* blkmax;
    float* sblkmax;
    float* tmax;
    uint8_t* sdirty;
    uint8_t* bdirty;
    uint32_t* sync;
    int fin_launch;
    float div;                   // MODE 1: divide each lookup's gradient by this (1 = not)
    const float* scale;
    const float* pscale;
    const int64_t* meta;
    uint32_t* err;
    const int64_t* idx;
    const int64_t* off;
    const int64_t* idx_base;
    int64_t B;
    int pool1;
    const float* dy;
    int64_t dst_t, dst_b;
    int T;
    int ste;
    float nlr;
    int repack;
    const int32_t* tmask;
    const int64_t* ws_cap_base;  // MODE 1 outputs
    int32_t* ws_rows;
    float* ws_vals;
    int32_t* ws_ucount;
    float* ws_absmax;
    uint64_t* gkey;              // [T*S][Lc] spill of slots with > SORT_LDS_KEYS keys
    uint64_t* gtmp;
    uint32_t* gbag;
    int64_t Lc;
    // k_sgd_small<LPR, true>: the next Criteo-form batch's forward after the table's update
    // (dqrm_emb_bwd_sgd_fwd; the same B), emb_fwd_table's arithmetic
    const int64_t* fwd_idx;
    float* fwd_out;
    int64_t fwd_ost_t, fwd_ost_b;
    float* fwd_scale;
    int fwd_bits;
    uint32_t fwd_flags;
};

// workspace: the spill regions, only when a slot can exceed the in-LDS key capacity
__host__ __device__ inline int64_t fused_ws_layout(unsigned char* base, int T, int64_t Lc, FArgs* fa) {
    if (Lc <= SORT_LDS_KEYS) {
        if (fa) { fa->gkey = nullptr; fa->gtmp = nullptr; fa->gbag = nullptr; }
        return 16;
    }
    const int64_t n = (int64_t)T * SPLIT * Lc;
    const int64_t o1 = align16(n * 8), o2 = o1 + align16(n * 8), o3 = o2 + align16(n * 4);
    if (fa) {
        fa->gkey = reinterpret_cast<uint64_t*>(base);
        fa->gtmp = reinterpret_cast<uint64_t*>(base + o1);
        fa->gbag = reinterpret_cast<uint32_t*>(base + o2);
    }
    return o3;
}

// row-range slot of a row (slot_rows' inverse): the largest s with floor(nblk*s/SPLIT) <= blk
DQRM_INLINE int slot_of_row(uint32_t row, int64_t nblk) {
    const uint32_t blk = row >> 8, nb = (uint32_t)nblk;  // 32-bit: nblk < 2^24
    return (int)((SPLIT * (blk + 1) + nb - 1) / nb) - 1;
}

template <int OP>
DQRM_INLINE float4 seg_op4(float4 acc, float4 v, float nlr) {
    if (OP == OP_FMA) {
        acc.x = fmaf(v.x, nlr, acc.x); acc.y = fmaf(v.y, nlr, acc.y);
        acc.z = fmaf(v.z, nlr, acc.z); acc.w = fmaf(v.w, nlr, acc.w);
    } else if (OP == OP_AXPY) {
        acc.x = acc.x + v.x * nlr; acc.y = acc.y + v.y * nlr;
        acc.z = acc.z + v.z * nlr; acc.w = acc.w + v.w * nlr;
    } else {
        acc.x = acc.x + v.x; acc.y = acc.y + v.y; acc.z = acc.z + v.z; acc.w = acc.w + v.w;
    }
    return acc;
}

// |W| hierarchy upkeep of one updated row of a wide table (see flat_row_update)
DQRM_INLINE void fused_row_upkeep(const FArgs& a, int t, int64_t grow, uint32_t x, int64_t bb, int64_t sbb,
                                  float old_rm, float rm, float old_blk) {
    st_wt(a.rowmax + grow, rm);
    const int64_t blk = x >> 8;
    const int64_t sb = sbb + (blk >> 8);
    if (rm > old_blk) {
        atomicMax(reinterpret_cast<unsigned int*>(a.blkmax) + bb + blk, __float_as_uint(rm));
        if (rm > a.sblkmax[sb]) {
            atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sb, __float_as_uint(rm));
            if (rm > a.tmax[t]) atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(rm));
        }
    }
    if (old_rm == old_blk && rm < old_rm) {
        flag_set(a.bdirty, bb + blk);
        flag_set(a.sdirty, sb);
    }
}

// One workgroup's segment outputs. LG lanes (float4 each) per segment, at float4 offset
// q0 = dim0/4 of the row.
struct FOut {
    int t;
    int64_t rb, bb, sbb;
    bool wide_upkeep;         // SGD on a row-split wide table: rowmax + flat protocol
    float r_pack;
    const int* ufirst;        // MODE 1: first segment of each row-range slot (LDS)
    const int64_t* cb;        // MODE 1: coalesced workspace slot bases (LDS, SPLIT + 1)
    int64_t nblk;
    int q0;
    // SGD on a row-split slot of <= FB_AGG blocks: per-block growth / shrink aggregated in
    // LDS (a slot owns its blocks), one update per block instead of one atomic per row
    unsigned int* bgrow;
    unsigned int* bshr;
    int64_t b0s;
};
constexpr int FB_AGG = 64;

template <int LPR, int MODE, int LG>
DQRM_INLINE void fused_write(const FArgs& a, const FOut& o, int u, uint32_t x, float4 acc, float4 wold, float oblk,
                             int lane, float& amax) {
    constexpr int D = LPR * 4;
    const int64_t grow = o.rb + x;
    if (MODE == 1) {
        const int s = slot_of_row(x, o.nblk);
        const int64_t e = o.cb[s] + (u - o.ufirst[s]);
        if (e < o.cb[s + 1]) {
            reinterpret_cast<float4*>(a.ws_vals + e * D)[o.q0 + lane] = acc;
            if (o.q0 == 0 && lane == 0) a.ws_rows[e] = (int32_t)x;
        }
        amax = fmaxf(amax, abs_max4(acc));
    } else {
        // narrow (dim-split) tables: write-through, the table's last workgroup rebuilds from W
        st4_w(reinterpret_cast<float4*>(a.W + grow * D) + o.q0 + lane, acc, !o.wide_upkeep);
        if (a.repack) pack4_row(acc, a.packed + grow * (D / 2), o.q0 + lane, o.r_pack);
        if (o.wide_upkeep) {
            const float old_rm = group_max<LG>(abs_max4(wold));
            const float rm = group_max<LG>(abs_max4(acc));
            if (lane == 0) {
                if (o.bgrow) {
                    st_wt(a.rowmax + grow, rm);
                    const int jb = (int)((x >> 8) - o.b0s);
                    atomicMax(&o.bgrow[jb], __float_as_uint(rm));
                    if (old_rm == oblk && rm < old_rm) o.bshr[jb] = 1u;
                } else {
                    fused_row_upkeep(a, o.t, grow, x, o.bb, o.sbb, old_rm, rm, oblk);
                }
            }
        }
    }
}

// Prefetched path: every gathered lookup's row slice sits in LDS at dyl[g * LG + lane].
// the ordered chain of sorted lookups [e, e1) of one segment from the prefetched rows:
// gather positions 4 per 16-B read, two batches of 8 rows in flight (double buffer)
template <int LG, int OP>
DQRM_INLINE float4 walk_prefetched(float4 acc, const float4* dyl, const uint32_t* gsp, int e, int e1, int lane,
                                   float nlr) {
    for (; e < e1 && (e & 3); ++e) acc = seg_op4<OP>(acc, dyl[gsp[e] * LG + lane], nlr);
    if (e + 8 <= e1) {
        const uint4* g4 = reinterpret_cast<const uint4*>(gsp);
        float4 va[8], vb[8];
        auto load8 = [&](float4 (&v)[8], int ee) {
            const uint4 p = g4[ee / 4], q = g4[ee / 4 + 1];
            v[0] = dyl[p.x * LG + lane]; v[1] = dyl[p.y * LG + lane]; v[2] = dyl[p.z * LG + lane];
            v[3] = dyl[p.w * LG + lane]; v[4] = dyl[q.x * LG + lane]; v[5] = dyl[q.y * LG + lane];
            v[6] = dyl[q.z * LG + lane]; v[7] = dyl[q.w * LG + lane];
        };
        auto add8 = [&](const float4 (&v)[8]) {
#pragma unroll
            for (int c = 0; c < 8; ++c) acc = seg_op4<OP>(acc, v[c], nlr);
        };
        load8(va, e);
        while (true) {
            const bool m1 = e + 16 <= e1;
            if (m1) load8(vb, e + 8);
            add8(va);
            e += 8;
            if (!m1) break;
            const bool m2 = e + 16 <= e1;
            if (m2) load8(va, e + 8);
            add8(vb);
            e += 8;
            if (!m2) break;
        }
    }
    for (; e < e1; ++e) acc = seg_op4<OP>(acc, dyl[gsp[e] * LG + lane], nlr);
    return acc;
}

template <int LPR, int MODE, int LG>
DQRM_INLINE void fused_segments_lds(const FArgs& a, const FOut& o, const uint64_t* keys, const uint32_t* gsp,
                                    const uint32_t* hpos, int U, int n, const float4* dyl, float& amax) {
    constexpr int D = LPR * 4;
    constexpr int NG = FB_TPB / LG;
    constexpr int OP = MODE == 0 ? OP_FMA : (MODE == 2 ? OP_AXPY : OP_SUM);
    const int lane = threadIdx.x % LG, grp = threadIdx.x / LG;
    for (int u0 = grp; u0 < U; u0 += NG * FB_SB) {
        int h[FB_SB], e1[FB_SB];
        uint32_t x[FB_SB];
        float4 wold[FB_SB];
        float oblk[FB_SB];
#pragma unroll
        for (int b = 0; b < FB_SB; ++b) {  // the W rows of all SB segments in flight
            const int u = u0 + b * NG;
            h[b] = 0; e1[b] = 0; x[b] = 0;
            if (u < U) {
                h[b] = (int)hpos[u];
                e1[b] = u + 1 < U ? (int)hpos[u + 1] : n;
                x[b] = key_row(keys[h[b]]);
                if (MODE != 1) {
                    const int64_t grow = o.rb + x[b];
                    wold[b] = reinterpret_cast<const float4*>(a.W + grow * D)[o.q0 + lane];
                    oblk[b] = o.wide_upkeep ? a.blkmax[o.bb + (x[b] >> 8)] : 0.0f;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < FB_SB; ++b) {
            const int u = u0 + b * NG;
            if (u >= U) continue;
            float4 acc;
            int e = h[b];
            if (MODE == 1) {
                acc = dyl[gsp[e] * LG + lane];
                ++e;
            } else {
                acc = wold[b];
            }
            acc = walk_prefetched<LG, OP>(acc, dyl, gsp, e, e1[b], lane, a.nlr);  // strictly in lookup order
            fused_write<LPR, MODE, LG>(a, o, u, x[b], acc, wold[b], oblk[b], lane, amax);
        }
    }
}

// Staged path (long chains, or rows that do not fit in LDS): after the sort, the sorted
// lookups' row slices stream through a DIM-MAJOR stage (stage[dim * SP + entry], CE entries
// per chunk), so a lane owning one dimension reads 4 consecutive lookups per 16-B LDS read
// and the ordered chain runs at add latency. Dim-lane group g (GL lanes, NDL dims each)
// combines segments u = g (mod NGL), carrying its running row in registers into the next
// chunk (only a chunk's last segment continues, and the same group owns it there).
template <int LPR, int MODE, int LG>
DQRM_INLINE void fused_segments_staged(const FArgs& a, const FOut& o, const uint64_t* keys, const uint32_t* bags,
                                       const uint32_t* hpos, int U, int n, float* stage, int stage_floats,
                                       const DySource& src, float& amax) {
    constexpr int D = LPR * 4;
    constexpr int SW = LG * 4;
    constexpr int GL = SW < 16 ? SW : (SW / 4 > 16 ? SW / 4 : 16);  // <= 4 dims per lane, >= 8 groups
    constexpr int NDL = SW / GL;
    constexpr int NGL = FB_TPB / GL;
    constexpr int OP = MODE == 0 ? OP_FMA : (MODE == 2 ? OP_AXPY : OP_SUM);
    constexpr int FQ = 16;  // (lookup, float4) items per thread in flight
    // SGD: W rows of a group's next WB segments loaded in one round trip (<= 32 KiB of LDS)
    constexpr int WB0 = 8192 / (NGL * (SW + 1));
    constexpr int WB = WB0 < 1 ? 1 : (WB0 > 8 ? 8 : WB0);
    // SGD: per-group LDS area for the batch of W row slices and their old block maxima
    float* wbuf = stage + (MODE != 1 ? stage_floats - NGL * WB * (SW + 1) : 0);
    if (MODE != 1) stage_floats -= NGL * WB * (SW + 1);
    int CE = (stage_floats / SW - 4) & ~3;
    CE = CE < n ? CE : ((n + 3) & ~3);
    const int SP = CE + 4;
    const int lig = threadIdx.x % GL, g = threadIdx.x / GL;
    const int dim0 = o.q0 * 4;
    float* wb = wbuf + g * WB * (SW + 1);
    auto seg_of = [&](int e) {  // segment holding sorted position e
        int lo = 0, hi = U - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((int)hpos[mid] <= e) lo = mid; else hi = mid - 1;
        }
        return lo;
    };
    float acc[NDL], wo[NDL];
    float orm = 0.0f, oblk = 0.0f;
#pragma unroll
    for (int d = 0; d < NDL; ++d) { acc[d] = 0.0f; wo[d] = 0.0f; }
    for (int c0 = 0; c0 < n; c0 += CE) {
        const int ce = min(CE, n - c0);
        for (int q0 = threadIdx.x; q0 < ce * LG; q0 += FB_TPB * FQ) {  // fetch, FQ items in flight
            float4 v[FQ];
#pragma unroll
            for (int f = 0; f < FQ; ++f) {
                const int q = q0 + f * FB_TPB;
                if (q < ce * LG) v[f] = src.fetch(bags[key_lo(keys[c0 + q / LG])], q % LG);
            }
#pragma unroll
            for (int f = 0; f < FQ; ++f) {
                const int q = q0 + f * FB_TPB;
                if (q < ce * LG) {
                    const float4 x = src.finish(v[f]);
                    float* col = stage + (4 * (q % LG)) * SP + q / LG;
                    col[0] = x.x; col[SP] = x.y; col[2 * SP] = x.z; col[3 * SP] = x.w;
                }
            }
        }
        __syncthreads();
        const int uf = seg_of(c0), ul = seg_of(c0 + ce - 1);
        const int ug = uf + ((g - uf % NGL) + NGL) % NGL;  // this group's first segment here
        for (int u = ug; u <= ul; u += NGL) {
            const int jb = ((u - ug) / NGL) % WB;  // slot in the group's W batch
            if (MODE != 1 && jb == 0) {  // the next WB segments' W slices (those that begin here)
#pragma unroll
                for (int j = 0; j < WB; ++j) {
                    const int uu = u + j * NGL;
                    if (uu <= ul && (int)hpos[uu] >= c0) {
                        const uint32_t xx = key_row(keys[hpos[uu]]);
                        const int64_t gr = o.rb + xx;
#pragma unroll
                        for (int d = 0; d < NDL; ++d) wb[j * (SW + 1) + lig + GL * d] = a.W[gr * D + dim0 + lig + GL * d];
                        if (lig == 0) wb[j * (SW + 1) + SW] = o.wide_upkeep ? a.blkmax[o.bb + (xx >> 8)] : 0.0f;
                    }
                }
            }
            const int sb = (int)hpos[u], se = u + 1 < U ? (int)hpos[u + 1] : n;
            const uint32_t x = key_row(keys[sb]);
            const int64_t grow = o.rb + x;
            const bool begin = sb >= c0;
            int e = (begin ? sb : c0) - c0;
            const int e1 = (se < c0 + ce ? se : c0 + ce) - c0;
            const float* col[NDL];
#pragma unroll
            for (int d = 0; d < NDL; ++d) col[d] = stage + (lig + GL * d) * SP;
            if (begin) {
                if (MODE == 1) {
#pragma unroll
                    for (int d = 0; d < NDL; ++d) acc[d] = col[d][e];
                    ++e;
                } else {
#pragma unroll
                    for (int d = 0; d < NDL; ++d) { acc[d] = wb[jb * (SW + 1) + lig + GL * d]; wo[d] = acc[d]; }
                    if (o.wide_upkeep) {
                        float mx = 0.0f;
#pragma unroll
                        for (int d = 0; d < NDL; ++d) mx = fmaxf(mx, fabsf(wo[d]));
                        orm = group_max<GL>(mx);
                        oblk = wb[jb * (SW + 1) + SW];
                    }
                }
            }
            for (; e < e1 && (e & 3); ++e)  // to a 16-B boundary
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = seg_op<OP>(acc[d], col[d][e], a.nlr);
            constexpr int VB = NDL >= 4 ? 1 : 4 / NDL;  // float4 per dim per batch
            constexpr int BE = 4 * VB;
            float4 xa[VB][NDL], xb[VB][NDL];
            auto loadb = [&](float4 (&xx)[VB][NDL], int jj) {
#pragma unroll
                for (int vv = 0; vv < VB; ++vv)
#pragma unroll
                    for (int d = 0; d < NDL; ++d) xx[vv][d] = *reinterpret_cast<const float4*>(col[d] + jj + 4 * vv);
            };
            auto addb = [&](const float4 (&xx)[VB][NDL]) {
#pragma unroll
                for (int vv = 0; vv < VB; ++vv)
#pragma unroll
                    for (int d = 0; d < NDL; ++d)
                        acc[d] = seg_op<OP>(seg_op<OP>(seg_op<OP>(seg_op<OP>(acc[d], xx[vv][d].x, a.nlr), xx[vv][d].y,
                                                                  a.nlr), xx[vv][d].z, a.nlr), xx[vv][d].w, a.nlr);
            };
            if (e + BE <= e1) {  // ping-pong: the next batch in flight while this one is added
                loadb(xa, e);
                while (true) {
                    const bool m1 = e + 2 * BE <= e1;
                    if (m1) loadb(xb, e + BE);
                    addb(xa);
                    e += BE;
                    if (!m1) break;
                    const bool m2 = e + 2 * BE <= e1;
                    if (m2) loadb(xa, e + BE);
                    addb(xb);
                    e += BE;
                    if (!m2) break;
                }
            }
            for (; e < e1; ++e)
#pragma unroll
                for (int d = 0; d < NDL; ++d) acc[d] = seg_op<OP>(acc[d], col[d][e], a.nlr);
            if (se > c0 + ce) continue;  // continues in the next chunk (same group, acc carried)
            if (MODE == 1) {
                const int sl = slot_of_row(x, o.nblk);
                const int64_t ew = o.cb[sl] + (u - o.ufirst[sl]);
                if (ew < o.cb[sl + 1]) {
#pragma unroll
                    for (int d = 0; d < NDL; ++d) a.ws_vals[ew * D + dim0 + lig + GL * d] = acc[d];
                    if (dim0 == 0 && lig == 0) a.ws_rows[ew] = (int32_t)x;
                }
#pragma unroll
                for (int d = 0; d < NDL; ++d) amax = fmaxf(amax, fabsf(acc[d]));
            } else {
#pragma unroll
                for (int d = 0; d < NDL; ++d) st_w(a.W + grow * D + dim0 + lig + GL * d, acc[d], !o.wide_upkeep);
                if (a.repack) {  // even lanes pack their nibble with the odd neighbour's
#pragma unroll
                    for (int d = 0; d < NDL; ++d) {
                        const int qv = (int)fake_quant(acc[d], o.r_pack, -8.0f, 7.0f) + 8;
                        const int qn = __shfl_xor(qv, 1, WAVE);
                        const int dim = dim0 + lig + GL * d;
                        if ((dim & 1) == 0) a.packed[grow * (D / 2) + dim / 2] = (uint8_t)(qv | (qn << 4));
                    }
                }
                if (o.wide_upkeep) {
                    float mx = 0.0f;
#pragma unroll
                    for (int d = 0; d < NDL; ++d) mx = fmaxf(mx, fabsf(acc[d]));
                    const float rm = group_max<GL>(mx);
                    if (lig == 0) {
                        if (o.bgrow) {
                            st_wt(a.rowmax + grow, rm);
                            const int jb = (int)((x >> 8) - o.b0s);
                            atomicMax(&o.bgrow[jb], __float_as_uint(rm));
                            if (orm == oblk && rm < orm) o.bshr[jb] = 1u;
                        } else {
                            fused_row_upkeep(a, o.t, grow, x, o.bb, o.sbb, orm, rm, oblk);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
}

template <int LPR, int MODE, int LG>
DQRM_INLINE void fused_slot(const FArgs& a, unsigned char* lds, int k, int t, int s, bool dsplit, int z, int64_t r0,
                            int64_t r1, int* s_scan, int* s_wl, int* s_ufirst, int64_t* s_cb, float& amax,
                            const int64_t (&pre)[8], int per) {
    constexpr int D = LPR * 4;
    constexpr int SW = LG * 4;  // dims this workgroup owns
    const Meta m = make_meta(a.meta, a.T);
    const int64_t nrows = m.num_rows[t];
    const int64_t ib = a.pool1 ? (int64_t)t * a.B : a.idx_base[t];
    const int64_t L = a.pool1 ? a.B : a.idx_base[t + 1] - ib;
    if (L > a.Lc) {  // more lookups than the caller planned for: skipped, flagged
        if (threadIdx.x == 0 && (dsplit ? s == 0 : s == SPLIT - 1)) flag_error(a.err, DQRM_ERRF_OVERFLOW);
        if (MODE == 1 && threadIdx.x < SPLIT && (!dsplit || z == 0)) s_ufirst[threadIdx.x] = 0;
        return;
    }
    // 1. gather (keys into LDS at offset 0 when they fit)
    uint64_t* lkeys = reinterpret_cast<uint64_t*>(lds);
    bool in_lds;
    uint64_t* gk = a.gkey ? a.gkey + (int64_t)k * a.Lc : nullptr;
    const bool report = dsplit ? s == 0 : s == SPLIT - 1;
    const int n = per > 0 ? gather_slot_keys_pre(lkeys, gk, &in_lds, s_scan, pre, per, a.B, nrows, r0, r1, report, a.err)
                          : gather_slot_keys(lkeys, gk, &in_lds, s_scan, a.off + (int64_t)t * a.B, a.idx + ib, a.B,
                                             L, nrows, r0, r1, report, a.err, a.pool1 != 0);
    if (n == 0) return;
    uint64_t* keys = in_lds ? lkeys : a.gkey + (int64_t)k * a.Lc;
    // LDS carve for n keys: keys | tmp (radix ping-pong / bitonic exchange / heads) | bags | data
    const int64_t o_tmp = align16((int64_t)n * 8);
    const int64_t o_bag = o_tmp + align16((int64_t)(n > FB_TPB ? n : FB_TPB) * 8);
    const int64_t o_dat = o_bag + align16((int64_t)n * 4);
    uint64_t* tmp = in_lds ? reinterpret_cast<uint64_t*>(lds + o_tmp) : a.gtmp + (int64_t)k * a.Lc;
    uint32_t* bags = in_lds ? reinterpret_cast<uint32_t*>(lds + o_bag) : a.gbag + (int64_t)k * a.Lc;
    unsigned char* data = in_lds ? lds + o_dat : lds;
    // prefetch (gather order) when the slot's rows fit and its segments are short on average
    // (a wide slot, or a dim-split table with enough rows); long chains take the staged path
    const int64_t span_rows = r1 - r0;
    const bool pf = in_lds && o_dat + (int64_t)n * SW * 4 <= FB_LDS && (int64_t)n <= 4 * span_rows;
    DIAG_T(1);
    // 2. prefetch this workgroup's slice of every gathered lookup's dy row into registers:
    //    the loads stay in flight across the sort (barriers wait for LDS traffic only)
    const DySource src{a.dy + (int64_t)t * a.dst_t, a.dst_b, a.scale[t], a.ste, dsplit ? z * LG : 0, a.div};
    float4 pfv[FB_PFR];
    if (pf) {
#pragma unroll
        for (int f = 0; f < FB_PFR; ++f) {
            const int q = threadIdx.x + FB_TPB * f;
            if (q < n * LG) pfv[f] = src.fetch(key_lo(lkeys[q / LG]), q % LG);
        }
    }
    __syncthreads();  // every key read: now rewrite them
    for (int g = threadIdx.x; g < n; g += FB_TPB) {  // keys -> (row, gather position), bags aside
        const uint64_t x = keys[g];
        bags[g] = key_lo(x);
        keys[g] = (x & 0xFFFFFFFF00000000ull) | (uint64_t)g;
    }
    __syncthreads();
    DIAG_T(6);
    // 3. sort by row
    const uint32_t span = (uint32_t)(r1 - r0);
    const int nbits = span <= 1 ? 0 : 32 - __builtin_clz(span - 1);
    if (nbits > 12 && n <= FB_TPB)  // a sparse wide slot (~1 key per bucket): one MSD pass + fix-up
        msd_sort_rows(keys, tmp, n, (uint32_t)r0, nbits, reinterpret_cast<int*>(data), s_scan, s_wl + FB_TPB / WAVE);
    else
        radix_sort_rows(keys, tmp, n, (uint32_t)r0, nbits, reinterpret_cast<int*>(data), s_scan);
    DIAG_T(2);
    // the prefetched rows land in LDS (the sort's histogram region is free again); rows past
    // the register budget are loaded now
    float4* dyl = reinterpret_cast<float4*>(data);
    if (pf) {
#pragma unroll
        for (int f = 0; f < FB_PFR; ++f) {
            const int q = threadIdx.x + FB_TPB * f;
            if (q < n * LG) dyl[q] = src.finish(pfv[f]);
        }
        for (int q = threadIdx.x + FB_TPB * FB_PFR; q < n * LG; q += FB_TPB)
            dyl[q] = src.load(bags[q / LG], q % LG);
    }
    // 4. heads (first sorted key of every distinct row) -> hpos (tmp is free)
    uint32_t* hpos = reinterpret_cast<uint32_t*>(tmp);
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    const uint64_t lt = lanemask_lt();
    int U;
    {
        const int kpl = (n + FB_TPB - 1) / FB_TPB;
        const int i0 = w * WAVE * kpl + lane;
        auto is_head = [&](int i) { return i < n && (i == 0 || key_row(keys[i]) != key_row(keys[i - 1])); };
        int hc = 0;
        for (int q = 0; q < kpl; ++q) hc += (int)__popcll(__ballot(is_head(i0 + q * WAVE)));
        if (lane == 0) s_wl[w] = hc;
        __syncthreads();
        int run = 0;
        U = 0;
        for (int q = 0; q < FB_TPB / WAVE; ++q) { const int c = s_wl[q]; run += q < w ? c : 0; U += c; }
        for (int q = 0; q < kpl; ++q) {
            const int i = i0 + q * WAVE;
            const bool hh = is_head(i);
            const uint64_t hm = __ballot(hh);
            if (hh) hpos[run + __popcll(hm & lt)] = (uint32_t)i;
            run += (int)__popcll(hm);
        }
        __syncthreads();
    }
    DIAG_T(3);
    // prefetched path: the sorted gather positions as a compact u32 array (the bags are no
    // longer needed), read 4 at a time by the walk
    uint32_t* gsp = bags;
    if (pf) {
        for (int e = threadIdx.x; e < n; e += FB_TPB) gsp[e] = key_lo(keys[e]);
        __syncthreads();
    }
    // MODE 1: first segment of every row-range slot (dim-split tables span several slots)
    const int64_t nblk = ceil_div(nrows, BLK);
    if (MODE == 1) {
        if (threadIdx.x < SPLIT) s_wl[threadIdx.x] = 0;
        __syncthreads();
        if (dsplit) {
            for (int u = threadIdx.x; u < U; u += FB_TPB) atomicAdd(&s_wl[slot_of_row(key_row(keys[hpos[u]]), nblk)], 1);
            __syncthreads();
            if (threadIdx.x < SPLIT) {
                int run = 0;
                for (int q = 0; q < (int)threadIdx.x; ++q) run += s_wl[q];
                s_ufirst[threadIdx.x] = run;
            }
        } else if (threadIdx.x < SPLIT) {
            s_ufirst[threadIdx.x] = 0;
            s_wl[threadIdx.x] = (int)threadIdx.x == s ? U : 0;
        }
        __syncthreads();
    }
    FOut o;
    o.t = t;
    o.rb = m.row_base[t];
    o.bb = m.blk_base[t];
    o.sbb = m.sblk_base[t];
    o.wide_upkeep = MODE != 1 && !dsplit;  // SGD row split implies > 256 rows
    o.r_pack = (MODE != 1 && a.repack) ? 1.0f / a.pscale[t] : 0.0f;
    o.ufirst = s_ufirst;
    o.cb = s_cb;
    o.nblk = nblk;
    o.q0 = dsplit ? z * LG : 0;
    // per-block aggregation of the SGD hierarchy upkeep (LDS after the stage / rows)
    __shared__ unsigned int s_bgrow[FB_AGG], s_bshr[FB_AGG];
    const int64_t b0s = r0 >> 8, nbs = ((r1 + BLK - 1) >> 8) - b0s;
    const bool agg = o.wide_upkeep && nbs <= FB_AGG;
    o.bgrow = agg ? s_bgrow : nullptr;
    o.bshr = agg ? s_bshr : nullptr;
    o.b0s = b0s;
    if (agg) {
        if (threadIdx.x < FB_AGG) { s_bgrow[threadIdx.x] = 0u; s_bshr[threadIdx.x] = 0u; }
        __syncthreads();
    }
    if (pf)
        fused_segments_lds<LPR, MODE, LG>(a, o, keys, gsp, hpos, U, n, dyl, amax);
    else
        fused_segments_staged<LPR, MODE, LG>(a, o, keys, bags, hpos, U, n, reinterpret_cast<float*>(data),
                                             (int)((FB_LDS - (data - lds)) / 4), src, amax);
    if (agg) {  // one update per block: growth by max (the slot owns the block), shrunk holders flagged
        __syncthreads();
        if (threadIdx.x < nbs) {
            const int64_t blk = b0s + threadIdx.x;
            const float cand = __uint_as_float(s_bgrow[threadIdx.x]);
            const float old_blk = a.blkmax[o.bb + blk];
            const int64_t sb = o.sbb + (blk >> 8);
            if (cand > old_blk) {
                st_wt(a.blkmax + o.bb + blk, cand);
                if (cand > a.sblkmax[sb]) {
                    atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sb, __float_as_uint(cand));
                    if (cand > a.tmax[t]) atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(cand));
                }
            }
            if (s_bshr[threadIdx.x]) {
                flag_set(a.bdirty, o.bb + blk);
                flag_set(a.sdirty, sb);
            }
        }
    }
    DIAG_W(4);
    (void)D;
}

template <int LPR, int MODE>
__global__ void __launch_bounds__(FB_TPB) k_bwd_fused(FArgs a) {
    using FG = FGeom<LPR>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int s_scan[FB_TPB / WAVE + 1];
    __shared__ int s_wl[2 * (FB_TPB / WAVE) + 1];
    __shared__ int s_ufirst[SPLIT];
    __shared__ int64_t s_cb[SPLIT + 1];
    __shared__ float s_red[FB_TPB / WAVE];
    const int k = blockIdx.x, t = k / SPLIT, s = k % SPLIT;
    DIAG_T(0);
    DIAG_C(7);
    // Criteo form with <= 8 bags per thread: the thread's indices are loaded right away, in
    // parallel with the table metadata (no dependent round trip before the gather)
    int64_t pre[8];
    const int per = (a.pool1 && a.B <= (int64_t)FB_TPB * 8) ? (int)((a.B + FB_TPB - 1) / FB_TPB) : 0;
    if (per > 0) {
        const int64_t* ti = a.idx + (int64_t)t * a.B + (int64_t)threadIdx.x * per;
#pragma unroll
        for (int j = 0; j < 8; ++j) pre[j] = (j < per && (int64_t)threadIdx.x * per + j < a.B) ? ti[j] : -1;
    }
    DIAG_W(8);
    const Meta m = make_meta(a.meta, a.T);
    const int64_t nrows = m.num_rows[t];
    const int64_t nblk = ceil_div(nrows, BLK);
    const bool dsplit = MODE == 1 ? nblk < SPLIT : nrows <= BLK;
    const bool masked = MODE == 2 && a.tmask != nullptr && a.tmask[t] == 0;
    int64_t r0 = 0, r1 = nrows;
    if (!dsplit) slot_rows(nrows, s, r0, r1);
    const bool active = !masked && (dsplit ? s < FG::DSPLIT : r0 < r1);
    if (MODE == 1) {
        if (threadIdx.x <= SPLIT) s_cb[threadIdx.x] = a.ws_cap_base[t * SPLIT + threadIdx.x];
        if (threadIdx.x < SPLIT) { s_ufirst[threadIdx.x] = 0; s_wl[threadIdx.x] = 0; }
    }
    __syncthreads();
    float amax = 0.0f;
    if (active) {  // uniform
        if (dsplit)
            fused_slot<LPR, MODE, LPR / FG::DSPLIT>(a, lds, k, t, s, true, s, r0, r1, s_scan, s_wl, s_ufirst, s_cb,
                                                    amax, pre, per);
        else
            fused_slot<LPR, MODE, LPR>(a, lds, k, t, s, false, 0, r0, r1, s_scan, s_wl, s_ufirst, s_cb, amax, pre, per);
    }
    if (MODE == 1) {  // the slot's max|grad| (dim-split: this slice's), and the slot counts
        amax = wave_max(amax);
        if (threadIdx.x % WAVE == 0) s_red[threadIdx.x / WAVE] = amax;
        __syncthreads();
        if (threadIdx.x == 0) {
            float r = 0.0f;
            for (int q = 0; q < FB_TPB / WAVE; ++q) r = fmaxf(r, s_red[q]);
            a.ws_absmax[k] = r;
        }
        if (threadIdx.x < SPLIT && (dsplit ? s == 0 : (int)threadIdx.x == s)) {
            const int64_t cap = s_cb[threadIdx.x + 1] - s_cb[threadIdx.x];
            int c = s_wl[threadIdx.x];
            if (c > cap) { flag_error(a.err, DQRM_ERRF_OVERFLOW); c = (int)cap; }
            a.ws_ucount[t * SPLIT + threadIdx.x] = c;
        }
    }
    DIAG_W(5);
    DIAG_C(15);
    // SGD / local update: the table's last slot workgroup finalizes its |W| hierarchy
    if (MODE != 1 && !a.fin_launch && arrive_last(a.sync + (int64_t)t * DQRM_SYNC_STRIDE, SPLIT))
        finalize_table<true>(m, t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax, LPR * 4, true);
}

// ------------------------------------------------------------------------------------
// K4 SGD for small batches (BASELINE config 3: Kaggle, B = 128): ONE workgroup per table
// owns all of the table's lookups, so duplicate rows, the ordered update chains and the
// |W| hierarchy are resolved inside the workgroup -- no sort, no workspace, no hand-off,
// no finalize. dqrm_emb_bwd_sgd takes it when max_lookups <= min(SG_MAXL, 64 * D/4) and
// B * D <= SG_DY_FLOATS. Same arithmetic and order as k_bwd_fused<LPR, 0>: per row, in
// ascending lookup position j,  W = fma((dy[bag(j)] * s) / s, -lr, W).
//   1. one round trip: the table's indices, every bag's dy slice (STE applied, staged in
//      LDS), the offsets (bag form) and, for a narrow table, its rows' |W| maxima;
//   2. Criteo form: every lookup inserts its row into an LDS hash (row -> bitmask of its
//      positions, one atomicCAS probe chain + one 64-bit atomicOr); the row's owner is its
//      lowest position, and the mask IS its positions in ascending order (no scan, no list).
//      Bag form: one lane group (LPR lanes) per lookup i, the group's lanes compare x_i with
//      disjoint position ranges (one 64-bit match mask each); i owns its row iff no earlier
//      position matches;
//   3. owners load their W row and the old block / superblock / table maxima (one round
//      trip), walk the matches in position order out of LDS, store W (+ INT4 repack);
//   4. |W| hierarchy: growth by atomicMax; a shrunk block-max holder queues its block,
//      re-reduced from rowmax once the workgroup's stores have landed, then (rarely) its
//      superblock, then (more rarely) the table maximum; a narrow table reduces its row
//      maxima in LDS.
// ------------------------------------------------------------------------------------
constexpr int SG_TPB = 512;
constexpr int SG_MAXL = 512;           // lookups per table: at most one per thread
constexpr int SG_DY_FLOATS = 16384;    // dy staging, dynamic LDS (64 KiB)
// lookups per table k_sgd_small takes: one per thread, 64 positions per lane's match mask,
// at most 8 lookups per lane group
__host__ __device__ constexpr int sg_maxl(int lpr) {
    return SG_MAXL < 64 * lpr ? (SG_MAXL < 8 * (SG_TPB / lpr) ? SG_MAXL : 8 * (SG_TPB / lpr))
                              : (64 * lpr < 8 * (SG_TPB / lpr) ? 64 * lpr : 8 * (SG_TPB / lpr));
}

// the Criteo-form row hash of k_sgd_small: 2^sg_hash_log(L) >= 4L slots of {row + 1, [MW]
// 64-bit position masks} after the dy staging in dynamic LDS
__host__ __device__ constexpr int sg_hash_log(int L) {
    int lg = 6;
    while ((1 << lg) < 4 * L) ++lg;  // load <= 1/4: short probe chains
    return lg;
}
#ifndef DQRM_SG_RUN
#define DQRM_SG_RUN 8
#endif
constexpr int SG_RUN = DQRM_SG_RUN;  // positions (dy rows) of an owner's walk in flight
__host__ __device__ constexpr int64_t sg_hash_bytes(int L) {
    return (int64_t)(1 << sg_hash_log(L)) * (4 + 8 * ((L + 63) / 64));
}

template <int LPR, bool FWD>
__global__ void __launch_bounds__(SG_TPB) k_sgd_small(FArgs a) {
    // FWD: after the table's update and |W| maxima (one workgroup holds the whole table, so they
    // are final at its end -- no other workgroup to wait for), the next batch's forward of the
    // table: its rows are this workgroup's own stores or untouched
    constexpr int D = LPR * 4;
    constexpr int G = SG_TPB / LPR;                              // lane groups
    constexpr int MAXL = sg_maxl(LPR);
    constexpr int NPG = (MAXL + G - 1) / G;                      // lookups per lane group (<= 8)
    static_assert(NPG <= 8 && MAXL <= 64 * LPR, "k_sgd_small geometry");
    constexpr int DYF = SG_DY_FLOATS / 4 / SG_TPB;               // dy float4 per thread
    constexpr int NW = SG_TPB / WAVE;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* s_dy = reinterpret_cast<float4*>(lds);               // [B][LPR], STE applied
    __shared__ int32_t s_row[SG_MAXL];                           // local row of lookup j, -1 invalid
    __shared__ int32_t s_bag[SG_MAXL];                           // bag of lookup j (offsets form)
    __shared__ float s_rm[BLK];                                  // narrow table: row maxima
    __shared__ int32_t s_q[SG_MAXL];                             // offsets, then queued blocks
    __shared__ float s_qo[SG_MAXL], s_qso[SG_MAXL];              // their old block / superblock max
    __shared__ int32_t s_sq[SG_MAXL];                            // queued superblocks
    __shared__ float s_sqo[SG_MAXL];                             // ... their old max
    __shared__ float s_red[NW];
    __shared__ int s_n[3];                                       // queue lengths, rescan flag
    const int t = blockIdx.x;
    DIAG_T(0);
    const Meta m = make_meta(a.meta, a.T);
    const int64_t nrows = m.num_rows[t], rb = m.row_base[t], bb = m.blk_base[t], sbb = m.sblk_base[t];
    const bool narrow = nrows <= BLK;
    const int B = (int)a.B;
    const bool p1 = a.pool1 != 0;
    const int64_t ib = p1 ? (int64_t)t * B : a.idx_base[t];
    const int L = p1 ? B : (int)(a.idx_base[t + 1] - ib);
    const bool overflow = L > a.Lc || L > MAXL;  // more lookups than the caller planned for
    const int Lv = overflow ? 0 : L;              // (checked below, after the forward's setup)
    const float s = a.scale[t];
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int gbase = (threadIdx.x % WAVE) - sub;
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    // 1. every independent load of the table in flight together: each lane group's lookups
    //    (its LPR lanes load the same index), the bags' dy slices, offsets, narrow row maxima
    int64_t xr[NPG];
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
        const int i = grp + k * G;
        xr[k] = i < Lv ? a.idx[ib + i] : -1;
    }
    const int64_t o0 = (!p1 && (int)threadIdx.x < B) ? a.off[(int64_t)t * B + threadIdx.x] : 0;
    int64_t nxr[FWD ? NPG : 1];  // the next batch's rows of this lane group's bags (FWD)
    if constexpr (FWD) {
#pragma unroll
        for (int k = 0; k < NPG; ++k) {
            const int i = grp + k * G;
            nxr[k] = i < B ? a.fwd_idx[(int64_t)t * B + i] : -1;
        }
    }
    // the next batch's forward of this table, after its update and maxima (all threads, at
    // every exit below): the final table max, the scale, then the rows and their stores
    __shared__ float s_ftm;
    auto fwd_tail = [&]() {
        if constexpr (FWD) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's stores and atomics landed
            __syncthreads();
            if (threadIdx.x == 0) s_ftm = ld_wt(a.tmax + t);
            __syncthreads();
            const bool refresh = (a.fwd_flags & DQRM_FWD_REFRESH_SCALE) != 0;
            const bool fullp = (a.fwd_flags & DQRM_FWD_FULL_PRECISION) != 0;
            const float sf = fullp ? 1.0f : (refresh ? sym_scale(s_ftm, a.fwd_bits) : a.fwd_scale[t]);
            if (refresh && !fullp && threadIdx.x == 0) a.fwd_scale[t] = sf;
            const float rf = 1.0f / sf;
            const float qlo = -(float)(1 << (a.fwd_bits - 1)), qhi = (float)((1 << (a.fwd_bits - 1)) - 1);
            float4 v[NPG];
#pragma unroll
            for (int k = 0; k < NPG; ++k) {  // every row load issued, clamped, then dropped if invalid
                const int64_t x = nxr[k];
                const bool ok = x >= 0 && x < nrows;
                v[k] = nrows > 0 ? reinterpret_cast<const float4*>(a.W + (rb + (ok ? x : 0)) * D)[sub]
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            float* outt = a.fwd_out + (int64_t)t * a.fwd_ost_t;
#pragma unroll
            for (int k = 0; k < NPG; ++k) {
                const int i = grp + k * G;
                if (i >= B) continue;
                const bool ok = nxr[k] >= 0 && nxr[k] < nrows;
                if (!ok && sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                float4 y = ok ? v[k] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (!fullp) {
                    y.x = fake_quant(y.x, rf, qlo, qhi) * sf;
                    y.y = fake_quant(y.y, rf, qlo, qhi) * sf;
                    y.z = fake_quant(y.z, rf, qlo, qhi) * sf;
                    y.w = fake_quant(y.w, rf, qlo, qhi) * sf;
                }
                reinterpret_cast<float4*>(outt + (int64_t)i * a.fwd_ost_b)[sub] = y;
            }
        }
    };
    if (overflow) {  // the update is skipped and flagged; the next batch's forward still runs
        if (threadIdx.x == 0) flag_error(a.err, DQRM_ERRF_OVERFLOW);
        fwd_tail();
        return;
    }
    const float* dyt = a.dy + (int64_t)t * a.dst_t;
    float4 gv[DYF];
#pragma unroll
    for (int f = 0; f < DYF; ++f) {
        const int q = threadIdx.x + f * SG_TPB;
        if (q < B * LPR) gv[f] = reinterpret_cast<const float4*>(dyt + (int64_t)(q / LPR) * a.dst_b)[q % LPR];
    }
    const float rmv = (narrow && threadIdx.x < nrows) ? a.rowmax[rb + threadIdx.x] : 0.0f;
    const float otm = narrow ? 0.0f : a.tmax[t];
    // 2. as soon as the indices land: every lookup's W row slice and old block / superblock
    //    maxima (speculatively, owner or not), in flight across the LDS staging and the scan
    int32_t xk[NPG];
    float4 w0[NPG];
    float ob[NPG], osb[NPG];
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
        const int i = grp + k * G;
        const bool ok = xr[k] >= 0 && xr[k] < nrows;
        if (i < L && !ok && sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
        xk[k] = (i < L && ok) ? (int32_t)xr[k] : -1;
        ob[k] = 0.0f; osb[k] = 0.0f;
        if (xk[k] >= 0) {
            w0[k] = reinterpret_cast<const float4*>(a.W + (rb + xk[k]) * D)[sub];
            if (!narrow) {
                ob[k] = a.blkmax[bb + (xk[k] >> 8)];
                osb[k] = a.sblkmax[sbb + (xk[k] >> 16)];
            }
        }
        if (i < L && sub == 0) s_row[i] = xk[k];
    }
    DIAG_T(1);
#pragma unroll
    for (int f = 0; f < DYF; ++f) {
        const int q = threadIdx.x + f * SG_TPB;
        if (q < B * LPR) {
            float4 g = gv[f];
            if (a.ste) { g.x = (g.x * s) / s; g.y = (g.y * s) / s; g.z = (g.z * s) / s; g.w = (g.w * s) / s; }
            s_dy[q] = g;
        }
    }
    if (narrow && threadIdx.x < nrows) s_rm[threadIdx.x] = rmv;
    if (threadIdx.x < 3) s_n[threadIdx.x] = 0;
    // Criteo form: the row hash after the dy staging (sized by the host, sg_hash_bytes)
    const int MW = (L + 63) >> 6;               // mask words per row
    const int hs_log = sg_hash_log(L);
    const int HS = 1 << hs_log;
    int32_t* s_hk = reinterpret_cast<int32_t*>(lds + (size_t)B * D * 4);           // row + 1, 0 = empty
    unsigned long long* s_hm = reinterpret_cast<unsigned long long*>(s_hk + HS);  // [HS][MW] positions
    if (p1)
        for (int i = threadIdx.x; i < HS * (1 + 2 * MW); i += SG_TPB) s_hk[i] = 0;
    if (!p1 && (int)threadIdx.x < B) s_q[threadIdx.x] = o0 < 0 ? -1 : (o0 > L ? L + 1 : (int32_t)o0);
    if (!p1)
        for (int j = threadIdx.x; j < L; j += SG_TPB) s_bag[j] = -1;
    __syncthreads();
    if (!p1 && (int)threadIdx.x < B) {  // bag b = lookups [off[b], off[b+1]) (the last ends at L)
        const int b = threadIdx.x;
        int s0 = s_q[b], s1 = b + 1 < B ? s_q[b + 1] : L;
        if (s0 < 0 || s1 > L || s1 < s0 || (b == 0 && s0 != 0)) {  // as visit_slot_lookups; off[0] must be 0
            flag_error(a.err, DQRM_ERRF_OFFSET);
            s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
            s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
        }
        for (int j = s0; j < s1; ++j) s_bag[j] = b;
    }
    if (!p1) __syncthreads();
    DIAG_T(2);
    // 3. duplicates. Criteo form: the row hash (see the header); bag form: lane `sub` of a
    //    group compares positions [sub*ch, sub*ch + ch)
    const int ch = (L + LPR - 1) / LPR;  // <= 64
    const int j0 = sub * ch, j1 = j0 + ch < L ? j0 + ch : L;
    uint64_t mk[NPG];
    int hslot[NPG];
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
        mk[k] = 0ull;
        hslot[k] = -1;
    }
    if (p1) {
#pragma unroll
        for (int k = 0; k < NPG; ++k) {
            const int i = grp + k * G;
            if (sub == 0 && xk[k] >= 0) {
                const int key = xk[k] + 1;
                uint32_t h = ((uint32_t)xk[k] * 2654435761u) >> (32 - hs_log);
                for (;;) {  // linear probing; HS >= 4L, so a free or matching slot exists
                    const int old = atomicCAS(&s_hk[h], 0, key);
                    if (old == 0 || old == key) break;
                    h = (h + 1) & (uint32_t)(HS - 1);
                }
                hslot[k] = (int)h;
                atomicOr(&s_hm[h * MW + (i >> 6)], 1ull << (i & 63));
            }
            hslot[k] = __shfl(hslot[k], gbase, WAVE);
        }
        __syncthreads();
    }
    for (int jb = j0; jb < j1 && !p1; jb += 8) {  // 8 unconditional LDS reads in flight, then the compares
        int32_t v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = s_row[jb + i < j1 ? jb + i : j1 - 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = jb + i < j1 ? v[i] : -1;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int k = 0; k < NPG; ++k) mk[k] |= (uint64_t)(v[i] == xk[k] && v[i] >= 0) << (jb + i - j0);
    }
    bool own[NPG];
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
        const int i = grp + k * G;
        if (p1) {  // the owner is the row's lowest position: the first set bit of its mask
            bool first = false;
            if (hslot[k] >= 0) {
                const unsigned long long* hm = s_hm + hslot[k] * MW;
                int wd = 0;
                unsigned long long m0 = hm[0];
                while (m0 == 0ull && wd + 1 < MW) m0 = hm[++wd];
                first = wd * 64 + __ffsll((long long)m0) - 1 == i;
            }
            own[k] = i < L && xk[k] >= 0 && first;
        } else {
            const int lo = i - j0;  // positions of this lane's range that precede i
            const uint64_t earlier = lo <= 0 ? 0ull : (lo >= 64 ? mk[k] : (mk[k] & ((1ull << lo) - 1ull)));
            own[k] = i < L && xk[k] >= 0 && !(__ballot(earlier != 0ull) & gmask);
        }
    }
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    DIAG_T(3);
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
        if (!own[k]) continue;  // group-uniform
        float4 acc = w0[k];
        if (p1) {  // the row's positions, ascending, straight from its mask: SG_RUN dy rows in flight
            const unsigned long long* hm = s_hm + hslot[k] * MW;
            for (int wd = 0; wd < MW; ++wd) {
                unsigned long long mm = hm[wd];
                while (mm) {
                    int jj[SG_RUN], nv = 0;
#pragma unroll
                    for (int q = 0; q < SG_RUN; ++q) {
                        jj[q] = mm ? wd * 64 + __ffsll((long long)mm) - 1 : (q ? jj[q - 1] : 0);
                        nv += mm ? 1 : 0;
                        mm &= mm - 1;
                    }
                    float4 g[SG_RUN];
#pragma unroll
                    for (int q = 0; q < SG_RUN; ++q) g[q] = s_dy[jj[q] * LPR + sub];
#pragma unroll
                    for (int q = 0; q < SG_RUN; ++q)
                        if (q < nv) acc = seg_op4<OP_FMA>(acc, g[q], a.nlr);
                }
            }
        }
        for (int l = 0; l < LPR && !p1; ++l) {  // the row's positions, ascending
            const uint32_t lo32 = (uint32_t)__shfl((int)(uint32_t)mk[k], gbase + l, WAVE);
            const uint32_t hi32 = (uint32_t)__shfl((int)(uint32_t)(mk[k] >> 32), gbase + l, WAVE);
            uint64_t ml = ((uint64_t)hi32 << 32) | lo32;
            while (ml) {
                const int j = l * ch + __ffsll((long long)ml) - 1;
                ml &= ml - 1;
                const int bag = p1 ? j : s_bag[j];
                if (bag < 0) continue;  // a lookup outside every bag (flagged offsets)
                acc = seg_op4<OP_FMA>(acc, s_dy[bag * LPR + sub], a.nlr);
            }
        }
        const int64_t grow = rb + xk[k];
        reinterpret_cast<float4*>(a.W + grow * D)[sub] = acc;
        if (a.repack) pack4_row(acc, a.packed + grow * (D / 2), sub, r_pack);
        const float orm = group_max<LPR>(abs_max4(w0[k]));
        const float rm = group_max<LPR>(abs_max4(acc));
        if (sub == 0) {
            if (narrow) {
                a.rowmax[grow] = rm;
                s_rm[xk[k]] = rm;
            } else {
                st_wt(a.rowmax + grow, rm);
                const int64_t blk = xk[k] >> 8, sb = blk >> 8;
                if (rm > ob[k]) {
                    atomicMax(reinterpret_cast<unsigned int*>(a.blkmax) + bb + blk, __float_as_uint(rm));
                    if (rm > osb[k]) {
                        atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sbb + sb, __float_as_uint(rm));
                        if (rm > otm) atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(rm));
                    }
                }
                if (orm == ob[k] && rm < orm) {  // held its block's max and shrank
                    const int q = atomicAdd(&s_n[0], 1);
                    s_q[q] = (int32_t)blk;
                    s_qo[q] = ob[k];
                    s_qso[q] = osb[k];
                }
            }
        }
    }
    // 4. the table's maxima (LDS work first; a store round trip only when a block needs its
    //    row maxima re-read)
    __syncthreads();
    DIAG_T(4);
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    if (narrow) {
        float v = threadIdx.x < nrows ? s_rm[threadIdx.x] : 0.0f;
        v = wave_max(v);
        if (lane == 0) s_red[w] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float r = 0.0f;
            for (int q = 0; q < NW; ++q) r = fmaxf(r, s_red[q]);
            a.blkmax[bb] = r;
            a.sblkmax[sbb] = r;
            a.tmax[t] = r;
        }
        fwd_tail();
        DIAG_W(5);
        return;
    }
    const int64_t nblk = ceil_div(nrows, BLK);
    const int nq = s_n[0];
    if (nq == 0) {  // uniform: no block max holder shrank (the common case)
        fwd_tail();
        DIAG_W(5);
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the workgroup's row maxima have landed
    __syncthreads();
    for (int q = w; q < nq; q += NW) {  // a wave per shrunk block: its 256 row maxima
        const int64_t blk = s_q[q];
        float v = 0.0f;
#pragma unroll
        for (int i = 0; i < BLK / WAVE; ++i) {
            const int64_t r = blk * BLK + lane + i * WAVE;
            if (r < nrows) v = fmaxf(v, ld_wt(a.rowmax + rb + r));
        }
        v = wave_max(v);
        if (lane == 0) {
            st_wt(a.blkmax + bb + blk, v);
            if (s_qo[q] == s_qso[q] && v < s_qo[q]) {  // it held its superblock's max
                const int p = atomicAdd(&s_n[1], 1);
                s_sq[p] = (int32_t)(blk >> 8);
                s_sqo[p] = s_qso[q];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nsq = s_n[1];
    for (int q = w; q < nsq; q += NW) {  // a wave per shrunk superblock: its 256 block maxima
        const int64_t sb = s_sq[q];
        float v = 0.0f;
#pragma unroll
        for (int i = 0; i < SBLK_BLOCKS / WAVE; ++i) {
            const int64_t b = sb * SBLK_BLOCKS + lane + i * WAVE;
            if (b < nblk) v = fmaxf(v, ld_wt(a.blkmax + bb + b));
        }
        v = wave_max(v);
        if (lane == 0) {
            st_wt(a.sblkmax + sbb + sb, v);
            if (s_sqo[q] == otm && v < otm) s_n[2] = 1;  // it held the table max
        }
    }
    DIAG_T(6);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (s_n[2]) {  // uniform: rescan the table's superblock maxima
        const int64_t ns = ceil_div(nblk, SBLK_BLOCKS);
        float v = 0.0f;
        for (int64_t k = threadIdx.x; k < ns; k += SG_TPB) v = fmaxf(v, ld_wt(a.sblkmax + sbb + k));
        v = wave_max(v);
        if (lane == 0) s_red[w] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float r = 0.0f;
            for (int q = 0; q < NW; ++q) r = fmaxf(r, s_red[q]);
            a.tmax[t] = r;
        }
    }
    fwd_tail();
    DIAG_W(5);
}

// ------------------------------------------------------------------------------------
// Row-wise PTQ formats of the reference's inference path:
//   prepack   torch.ops.quantized.embedding_bag_{4bit,byte}_prepack
//             (DLRM_Net.quantize_embedding, dlrm_s_pytorch_single_gpu_documentingp.py:689-704)
//   gather    torch.ops.quantized.embedding_bag_{4bit,byte}_rowwise_offsets, mode sum
//             (DLRM_Net.apply_emb, dlrm_s_pytorch_single_gpu_documentingp.py:648-663)
// Row layout (FBGEMM fused row-wise): 4-bit: D/2 nibble bytes (element 2j in the low
// nibble), fp16 scale, fp16 bias; 8-bit: D bytes, f32 scale, f32 bias. A row's scale and
// bias are read once per lookup next to its payload; G = D/8 lanes per row, 8 dims per lane.
// ------------------------------------------------------------------------------------
__host__ __device__ inline int rowwise_row_bytes(int bits, int D) { return bits == 4 ? D / 2 + 4 : D + 8; }

template <int G>
DQRM_INLINE float group_min(float v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, WAVE));
    return v;
}

template <int G>
DQRM_INLINE float group_fmax(float v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
    return v;
}

template <int BITS, int G>
__global__ void __launch_bounds__(256) k_rowwise_prepack(const float* __restrict__ W, int64_t n,
                                                         uint8_t* __restrict__ out) {
    constexpr int D = G * 8;
    constexpr int RB = BITS == 4 ? D / 2 + 4 : D + 8;
    const int lane = threadIdx.x % G;
    const int64_t rows_per_pass = (int64_t)gridDim.x * (256 / G);
    for (int64_t r = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G; r < n; r += rows_per_pass) {
        const float4* src = reinterpret_cast<const float4*>(W + r * D) + lane * 2;
        const float4 a = src[0], b = src[1];
        float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        float mn = x[0], mx = x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) { mn = fminf(mn, x[j]); mx = fmaxf(mx, x[j]); }
        mn = group_min<G>(mn);
        mx = group_fmax<G>(mx);
        uint8_t* orow = out + r * RB;
        if (BITS == 4) {  // FloatOrHalfToFusedNBitRowwiseQuantizedSBHalf, bit_rate 4
            const _Float16 mn16 = (_Float16)mn;  // round-to-nearest-even
            const float mnh = (float)mn16;
            const float range = mx - mnh;
            const float scale = range == 0.0f ? 1.0f : range / 15.0f;
            _Float16 s16 = (_Float16)scale;
            const float sh = (float)s16;
            float inv = sh == 0.0f ? 1.0f : 1.0f / sh;
            if (sh == 0.0f || isinf(inv)) { s16 = (_Float16)1.0f; inv = 1.0f; }
            uint32_t word = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float q = fminf(fmaxf(rintf((x[j] - mnh) * inv), 0.0f), 15.0f);
                word |= (uint32_t)q << (4 * j);
            }
            reinterpret_cast<uint32_t*>(orow)[lane] = word;
            if (lane == 0)
                reinterpret_cast<uint32_t*>(orow + D / 2)[0] =
                    (uint32_t)__builtin_bit_cast(uint16_t, s16) | ((uint32_t)__builtin_bit_cast(uint16_t, mn16) << 16);
        } else {          // FloatToFused8BitRowwiseQuantizedSBFloat
            const float range = mx - mn;
            const float scale = range / 255.0f;
            const float inv = 255.0f / (range + 1e-8f);
            uint2 words = make_uint2(0u, 0u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float q = fminf(fmaxf(rintf((x[j] - mn) * inv), 0.0f), 255.0f);
                if (j < 4) words.x |= (uint32_t)q << (8 * j); else words.y |= (uint32_t)q << (8 * (j - 4));
            }
            reinterpret_cast<uint2*>(orow)[lane] = words;
            if (lane == 0) reinterpret_cast<uint2*>(orow + D)[0] = make_uint2(__float_as_uint(scale), __float_as_uint(mn));
        }
    }
}

// EmbeddingSpMDM(NBit) reference semantics, mode sum: per lookup, in bag order,
//   acc = fma(scale * w, q, acc + bias * w)     (w = per-sample weight, omitted when null)
template <int BITS, int G>
__global__ void __launch_bounds__(256) k_rowwise_bag(const uint8_t* __restrict__ packed, int64_t n,
                                                     const int64_t* __restrict__ idx, int64_t L,
                                                     const int64_t* __restrict__ off, int64_t B,
                                                     const float* __restrict__ psw, int last_offset,
                                                     float* __restrict__ out, uint32_t* __restrict__ err) {
    constexpr int D = G * 8;
    constexpr int RB = BITS == 4 ? D / 2 + 4 : D + 8;
    const int lane = threadIdx.x % G;
    const int64_t bags_per_pass = (int64_t)gridDim.x * (256 / G);
    for (int64_t b = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G; b < B; b += bags_per_pass) {
        int64_t s0 = off[b], s1 = (b + 1 < B || last_offset) ? off[b + 1] : L;
        if (s0 < 0 || s1 > L || s1 < s0) {
            if (lane == 0) flag_error(err, DQRM_ERRF_OFFSET);
            s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
            s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
        }
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.0f;
        for (int64_t i = s0; i < s1; ++i) {
            const int64_t r = idx[i];
            if (r < 0 || r >= n) {
                if (lane == 0) flag_error(err, DQRM_ERRF_INDEX);
                continue;
            }
            const uint8_t* row = packed + r * RB;
            float sc, bi;
            uint32_t w0, w1 = 0;
            if (BITS == 4) {
                const uint32_t sb = *reinterpret_cast<const uint32_t*>(row + D / 2);
                sc = (float)__builtin_bit_cast(_Float16, (uint16_t)(sb & 0xFFFFu));
                bi = (float)__builtin_bit_cast(_Float16, (uint16_t)(sb >> 16));
                w0 = reinterpret_cast<const uint32_t*>(row)[lane];
            } else {
                const uint2 sb = *reinterpret_cast<const uint2*>(row + D);
                sc = __uint_as_float(sb.x);
                bi = __uint_as_float(sb.y);
                const uint2 w = reinterpret_cast<const uint2*>(row)[lane];
                w0 = w.x;
                w1 = w.y;
            }
            if (psw) {
                const float wt = psw[i];
                sc = sc * wt;
                bi = bi * wt;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float q = BITS == 4 ? (float)((w0 >> (4 * j)) & 15u)
                                          : (float)(((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 255u);
                acc[j] = fmaf(sc, q, acc[j] + bi);
            }
        }
        float4* o = reinterpret_cast<float4*>(out + b * D) + lane * 2;
        o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
}

// ------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------
int check_set(const dqrm_table_set* s) {
    if (!s) return set_error(DQRM_E_INVALID, "dqrm: null table set");
    if (s->num_tables <= 0 || s->num_tables > MAX_TABLES)
        return set_error(DQRM_E_INVALID, "dqrm: num_tables out of range (%d)", s->num_tables);
    const int D = s->dim;
    if (D < 4 || D > 256 || (D & 3) || ((D / 4) & (D / 4 - 1)))
        return set_error(DQRM_E_INVALID, "dqrm: dim must be 4*2^k <= 256 (got %d)", D);
    if (!s->W || !s->rowmax || !s->blkmax || !s->sblkmax || !s->tmax || !s->scale || !s->pscale ||
        !s->meta || !s->err || !s->tflags || !s->sdirty || !s->bdirty || !s->sync)
        return set_error(DQRM_E_INVALID, "dqrm: null state pointer");
    if (((uintptr_t)s->W) & 15)
        return set_error(DQRM_E_INVALID, "dqrm: W must be 16-byte aligned");
    return DQRM_OK;
}

// tracked: the preceding kernel raised tmax for every grown row (the flat apply kernels)
// flagged: after the flat apply kernels (k_apply_flat / k_apply_local), which mark the tables
// they flagged (FLAG_WORD) and keep narrow tables' maxima themselves
static bool fin_flagged_skip() {  // DQRM_FIN_FLAGGED=0: finalize every table (A/B)
    static const bool no_skip = [] {
        const char* e = getenv("DQRM_FIN_FLAGGED");
        return e && !strcmp(e, "0");
    }();
    return !no_skip;
}

int launch_finalize(const dqrm_table_set* set, hipStream_t st, bool tracked = false, bool flagged = false) {
    static_assert(BLK <= 1024, "finalize: one thread per row of a narrow table");
    if (!fin_flagged_skip()) flagged = false;
    hipLaunchKernelGGL(k_table_finalize, dim3(set->num_tables), dim3(1024), 0, st, set->W, set->rowmax,
                       set->blkmax, set->sblkmax, set->sdirty, set->bdirty, set->tmax, set->meta, set->num_tables,
                       set->dim, tracked ? 1 : 0, set->sync, flagged ? 1 : 0);
    LAUNCH_CHECK();
    return DQRM_OK;
}

int grid_for(int64_t work_items, int threads, int max_blocks = 2048) {
    int64_t b = (work_items + threads - 1) / threads;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (int)b;
}

// ------------------------------------------------------------------------------------
// Rows rewritten outside libdqrm (torch.optim.SGD stepping on the grad_mode="sparse" COO):
// one lane group per listed slab row recomputes its rowmax (and, repack, its INT4 row with
// the frozen pscale) and flags its block and superblock; the untracked finalize then
// re-reduces exactly those blocks and every table maximum -- for a one-table set (the
// drivers' per-table modules) inside the launch, in its last workgroup (arrival counter in
// sync word 1; row maxima stored write-through), instead of a second launch.
// ------------------------------------------------------------------------------------
struct RcFin {  // the in-launch finalize of a one-table set
    float* blkmax;
    float* sblkmax;
    float* tmax;
    uint32_t* sync;
};
template <int LPR, bool FIN>
__global__ void __launch_bounds__(256) k_rows_changed(const float* __restrict__ W, float* __restrict__ rowmax,
                                                      uint8_t* __restrict__ bdirty, uint8_t* __restrict__ sdirty,
                                                      uint8_t* __restrict__ packed, const float* __restrict__ pscale,
                                                      const int64_t* __restrict__ meta, int T,
                                                      const int64_t* __restrict__ rows, int64_t n, int64_t total,
                                                      uint32_t* __restrict__ err, RcFin fin) {
    constexpr int G = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const Meta m = make_meta(meta, T);
    for (int64_t i = (int64_t)blockIdx.x * G + threadIdx.x / LPR; i < n; i += (int64_t)gridDim.x * G) {
        const int64_t g = rows[i];
        if (g < 0 || g >= total) {
            if (lane == 0) flag_error(err, DQRM_ERRF_INDEX);
            continue;
        }
        const int t = find_table(m.row_base, T, g);
        const int64_t r = g - m.row_base[t];
        const float4 w = reinterpret_cast<const float4*>(W + g * (LPR * 4))[lane];
        float v = abs_max4(w);
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, LPR));
        if (packed) pack_row_int4<LPR>(w, packed, g, lane, 1.0f / pscale[t]);
        if (lane == 0) {
            if (FIN) st_wt(rowmax + g, v);
            else rowmax[g] = v;
            flag_set(bdirty, m.blk_base[t] + r / BLK);
            flag_set(sdirty, m.sblk_base[t] + r / ((int64_t)BLK * SBLK_BLOCKS));
        }
    }
    if constexpr (FIN) {
        if (arrive_last(fin.sync + 1, gridDim.x))
            finalize_table<true>(m, 0, W, rowmax, fin.blkmax, fin.sblkmax, sdirty, bdirty, fin.tmax, LPR * 4, false);
    }
}

// One workgroup, a one-table set: k_rows_changed's work and finalize for the rows an optimizer
// rewrote, then the table's forward with the refreshed scale -- the per-table module's
// external-update sync and its forward as ONE launch (the drivers call 26 modules a step).
template <int LPR>
__global__ void __launch_bounds__(256) k_fwd_after_update(FwdArgs a, float* __restrict__ rowmax,
                                                          uint8_t* __restrict__ bdirty, uint8_t* __restrict__ sdirty,
                                                          float* __restrict__ blkmax, float* __restrict__ sblkmax,
                                                          float* __restrict__ tmax, const int64_t* __restrict__ rows,
                                                          int64_t n, int64_t total) {
    constexpr int G = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const Meta m = make_meta(a.meta, 1);
    for (int64_t i = threadIdx.x / LPR; i < n; i += G) {
        const int64_t g = rows[i];
        if (g < 0 || g >= total) {
            if (lane == 0) flag_error(a.err, DQRM_ERRF_INDEX);
            continue;
        }
        const float4 w = reinterpret_cast<const float4*>(a.W + g * (LPR * 4))[lane];
        float v = abs_max4(w);
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, LPR));
        if (lane == 0) {
            st_wt(rowmax + g, v);
            flag_set(bdirty, g / BLK);
            flag_set(sdirty, g / ((int64_t)BLK * SBLK_BLOCKS));
        }
    }
    // the row maxima and flags landed (write-through) before the finalize reads them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    finalize_table<true>(m, 0, a.W, rowmax, blkmax, sblkmax, sdirty, bdirty, tmax, LPR * 4, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    emb_fwd_table<LPR, 4, true>(a, 0, 0, 1);
}

// ------------------------------------------------------------------------------------
// Per-lookup (uncoalesced) sparse gradient, the form nn.EmbeddingBag(sparse=True) hands to
// autograd (embedding_bag_backward's sparse branch: indices = the input indices, values =
// the bag's gradient row once per lookup, in lookup order): lookup j of table t gets
// rows[j] = row_base[t] + idx[j] and vals[j] = (dy[t, bag(j)] * s_t) / s_t (STE,
// quant_utils.py:349-363). One lane group per bag, its dy row loaded once and stored for
// each of its lookups (coalesced float4 stores), grid (bag chunks, tables).
// ------------------------------------------------------------------------------------
struct LgArgs {
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
    int ste;
    int pool1;
};

template <int LPR>
__global__ void __launch_bounds__(256) k_lookup_grad(LgArgs a) {
    const int t = blockIdx.y;
    constexpr int G = 256 / LPR;
    const int lane = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int D = LPR * 4;
    const float s = a.scale[t];
    const int64_t rowbase = a.meta[t], nrows = a.meta[a.T + t];
    // Criteo form: table t's lookups are idx[t*B, (t+1)*B) -- no idx_base round trip in front of the index loads
    const int64_t ibase = a.pool1 ? (int64_t)t * a.B : a.idx_base[t];
    const int64_t L = a.pool1 ? a.B : a.idx_base[t + 1] - ibase;
    const int64_t B = a.B;
    const int64_t* __restrict__ off = a.off + (int64_t)t * B;
    const bool p1 = a.pool1 && L == B;
    for (int64_t b = (int64_t)blockIdx.x * G + grp; b < B; b += (int64_t)gridDim.x * G) {
        int64_t s0 = p1 ? b : off[b];
        int64_t s1 = p1 ? b + 1 : ((b + 1 < B) ? off[b + 1] : L);
        if (s0 < 0 || s1 > L || s1 < s0 || (b == 0 && s0 != 0)) {  // nn.EmbeddingBag needs off[0] == 0
            if (lane == 0) flag_error(a.err, DQRM_ERRF_OFFSET);
            s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
            s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
            if (b == 0)  // lookups before the first bag: zero rows on the table's row 0, never garbage
                for (int64_t j = 0; j < s0; ++j) {
                    if (lane == 0) a.rows[ibase + j] = rowbase;
                    reinterpret_cast<float4*>(a.vals + (ibase + j) * D)[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
        }
        if (s1 == s0) continue;
        float4 g = reinterpret_cast<const float4*>(a.dy + (int64_t)t * a.dst_t + b * a.dst_b)[lane];
        if (a.ste) { g.x = (g.x * s) / s; g.y = (g.y * s) / s; g.z = (g.z * s) / s; g.w = (g.w * s) / s; }
        for (int64_t j = s0; j < s1; ++j) {
            int64_t r = a.idx[ibase + j];
            float4 v = g;
            if (r < 0 || r >= nrows) {  // flagged; the entry becomes a zero row on the table's row 0
                if (lane == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                r = 0;
                v = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            if (lane == 0) a.rows[ibase + j] = rowbase + r;
            reinterpret_cast<float4*>(a.vals + (ibase + j) * D)[lane] = v;
        }
    }
}

#define DISPATCH_LPR(D, ...)                                  \
    switch ((D) / 4) {                                        \
        case 1: { constexpr int LPR = 1; __VA_ARGS__; } break;  \
        case 2: { constexpr int LPR = 2; __VA_ARGS__; } break;  \
        case 4: { constexpr int LPR = 4; __VA_ARGS__; } break;  \
        case 8: { constexpr int LPR = 8; __VA_ARGS__; } break;  \
        case 16: { constexpr int LPR = 16; __VA_ARGS__; } break; \
        case 32: { constexpr int LPR = 32; __VA_ARGS__; } break; \
        case 64: { constexpr int LPR = 64; __VA_ARGS__; } break; \
        default: return set_error(DQRM_E_INVALID, "dqrm: unsupported dim %d", (int)(D)); \
    }

// allow the per-table kernels more than the default 64 KiB of dynamic LDS (gfx950: 160 KiB/CU)
template <typename K>
int allow_lds(K kernel, size_t bytes) {
    // once per kernel instantiation and size (the attribute is per-function, process-wide;
    // re-setting it on every call costs host time on the launch path)
    // (keyed by the kernel's address: several kernels share one function-pointer type)
    if (bytes <= 65536) return DQRM_OK;
    static std::mutex mu;  // launches may come from several host threads
    std::lock_guard<std::mutex> lock(mu);
    static const void* seen[64];
    static size_t seen_bytes[64];
    static int nseen = 0;
    const void* f = reinterpret_cast<const void*>(kernel);
    for (int i = 0; i < nseen; ++i)
        if (seen[i] == f && seen_bytes[i] >= bytes) return DQRM_OK;
    HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    if (nseen < 64) { seen[nseen] = f; seen_bytes[nseen] = bytes; ++nseen; }
    return DQRM_OK;
}

constexpr int LDS_PER_CU = 160 * 1024;  // gfx950: static + dynamic LDS of one workgroup

// a kernel's static LDS bytes (hipFuncGetAttributes, cached per kernel address)
template <typename K>
size_t static_lds_bytes(K kernel) {
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    static const void* seen[64];
    static size_t seen_bytes[64];
    static int nseen = 0;
    const void* f = reinterpret_cast<const void*>(kernel);
    for (int i = 0; i < nseen; ++i)
        if (seen[i] == f) return seen_bytes[i];
    hipFuncAttributes at{};
    if (hipFuncGetAttributes(&at, f) != hipSuccess) return (size_t)LDS_PER_CU;  // unknown: treat as full
    if (nseen < 64) { seen[nseen] = f; seen_bytes[nseen] = at.sharedSizeBytes; ++nseen; }
    return at.sharedSizeBytes;
}

// dqrm_emb_bwd_coalesce's kernel choice (dqrm_set_coalesce_kernel)
std::atomic<int> g_coalesce_kernel{DQRM_COALESCE_AUTO};

// dqrm_apply_sparse_update's kernel choice: -1 = not yet read from DQRM_APPLY
std::atomic<int> g_apply_kernel{-1};

int apply_kernel_kind() {
    int k = g_apply_kernel.load();
    if (k < 0) {
        const char* e = getenv("DQRM_APPLY");
        k = (e && !strcmp(e, "flat")) ? DQRM_APPLY_FLAT : (e && !strcmp(e, "slot")) ? DQRM_APPLY_SLOT
            : (e && !strcmp(e, "ranges")) ? DQRM_APPLY_RANGES : (e && !strcmp(e, "merge")) ? DQRM_APPLY_MERGE
            : DQRM_APPLY_AUTO;
        int expect = -1;
        g_apply_kernel.compare_exchange_strong(expect, k);
        k = g_apply_kernel.load();
    }
    return k;
}

// Where the |W| hierarchy of an updating kernel is finalized. Measured: the
// flat apply kernels (thousands of short workgroups, latency-bound at full occupancy) are
// faster with their owned-block re-reduction plus a short k_table_finalize launch than with
// the in-launch hand-off (whose code and arrival protocol cost them occupancy and a tail
// round trip per workgroup); the slot kernels (one workgroup per table slot) finalize in
// the launch. DQRM_FINALIZE=launch / inline forces one scheme for every kernel (A/B).
int finalize_mode() {  // 0 auto, 1 launch, 2 inline
    static const int v = [] {
        const char* e = getenv("DQRM_FINALIZE");
        return (e && !strcmp(e, "launch")) ? 1 : (e && !strcmp(e, "inline")) ? 2 : 0;
    }();
    return v;
}
int finalize_launch() { return finalize_mode() == 1 ? 1 : 0; }          // slot kernels
int finalize_launch_flat() { return finalize_mode() == 2 ? 0 : 1; }     // flat apply kernels

// one backward call (K4a + K4b [+ finalize]) on the caller's workspace
struct BwdCall {
    const dqrm_table_set* set;
    const dqrm_batch* batch;
    const float* dy;
    int64_t dst_t, dst_b;
    int ste;
    float lr;
    int repack;
    const int32_t* tmask;
    const int64_t* ws_cap_base;
    int32_t* ws_rows;
    float* ws_vals;
    int32_t* ws_ucount;
    float* ws_absmax;
    void* ws;
    size_t ws_bytes;
    float div = 1.0f;
    // MODE 0: the next batch's forward (dqrm_emb_bwd_sgd_fwd); taken inside k_sgd_small when it
    // runs, else a dqrm_emb_fwd launch after the update
    const dqrm_batch* next = nullptr;
    int fwd_bits = 4;
    uint32_t fwd_flags = 0;
    float* fwd_out = nullptr;
    int64_t fwd_ost_t = 0, fwd_ost_b = 0;
};

int64_t bwd_lookup_cap(const dqrm_batch* batch) { return batch->max_lookups > 0 ? batch->max_lookups : 1; }

bool fused_sgd_fwd_on() {  // DQRM_FUSED_FWD=0: the next batch's forward as its own launch (A/B)
    static const bool off = [] {
        const char* e = getenv("DQRM_FUSED_FWD");
        return e && !strcmp(e, "0");
    }();
    return !off;
}

// Whether k_sgd_small takes an SGD call (MODE 0) of this batch, and whether the next batch's
// forward then runs inside it: returns 0 (k_bwd_fused), 1 (k_sgd_small, forward apart or none),
// 2 (k_sgd_small with the forward in the launch)
int sgd_small_plan(const dqrm_table_set* set, const dqrm_batch* batch, const dqrm_batch* next, uint32_t fwd_flags,
                   size_t* dyn_out) {
    const int D = set->dim;
    const int64_t Lc = bwd_lookup_cap(batch);
    if (!(g_coalesce_kernel.load() == DQRM_COALESCE_AUTO && Lc <= sg_maxl(D / 4) &&
          batch->num_bags * D <= SG_DY_FLOATS && set->total_rows <= 0x7fffffffll))
        return 0;
    // dy staging, then (Criteo form) the row hash; the kernel reads L = B lookups per table.
    // It takes the batch only if that dynamic LDS plus its static LDS fit one CU (else
    // k_bwd_fused, which has no per-batch LDS).
    const bool p1 = (batch->flags & DQRM_BATCH_POOLING_ONE) != 0;
    const size_t dyn = (size_t)batch->num_bags * D * sizeof(float) + (p1 ? (size_t)sg_hash_bytes((int)batch->num_bags) : 0);
    // the next batch's forward inside the launch: a Criteo-form batch of the same size on
    // the exact FP32 rows (the packed INT4 path stays a launch of its own)
    const bool fwd = next && (next->flags & DQRM_BATCH_POOLING_ONE) && next->num_bags == batch->num_bags &&
                     next->max_lookups >= next->num_bags && !(fwd_flags & DQRM_FWD_USE_PACKED) && fused_sgd_fwd_on();
    bool fits = false;
    DISPATCH_LPR(D, {
        fits = dyn + (fwd ? static_lds_bytes(k_sgd_small<LPR, true>) : static_lds_bytes(k_sgd_small<LPR, false>)) <=
               (size_t)LDS_PER_CU;
    });
    if (dyn_out) *dyn_out = dyn;
    return fits ? (fwd ? 2 : 1) : 0;
}

template <int MODE>
int launch_bwd(const BwdCall& c, hipStream_t st, const char* who) {
    const dqrm_table_set* set = c.set;
    const int T = set->num_tables, D = set->dim;
    const int64_t Lc = bwd_lookup_cap(c.batch);
    if (Lc > 0x3fffffffll)
        return set_error(DQRM_E_CAPACITY, "%s: max_lookups %lld too large", who, (long long)Lc);
    if (set->total_rows > 0xffffffffll)
        return set_error(DQRM_E_CAPACITY, "%s: more than 2^32 rows", who);
    FArgs fa{};
    const int64_t need = fused_ws_layout(nullptr, T, Lc, nullptr);
    if (!c.ws || (int64_t)c.ws_bytes < need || (((uintptr_t)c.ws) & 15))
        return set_error(DQRM_E_WORKSPACE, "%s: workspace needs %lld bytes, 16-B aligned (got %zu)", who,
                         (long long)need, c.ws_bytes);
    fused_ws_layout(reinterpret_cast<unsigned char*>(c.ws), T, Lc, &fa);
    fa.W = set->W; fa.packed = set->packed; fa.rowmax = set->rowmax; fa.blkmax = set->blkmax;
    fa.sblkmax = set->sblkmax; fa.tmax = set->tmax; fa.sdirty = set->sdirty; fa.bdirty = set->bdirty;
    fa.sync = set->sync; fa.fin_launch = finalize_launch(); fa.div = c.div;
    fa.scale = set->scale; fa.pscale = set->pscale; fa.meta = set->meta; fa.err = set->err;
    fa.idx = c.batch->idx; fa.off = c.batch->off; fa.idx_base = c.batch->idx_base; fa.B = c.batch->num_bags;
    fa.pool1 = (c.batch->flags & DQRM_BATCH_POOLING_ONE) != 0;
    fa.dy = c.dy; fa.dst_t = c.dst_t; fa.dst_b = c.dst_b; fa.T = T; fa.ste = c.ste; fa.nlr = -c.lr;
    fa.repack = c.repack; fa.tmask = c.tmask; fa.ws_cap_base = c.ws_cap_base; fa.ws_rows = c.ws_rows;
    fa.ws_vals = c.ws_vals; fa.ws_ucount = c.ws_ucount; fa.ws_absmax = c.ws_absmax; fa.Lc = Lc;
    int rc = 0;
    // SGD of a small batch: one workgroup per table, no sort, no hand-off (k_sgd_small)
    if (MODE == 0) {
        size_t dyn = 0;
        const int plan = sgd_small_plan(set, c.batch, c.next, c.fwd_flags, &dyn);
        const bool fwd = plan == 2;
        if (plan > 0) {
            if (fwd) {
                fa.fwd_idx = c.next->idx; fa.fwd_out = c.fwd_out; fa.fwd_ost_t = c.fwd_ost_t; fa.fwd_ost_b = c.fwd_ost_b;
                fa.fwd_scale = set->scale; fa.fwd_bits = c.fwd_bits; fa.fwd_flags = c.fwd_flags;
            }
            DISPATCH_LPR(D, {
                if (fwd) {
                    if ((rc = allow_lds(k_sgd_small<LPR, true>, dyn))) return rc;
                    hipLaunchKernelGGL((k_sgd_small<LPR, true>), dim3(T), dim3(SG_TPB), dyn, st, fa);
                } else {
                    if ((rc = allow_lds(k_sgd_small<LPR, false>, dyn))) return rc;
                    hipLaunchKernelGGL((k_sgd_small<LPR, false>), dim3(T), dim3(SG_TPB), dyn, st, fa);
                }
            });
            LAUNCH_CHECK();
            if (c.next && !fwd)
                return dqrm_emb_fwd(set, c.next, c.fwd_bits, c.fwd_flags, c.fwd_out, c.fwd_ost_t, c.fwd_ost_b, st);
            return DQRM_OK;
        }
    }
    DISPATCH_LPR(D, {
        if ((rc = allow_lds(k_bwd_fused<LPR, MODE>, FB_LDS))) return rc;
        hipLaunchKernelGGL((k_bwd_fused<LPR, MODE>), dim3(T * SPLIT), dim3(FB_TPB), FB_LDS, st, fa);
    });
    LAUNCH_CHECK();  // MODE 0 / 2: the |W| hierarchy is finalized inside the launch
    if (MODE != 1 && fa.fin_launch && (rc = launch_finalize(set, st, true))) return rc;
    if (MODE == 0 && c.next)  // the next batch's forward as its own launch
        return dqrm_emb_fwd(set, c.next, c.fwd_bits, c.fwd_flags, c.fwd_out, c.fwd_ost_t, c.fwd_ost_b, st);
    return DQRM_OK;
}

}  // namespace

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

#ifdef DQRM_DIAG_CLOCK
int dqrm_diag_clock_read(unsigned long long* host, int n) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag_clk), (size_t)n * sizeof(unsigned long long)));
    return DQRM_OK;
}
#endif

const char* dqrm_last_error(void) { return g_last_error; }

// other translation units of libdqrm (dqrm_dense.hip) report through the same slot
__attribute__((visibility("hidden"))) int dqrm_internal_set_error(int code, const char* msg) {
    return set_error(code, "%s", msg);
}
int dqrm_set_coalesce_kernel(int kind) {
    if (kind != DQRM_COALESCE_AUTO && kind != DQRM_COALESCE_GENERAL)
        return set_error(DQRM_E_INVALID, "dqrm_set_coalesce_kernel: unknown kind %d", kind);
    return g_coalesce_kernel.exchange(kind);
}

int dqrm_set_apply_kernel(int kind) {
    if (kind < DQRM_APPLY_AUTO || kind > DQRM_APPLY_MERGE)
        return set_error(DQRM_E_INVALID,
                         "dqrm_set_apply_kernel: kind must be 0 (auto), 1 (flat), 2 (slot), 3 (ranges) or 4 (merge)");
    const int prev = apply_kernel_kind();
    g_apply_kernel.store(kind);
    return prev;
}

int dqrm_abi_version(void) { return DQRM_ABI_VERSION; }

int dqrm_init_uniform(const dqrm_table_set* set, uint64_t seed, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int64_t n4 = set->total_rows * (set->dim / 4);
    hipLaunchKernelGGL(k_init_uniform, dim3(grid_for(n4, 256, 8192)), dim3(256), 0, st, set->W,
                       set->meta, set->num_tables, set->dim, set->total_rows, seed);
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_refresh_absmax(const dqrm_table_set* set, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int D = set->dim;
    DISPATCH_LPR(D, {
        hipLaunchKernelGGL(k_rowmax_all<LPR>, dim3(grid_for(set->total_rows * LPR, 256, 8192)), dim3(256), 0,
                           st, set->W, set->rowmax, set->total_rows);
    });
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_level_max, dim3(grid_for(set->total_blocks * WAVE, 256, 8192)), dim3(256), 0, st,
                       set->rowmax, set->blkmax, set->meta, set->num_tables, 1, set->total_blocks);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_level_max, dim3(grid_for(set->total_sblocks * WAVE, 256, 8192)), dim3(256), 0, st,
                       set->blkmax, set->sblkmax, set->meta, set->num_tables, 2, set->total_sblocks);
    LAUNCH_CHECK();
    HIP_TRY(hipMemsetAsync(set->sdirty, 0, (size_t)set->total_sblocks, st));
    HIP_TRY(hipMemsetAsync(set->bdirty, 0, (size_t)set->total_blocks, st));
    HIP_TRY(hipMemsetAsync(set->sync, 0, (size_t)set->num_tables * DQRM_SYNC_STRIDE * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_table_max, dim3(set->num_tables), dim3(256), 0, st, set->sblkmax, set->tmax,
                       set->meta, set->num_tables);
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_refresh_scale_and_pack(const dqrm_table_set* set, int bits, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if (bits < 2 || bits > 16) return set_error(DQRM_E_INVALID, "%s: bits %d unsupported", "refresh", bits);
    if (set->packed && bits != 4)
        return set_error(DQRM_E_INVALID, "%s: packed rows need bits == 4 (got %d)", "refresh", bits);
    hipStream_t st = (hipStream_t)stream;
    const int T = set->num_tables;
    hipLaunchKernelGGL(k_refresh_scale, dim3((T + 255) / 256), dim3(256), 0, st, set->tmax, set->scale,
                       set->pscale, set->tflags, T, bits, set->packed != nullptr);
    LAUNCH_CHECK();
    if (set->packed) {
        const int D = set->dim;
        DISPATCH_LPR(D, {
            hipLaunchKernelGGL(k_repack_flagged<LPR>, dim3(grid_for(set->total_rows * LPR, 256, 8192)),
                               dim3(256), 0, st, set->W, set->packed, set->scale, set->tflags, set->meta,
                               T, set->total_rows);
        });
        LAUNCH_CHECK();
    }
    return DQRM_OK;
}

// the forward's argument checks and kernel arguments (shared by the two forward entry points)
static int fwd_args(const dqrm_table_set* set, const dqrm_batch* batch, int bits, uint32_t flags, float* out,
                    int64_t out_stride_t, int64_t out_stride_b, const char* who, FwdArgs* a) {
    int rc = check_set(set);
    if (rc) return rc;
    if (!batch || !batch->idx || !batch->off || !batch->idx_base || !out)
        return set_error(DQRM_E_INVALID, "%s: null batch/out pointer", who);
    if (!(flags & DQRM_FWD_FULL_PRECISION) && (bits < 2 || bits > 16))
        return set_error(DQRM_E_INVALID, "%s: embedding_bit %d unsupported", who, bits);
    if ((flags & DQRM_FWD_USE_PACKED) && (!set->packed || bits != 4))
        return set_error(DQRM_E_INVALID, "%s: packed path needs packed rows and bits == 4", who);
    if ((((uintptr_t)out) & 15) || (out_stride_t & 3) || (out_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: out must be 16-B aligned with strides %% 4 == 0", who);
    a->W = set->W; a->packed = set->packed; a->tmax = set->tmax; a->scale = set->scale;
    a->meta = set->meta; a->err = set->err;
    a->idx = batch->idx; a->off = batch->off; a->idx_base = batch->idx_base;
    a->pool1 = (batch->flags & DQRM_BATCH_POOLING_ONE) != 0;
    a->out = out; a->B = batch->num_bags; a->ost_t = out_stride_t; a->ost_b = out_stride_b;
    a->T = set->num_tables; a->bits = bits; a->flags = flags;
    return DQRM_OK;
}

int dqrm_emb_fwd(const dqrm_table_set* set, const dqrm_batch* batch, int bits, uint32_t flags,
                 float* out, int64_t out_stride_t, int64_t out_stride_b, void* stream) {
    FwdArgs a;
    int rc = fwd_args(set, batch, bits, flags, out, out_stride_t, out_stride_b, "dqrm_emb_fwd", &a);
    if (rc) return rc;
    if (batch->num_bags <= 0) return DQRM_OK;
    hipStream_t st = (hipStream_t)stream;
    const int D = set->dim;
    const bool packed_path = (flags & DQRM_FWD_USE_PACKED) && !(flags & DQRM_FWD_FULL_PRECISION) && D >= 8;
    if (packed_path) {
        int64_t bx = (a.B + 255) / 256;
        const int64_t cap = (16384 + a.T - 1) / a.T;
        if (bx > cap) bx = cap;
        const bool nt = (flags & DQRM_FWD_NT_STORE) != 0;
        DISPATCH_LPR(D, {
            if constexpr (LPR >= 2) {
                if (nt)
                    hipLaunchKernelGGL((k_emb_fwd_packed<LPR, true>), dim3((unsigned)bx, (unsigned)a.T), dim3(256), 0, st, a);
                else
                    hipLaunchKernelGGL((k_emb_fwd_packed<LPR, false>), dim3((unsigned)bx, (unsigned)a.T), dim3(256), 0, st, a);
            }
        });
        LAUNCH_CHECK();
        return DQRM_OK;
    }
    DISPATCH_LPR(D, {
        constexpr int UNR = 4;
        constexpr int BAGS_PER_WG = (256 / LPR) * UNR;
        int64_t bx = (a.B + BAGS_PER_WG - 1) / BAGS_PER_WG;
        const int64_t cap = (8192 + a.T - 1) / a.T;  // ~8k workgroups in total, grid-stride beyond
        if (bx > cap) bx = cap;
        hipLaunchKernelGGL((k_emb_fwd<LPR, UNR>), dim3((unsigned)bx, (unsigned)a.T), dim3(256), 0, st, a);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_emb_fwd_after_update(const dqrm_table_set* set, const dqrm_batch* batch, int bits, uint32_t flags,
                              float* out, int64_t out_stride_t, int64_t out_stride_b, const int64_t* rows,
                              int64_t n, int repack_bits, void* stream) {
    FwdArgs a;
    int rc = fwd_args(set, batch, bits, flags, out, out_stride_t, out_stride_b, "dqrm_emb_fwd_after_update", &a);
    if (rc) return rc;
    if (n < 0 || (n > 0 && !rows))
        return set_error(DQRM_E_INVALID, "%s: bad row list", "dqrm_emb_fwd_after_update");
    // one workgroup does it all: a one-table set, a small batch and row list, FP32 rows
    const int lpr = set->dim / 4;
    const bool one = n > 0 && n <= 4096 && set->num_tables == 1 && repack_bits == 0 &&
                     !(flags & DQRM_FWD_USE_PACKED) && batch->num_bags > 0 &&
                     batch->num_bags * (int64_t)lpr <= 16 * 256 && finalize_mode() != 1;
    if (!one) {  // the two calls
        if (n > 0 && (rc = dqrm_rows_changed(set, rows, n, repack_bits, stream))) return rc;
        return dqrm_emb_fwd(set, batch, bits, flags, out, out_stride_t, out_stride_b, stream);
    }
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_LPR(set->dim, {
        hipLaunchKernelGGL((k_fwd_after_update<LPR>), dim3(1), dim3(256), 0, st, a, set->rowmax, set->bdirty,
                           set->sdirty, set->blkmax, set->sblkmax, set->tmax, rows, n, set->total_rows);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

static int check_batch(const dqrm_batch* batch, const char* who) {
    if (!batch || !batch->idx || !batch->off || !batch->idx_base)
        return set_error(DQRM_E_INVALID, "%s: null batch pointer", who);
    if (batch->num_bags > 0xFFFFFFFFll)
        return set_error(DQRM_E_CAPACITY, "%s: more than 2^32 bags", who);
    return DQRM_OK;
}

size_t dqrm_bwd_workspace_bytes(int num_tables, int64_t max_lookups) {
    if (num_tables <= 0 || num_tables > MAX_TABLES || max_lookups < 0) return 0;
    return (size_t)fused_ws_layout(nullptr, num_tables, max_lookups > 0 ? max_lookups : 1, nullptr);
}

int dqrm_emb_bwd_sgd(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                     int64_t dy_stride_t, int64_t dy_stride_b, int ste, float lr, int repack_bits,
                     void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_sgd"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0", "dqrm_emb_bwd_sgd");
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_emb_bwd_sgd", repack_bits);
    if (batch->num_bags <= 0) return DQRM_OK;
    BwdCall c{};
    c.set = set; c.batch = batch; c.dy = dy; c.dst_t = dy_stride_t; c.dst_b = dy_stride_b; c.ste = ste;
    c.lr = lr; c.repack = repack_bits == 4; c.ws = workspace; c.ws_bytes = workspace_bytes;
    return launch_bwd<0>(c, (hipStream_t)stream, "dqrm_emb_bwd_sgd");
}

int dqrm_emb_bwd_sgd_fwd(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                         int64_t dy_stride_t, int64_t dy_stride_b, int ste, float lr, int repack_bits,
                         void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                         uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_sgd_fwd"))) return rc;
    FwdArgs fa;  // the forward's arguments, validated as dqrm_emb_fwd validates them
    if ((rc = fwd_args(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b, "dqrm_emb_bwd_sgd_fwd", &fa)))
        return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0", "dqrm_emb_bwd_sgd_fwd");
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_emb_bwd_sgd_fwd",
                         repack_bits);
    if (batch->num_bags <= 0)
        return dqrm_emb_fwd(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b, stream);
    BwdCall c{};
    c.set = set; c.batch = batch; c.dy = dy; c.dst_t = dy_stride_t; c.dst_b = dy_stride_b; c.ste = ste;
    c.lr = lr; c.repack = repack_bits == 4; c.ws = workspace; c.ws_bytes = workspace_bytes;
    c.next = next; c.fwd_bits = fwd_bits; c.fwd_flags = fwd_flags; c.fwd_out = out;
    c.fwd_ost_t = out_stride_t; c.fwd_ost_b = out_stride_b;
    return launch_bwd<0>(c, (hipStream_t)stream, "dqrm_emb_bwd_sgd_fwd");
}

int dqrm_rows_changed(const dqrm_table_set* set, const int64_t* rows, int64_t n, int repack_bits, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if (n < 0 || (n > 0 && !rows)) return set_error(DQRM_E_INVALID, "%s: bad row list", "dqrm_rows_changed");
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_rows_changed",
                         repack_bits);
    if (n == 0) return DQRM_OK;
    hipStream_t st = (hipStream_t)stream;
    uint8_t* pk = repack_bits == 4 ? set->packed : nullptr;
    // a one-table set finalizes inside the launch (its last workgroup); larger sets launch
    // the per-table finalize
    const bool fin = set->num_tables == 1 && finalize_mode() != 1;
    const RcFin rf{set->blkmax, set->sblkmax, set->tmax, set->sync};
    DISPATCH_LPR(set->dim, {
        constexpr int G = 256 / LPR;
        if (fin)
            hipLaunchKernelGGL((k_rows_changed<LPR, true>), dim3(grid_for(n, G, 4096)), dim3(256), 0, st, set->W,
                               set->rowmax, set->bdirty, set->sdirty, pk, set->pscale, set->meta, set->num_tables,
                               rows, n, set->total_rows, (uint32_t*)set->err, rf);
        else
            hipLaunchKernelGGL((k_rows_changed<LPR, false>), dim3(grid_for(n, G, 4096)), dim3(256), 0, st, set->W,
                               set->rowmax, set->bdirty, set->sdirty, pk, set->pscale, set->meta, set->num_tables,
                               rows, n, set->total_rows, (uint32_t*)set->err, rf);
    });
    LAUNCH_CHECK();
    return fin ? DQRM_OK : launch_finalize(set, st, false);
}

int dqrm_emb_bwd_lookup_grad(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                             int64_t dy_stride_t, int64_t dy_stride_b, int ste, int64_t* rows, float* vals,
                             void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_lookup_grad"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0",
                         "dqrm_emb_bwd_lookup_grad");
    if (!rows || !vals || (((uintptr_t)vals) & 15))
        return set_error(DQRM_E_INVALID, "%s: rows / 16-B aligned vals required", "dqrm_emb_bwd_lookup_grad");
    if (batch->num_bags <= 0) return DQRM_OK;
    LgArgs a;
    a.meta = set->meta; a.scale = set->scale; a.err = (uint32_t*)set->err; a.idx = batch->idx; a.off = batch->off;
    a.idx_base = batch->idx_base; a.dy = dy; a.dst_t = dy_stride_t; a.dst_b = dy_stride_b; a.B = batch->num_bags;
    a.rows = rows; a.vals = vals; a.T = set->num_tables; a.ste = ste;
    a.pool1 = (batch->flags & DQRM_BATCH_POOLING_ONE) != 0;
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_LPR(set->dim, {
        constexpr int G = 256 / LPR;
        int64_t gx = (a.B + G - 1) / G;
        if (gx > 4096) gx = 4096;
        hipLaunchKernelGGL(k_lookup_grad<LPR>, dim3((unsigned)gx, (unsigned)a.T), dim3(256), 0, st, a);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

int64_t dqrm_coalesce_slot_caps(const int64_t* num_rows_host, int num_tables, int64_t max_lookups,
                                int64_t* ws_cap_base_host) {
    if (!num_rows_host || !ws_cap_base_host || num_tables <= 0 || max_lookups < 0)
        return set_error(DQRM_E_INVALID, "dqrm_coalesce_slot_caps: bad arguments");
    int64_t run = 0;
    for (int t = 0; t < num_tables; ++t) {
        for (int s = 0; s < SPLIT; ++s) {
            const int64_t nblk = (num_rows_host[t] + BLK - 1) / BLK;
            const int64_t b0 = nblk * s / SPLIT, b1 = nblk * (s + 1) / SPLIT;
            const int64_t r1 = b1 * BLK < num_rows_host[t] ? b1 * BLK : num_rows_host[t];
            int64_t rows = r1 - b0 * BLK;
            if (rows < 0) rows = 0;
            const int64_t lim = max_lookups;  // distinct rows <= lookups: never exceeded
            ws_cap_base_host[t * SPLIT + s] = run;
            run += rows < lim ? rows : lim;
        }
    }
    ws_cap_base_host[num_tables * SPLIT] = run;
    return run;
}

int dqrm_emb_bwd_coalesce(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                          int64_t dy_stride_t, int64_t dy_stride_b, int ste, const int64_t* ws_cap_base,
                          int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount, float* ws_absmax,
                          void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_coalesce"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0", "dqrm_emb_bwd_coalesce");
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !ws_absmax || (((uintptr_t)ws_vals) & 15))
        return set_error(DQRM_E_INVALID, "%s: null/unaligned workspace", "dqrm_emb_bwd_coalesce");
    BwdCall c{};
    c.set = set; c.batch = batch; c.dy = dy; c.dst_t = dy_stride_t; c.dst_b = dy_stride_b; c.ste = ste;
    c.ws_cap_base = ws_cap_base; c.ws_rows = ws_rows; c.ws_vals = ws_vals; c.ws_ucount = ws_ucount;
    c.ws_absmax = ws_absmax; c.ws = workspace; c.ws_bytes = workspace_bytes;
    if (g_coalesce_kernel.load() == DQRM_COALESCE_AUTO && (batch->flags & DQRM_BATCH_POOLING_ONE) &&
        batch->num_bags <= dqrm_internal::kCoalesceMaxB && batch->max_lookups >= batch->num_bags &&
        set->total_rows <= 0xffffffffll) {
        dqrm_internal::CoalesceArgs ca{};
        ca.meta = set->meta; ca.T = set->num_tables; ca.D = set->dim; ca.B = batch->num_bags; ca.idx = batch->idx;
        ca.dy = dy; ca.dst_t = dy_stride_t; ca.dst_b = dy_stride_b; ca.scale = set->scale; ca.ste = ste;
        ca.err = set->err; ca.ws_cap_base = ws_cap_base; ca.ws_rows = ws_rows; ca.ws_vals = ws_vals;
        ca.ws_ucount = ws_ucount; ca.ws_absmax = ws_absmax;
        const hipError_t e = dqrm_internal::launch_coalesce_pool1(ca, nullptr, (hipStream_t)stream);
        if (e != hipSuccess)
            return set_error(DQRM_E_HIP, "dqrm_emb_bwd_coalesce: launch failed: %s (%d)", hipGetErrorString(e), (int)e);
        return DQRM_OK;
    }
    return launch_bwd<1>(c, (hipStream_t)stream, "dqrm_emb_bwd_coalesce");
}

int dqrm_emb_bwd_coalesce_scaled(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                                 int64_t dy_stride_t, int64_t dy_stride_b, int ste, int divisor,
                                 const int64_t* ws_cap_base, int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount,
                                 float* ws_absmax, void* workspace, size_t workspace_bytes, void* stream) {
    if (divisor < 1) return set_error(DQRM_E_INVALID, "%s: divisor must be >= 1", "dqrm_emb_bwd_coalesce_scaled");
    if (divisor == 1)
        return dqrm_emb_bwd_coalesce(set, batch, dy, dy_stride_t, dy_stride_b, ste, ws_cap_base, ws_rows, ws_vals,
                                     ws_ucount, ws_absmax, workspace, workspace_bytes, stream);
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_coalesce_scaled"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0",
                         "dqrm_emb_bwd_coalesce_scaled");
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !ws_absmax || (((uintptr_t)ws_vals) & 15))
        return set_error(DQRM_E_INVALID, "%s: null/unaligned workspace", "dqrm_emb_bwd_coalesce_scaled");
    BwdCall c{};
    c.set = set; c.batch = batch; c.dy = dy; c.dst_t = dy_stride_t; c.dst_b = dy_stride_b; c.ste = ste;
    c.ws_cap_base = ws_cap_base; c.ws_rows = ws_rows; c.ws_vals = ws_vals; c.ws_ucount = ws_ucount;
    c.ws_absmax = ws_absmax; c.ws = workspace; c.ws_bytes = workspace_bytes; c.div = (float)divisor;
    return launch_bwd<1>(c, (hipStream_t)stream, "dqrm_emb_bwd_coalesce_scaled");  // the general kernel
}

size_t dqrm_payload_bytes(int num_tables, int64_t cap_total, int dim, int grad_bits) {
    return (size_t)payload_layout(num_tables, cap_total, dim, grad_bits).bytes;
}

int dqrm_grad_quant_pack_strided(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                                 const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                                 const float* absmax_all, int64_t absmax_pitch, int num_ranks, int grad_bits,
                                 const int64_t* cap_base, int64_t cap_total, float* s_avg, void* payload,
                                 void* stream) {
    if (num_tables <= 0 || num_tables > MAX_TABLES || num_ranks <= 0 || num_ranks > 64)
        return set_error(DQRM_E_INVALID, "%s: bad num_tables/num_ranks", "dqrm_grad_quant_pack");
    if (!(grad_bits == 32 || (grad_bits >= 2 && grad_bits <= 16)))
        return set_error(DQRM_E_INVALID, "%s: grad bits %d unsupported", "dqrm_grad_quant_pack", grad_bits);
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !cap_base || !payload ||
        (grad_bits != 32 && (!absmax_all || !s_avg)))
        return set_error(DQRM_E_INVALID, "%s: null pointer", "dqrm_grad_quant_pack");
    if (num_ranks > 1 && absmax_pitch < (int64_t)num_tables * SPLIT)
        return set_error(DQRM_E_INVALID, "%s: absmax pitch %lld < %d", "dqrm_grad_quant_pack",
                         (long long)absmax_pitch, num_tables * SPLIT);
    if (((uintptr_t)payload) & 15)
        return set_error(DQRM_E_INVALID, "%s: payload must be 16-B aligned", "dqrm_grad_quant_pack");
    hipStream_t st = (hipStream_t)stream;
    static const bool legacy = [] {  // DQRM_QPACK=legacy: the one-workgroup-per-slot kernel (A/B)
        const char* e = getenv("DQRM_QPACK");
        return e && !strcmp(e, "legacy");
    }();
    if (!legacy) {
        dqrm_internal::QuantPackArgs q{num_tables, dim, ws_cap_base, ws_rows, ws_vals, ws_ucount, absmax_all,
                                       absmax_pitch, num_ranks, grad_bits, cap_base, cap_total, s_avg,
                                       (unsigned char*)payload};
        HIP_TRY(dqrm_internal::launch_quant_pack(q, st));
        return DQRM_OK;
    }
    DISPATCH_LPR(dim, {
        hipLaunchKernelGGL(k_quant_pack<LPR>, dim3(num_tables * SPLIT), dim3(512), 0, st,
                           num_tables, ws_cap_base, ws_cap_total, ws_rows, ws_vals, ws_ucount, absmax_all,
                           absmax_pitch, num_ranks, grad_bits, cap_base, cap_total, s_avg, (unsigned char*)payload,
                           (const int32_t*)nullptr, (const float*)nullptr);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_grad_quant_pack(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                         const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                         const float* absmax_all, int num_ranks, int grad_bits, const int64_t* cap_base,
                         int64_t cap_total, float* s_avg, void* payload, void* stream) {
    return dqrm_grad_quant_pack_strided(num_tables, dim, ws_cap_base, ws_cap_total, ws_rows, ws_vals, ws_ucount,
                                        absmax_all, (int64_t)num_tables * SPLIT, num_ranks, grad_bits, cap_base,
                                        cap_total, s_avg, payload, stream);
}

int dqrm_grad_quant_pack_ranked(int num_tables, int dim, const int64_t* ws_cap_base, int64_t ws_cap_total,
                                const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                                const int32_t* table_bits, const float* table_scale, const int64_t* cap_base,
                                int64_t cap_total, void* payload, void* stream) {
    if (num_tables <= 0 || num_tables > MAX_TABLES)
        return set_error(DQRM_E_INVALID, "%s: bad num_tables", "dqrm_grad_quant_pack_ranked");
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !table_bits || !table_scale || !cap_base || !payload)
        return set_error(DQRM_E_INVALID, "%s: null pointer", "dqrm_grad_quant_pack_ranked");
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_LPR(dim, {
        hipLaunchKernelGGL(k_quant_pack<LPR>, dim3(num_tables * SPLIT), dim3(512), 0, st,
                           num_tables, ws_cap_base, ws_cap_total, ws_rows, ws_vals, ws_ucount,
                           (const float*)nullptr, (int64_t)0, 1, 8, cap_base, cap_total, (float*)nullptr,
                           (unsigned char*)payload, table_bits, table_scale);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_emb_local_update(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                          int64_t dy_stride_t, int64_t dy_stride_b, int ste, float lr, const int32_t* table_mask,
                          int repack_bits, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_local_update"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0", "dqrm_emb_local_update");
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_emb_local_update", repack_bits);
    if (batch->num_bags <= 0) return DQRM_OK;
    BwdCall c{};
    c.set = set; c.batch = batch; c.dy = dy; c.dst_t = dy_stride_t; c.dst_b = dy_stride_b; c.ste = ste;
    c.lr = lr; c.repack = repack_bits == 4; c.tmask = table_mask; c.ws = workspace; c.ws_bytes = workspace_bytes;
    return launch_bwd<2>(c, (hipStream_t)stream, "dqrm_emb_local_update");
}

// recover the per-rank batch B from cap_total = sum_t min(B, n_t) (host row counts), -1 without them
static int64_t recover_batch(const dqrm_table_set* set, int64_t cap_total) {
    const int64_t* nr = set->num_rows_host;
    if (!nr) return -1;
    int64_t lo = 0, hi = 0;
    for (int t = 0; t < set->num_tables; ++t) hi = nr[t] > hi ? nr[t] : hi;
    while (lo < hi) {  // smallest B with sum_t min(B, n_t) >= cap_total
        const int64_t mid = (lo + hi) / 2;
        int64_t c = 0;
        for (int t = 0; t < set->num_tables; ++t) c += nr[t] < mid ? nr[t] : mid;
        if (c < cap_total) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// k_apply_pos: entry chunks per (table, rank) -- one pass of 4 entries per lane group covers the
// largest table's capacity min(B, n_t) -- at most 32768 workgroups
static int merge_apply_gx(const dqrm_table_set* set, int64_t cap_total, int num_ranks, int D) {
    const int64_t per = (256 / (D / 4)) * 4;  // entries per workgroup: (lane groups) x AP_INFL
    const int64_t B = recover_batch(set, cap_total);
    const int64_t cmax = B >= 0 ? B : cap_total;
    int64_t gx = (cmax + per - 1) / per;
    const int64_t lim = (32768 + (int64_t)set->num_tables * num_ranks - 1) / ((int64_t)set->num_tables * num_ranks);
    gx = gx > lim ? lim : gx;
    return (int)(gx < 1 ? 1 : gx);
}

// Chunks per row-range slot of each table for k_apply_merge: about DQRM_MERGE_KEYS (default 256)
// payload entries of all ranks per workgroup, from the table's payload capacity min(B, n_t)
// (B recovered from cap_total = sum_t min(B, n_t) and the host row counts; without those, an
// even split), at most the slot's blocks (chunks are block-aligned) and at most 64.
static void merge_plan(const dqrm_table_set* set, int64_t cap_total, int N, int* kt, int* kbase) {
    static const int64_t target = [] {
        const char* e = getenv("DQRM_MERGE_KEYS");
        const long v = e ? atol(e) : 256;
        return (int64_t)(v > 0 ? v : 256);
    }();
    const int T = set->num_tables;
    const int64_t* nr = set->num_rows_host;
    int64_t B = -1;
    if (nr) {  // smallest B with sum_t min(B, n_t) >= cap_total
        int64_t lo = 0, hi = 0;
        for (int t = 0; t < T; ++t) hi = nr[t] > hi ? nr[t] : hi;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            int64_t c = 0;
            for (int t = 0; t < T; ++t) c += nr[t] < mid ? nr[t] : mid;
            if (c < cap_total) lo = mid + 1; else hi = mid;
        }
        B = lo;
    }
    kbase[0] = 0;
    for (int t = 0; t < T; ++t) {
        const int64_t cap_t = B >= 0 ? (nr[t] < B ? nr[t] : B) : (cap_total + T - 1) / T;
        int64_t K = ((int64_t)N * cap_t + SPLIT * target - 1) / (SPLIT * target);
        if (nr) {
            const int64_t blocks_per_slot = ((nr[t] + BLK - 1) / BLK + SPLIT - 1) / SPLIT;
            K = K < blocks_per_slot ? K : blocks_per_slot;
        }
        K = K < 1 ? 1 : (K > 64 ? 64 : K);
        kt[t] = (int)K;
        kbase[t + 1] = kbase[t] + SPLIT * (int)K;
    }
}

static int fwd_args(const dqrm_table_set* set, const dqrm_batch* batch, int bits, uint32_t flags, float* out,
                    int64_t out_stride_t, int64_t out_stride_b, const char* who, FwdArgs* a);

// the flat apply's finalize launch together with the next forward (k_finalize_fwd): the exact
// FP32-row forward (the INT4 packed gather stays a launch of its own); DQRM_FIN_FWD=0 turns it off
static bool finfwd_fits(const dqrm_table_set* set, const dqrm_batch* next, uint32_t flags) {
    static const bool off = [] {
        const char* e = getenv("DQRM_FIN_FWD");
        return e && !strcmp(e, "0");
    }();
    const bool packed_path = (flags & DQRM_FWD_USE_PACKED) && !(flags & DQRM_FWD_FULL_PRECISION) && set->dim >= 8;
    return !off && next && next->num_bags > 0 && !packed_path;
}

static int launch_finalize_fwd(const dqrm_table_set* set, FwdArgs fa, hipStream_t st) {
    static const uint32_t spin = [] {  // DQRM_GATE_SPIN: gate polls before a forward flags a stall
        const char* e = getenv("DQRM_GATE_SPIN");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 20);
    }();
    fa.sync = set->sync;
    fa.spin = spin;
    FinArgs f{set->W, set->rowmax, set->blkmax, set->sblkmax, set->sdirty, set->bdirty, set->tmax, set->dim,
              1, fin_flagged_skip() ? 1 : 0};
    DISPATCH_LPR(set->dim, {
        constexpr int UNR = 4;
        constexpr int BAGS_PER_WG = (FINFWD_TPB / LPR) * UNR;
        int64_t bx = (fa.B + BAGS_PER_WG - 1) / BAGS_PER_WG;
        const int64_t cap = (2048 + fa.T - 1) / fa.T;  // ~2k forward workgroups of 1024 threads, grid-stride beyond
        if (bx > cap) bx = cap;
        const int64_t grid = (int64_t)fa.T * (1 + bx);
        hipLaunchKernelGGL((k_finalize_fwd<LPR, UNR>), dim3((unsigned)grid), dim3(FINFWD_TPB), 0, st, fa, f, (int)bx);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

// the apply's kernel choice: the merge kernels (with the next batch's forward in the update's
// launch when nf is given) when DQRM_APPLY=merge / dqrm_set_apply_kernel(DQRM_APPLY_MERGE) and
// the positions workspace is given (N = 1 needs none). Not AUTO: measured on the TB shape
// (profiles/r6_apply_ranks_*.txt) it is not faster than the flat kernel + finalize launch at
// N = 1..8 (2048 per rank: 20.6 / 53.4 / 75.8 / 143 us vs 15.4 / 39.4 / 68.0 / 138.8 us).
static bool apply_uses_merge(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t ws_bytes) {
    const int kind = apply_kernel_kind();
    const bool ok = num_ranks <= dqrm_internal::kMergeMaxRanks && set->num_tables <= dqrm_internal::kMergeMaxTables &&
                    ws_bytes >= dqrm_internal::apply_workspace_bytes(num_ranks, cap_total);
    return ok && kind == DQRM_APPLY_MERGE;
}

// the flat kernel takes the apply (the choice apply_update_ex makes below)
static bool apply_takes_flat(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t ws_bytes) {
    if (apply_uses_merge(set, num_ranks, cap_total, ws_bytes)) return false;
    const int kind = apply_kernel_kind();
    if (kind == DQRM_APPLY_RANGES) return false;
    return !(kind == DQRM_APPLY_SLOT || (kind == DQRM_APPLY_AUTO && num_ranks > 1 && num_ranks >= set->dim / 4));
}

size_t dqrm_apply_workspace_bytes(int num_ranks, int64_t cap_total) {
    if (num_ranks <= 0 || cap_total < 0) return 0;
    return dqrm_internal::apply_workspace_bytes(num_ranks, cap_total);
}

// the next batch's forward inside the merge kernel's launch: a Criteo-form batch on the exact
// FP32 rows (the INT4 packed path stays a launch of its own); DQRM_FUSED_FWD=0 turns it off
static bool merge_fwd_fits(const dqrm_batch* next, uint32_t flags) {
    static const bool off = [] {
        const char* e = getenv("DQRM_FUSED_FWD");
        return e && !strcmp(e, "0");
    }();
    return !off && next && (next->flags & DQRM_BATCH_POOLING_ONE) && next->num_bags > 0 &&
           next->max_lookups >= next->num_bags && !(flags & DQRM_FWD_USE_PACKED);
}

static int apply_update(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total, const void* payloads,
                        size_t payload_bytes, size_t rank_pitch, int num_ranks, int grad_bits, const float* s_avg,
                        float lr, int mode, int repack_bits, void* ws, size_t ws_bytes, const FwdArgs* nf,
                        void* stream);
static int apply_update_ex(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total, const void* payloads,
                           size_t payload_bytes, size_t rank_pitch, int num_ranks, int grad_bits, const float* s_avg,
                           float lr, int mode, int repack_bits, void* ws, size_t ws_bytes, const FwdArgs* nf,
                           bool* fin_deferred, void* stream);

int dqrm_apply_sparse_update_strided(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total,
                                     const void* payloads, size_t payload_bytes, size_t rank_pitch, int num_ranks,
                                     int grad_bits, const float* s_avg, float lr, int mode, int repack_bits,
                                     void* stream) {
    return apply_update(set, cap_base, cap_total, payloads, payload_bytes, rank_pitch, num_ranks, grad_bits, s_avg,
                        lr, mode, repack_bits, nullptr, 0, nullptr, stream);
}

int dqrm_apply_sparse_update_fwd(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total,
                                 const void* payloads, size_t payload_bytes, size_t rank_pitch, int num_ranks,
                                 int grad_bits, const float* s_avg, float lr, int mode, int repack_bits,
                                 void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                                 uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                                 void* stream) {
    if (workspace && (((uintptr_t)workspace) & 15))
        return set_error(DQRM_E_INVALID, "%s: workspace must be 16-B aligned", "dqrm_apply_sparse_update_fwd");
    if (!next)  // the apply alone, with the workspace
        return apply_update(set, cap_base, cap_total, payloads, payload_bytes, rank_pitch, num_ranks, grad_bits, s_avg,
                            lr, mode, repack_bits, workspace, workspace_bytes, nullptr, stream);
    FwdArgs fa;  // the forward's arguments, validated as dqrm_emb_fwd validates them
    int rc = fwd_args(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b, "dqrm_apply_sparse_update_fwd",
                      &fa);
    if (rc) return rc;
    if (apply_uses_merge(set, num_ranks, cap_total, workspace_bytes) && merge_fwd_fits(next, fwd_flags))
        return apply_update(set, cap_base, cap_total, payloads, payload_bytes, rank_pitch, num_ranks, grad_bits, s_avg,
                            lr, mode, repack_bits, workspace, workspace_bytes, &fa, stream);
    // the flat apply: its finalize and the forward in one launch when the forward takes the exact rows
    const bool fin_fwd = finfwd_fits(set, next, fwd_flags);
    bool deferred = false;
    if ((rc = apply_update_ex(set, cap_base, cap_total, payloads, payload_bytes, rank_pitch, num_ranks, grad_bits,
                              s_avg, lr, mode, repack_bits, workspace, workspace_bytes, nullptr,
                              fin_fwd ? &deferred : nullptr, stream)))
        return rc;
    if (deferred) return launch_finalize_fwd(set, fa, (hipStream_t)stream);
    return dqrm_emb_fwd(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b, stream);
}

int dqrm_apply_fwd_form(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t workspace_bytes,
                        const dqrm_batch* next, uint32_t fwd_flags) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(next, "dqrm_apply_fwd_form"))) return rc;
    if (num_ranks <= 0 || num_ranks > DQRM_MAX_RANKS)
        return set_error(DQRM_E_INVALID, "%s: bad ranks (%d)", "dqrm_apply_fwd_form", num_ranks);
    if (apply_uses_merge(set, num_ranks, cap_total, workspace_bytes) && merge_fwd_fits(next, fwd_flags))
        return DQRM_APPLY_FWD_ONE_LAUNCH;
    if (apply_takes_flat(set, num_ranks, cap_total, workspace_bytes) && finalize_launch_flat() &&
        finfwd_fits(set, next, fwd_flags))
        return DQRM_APPLY_FWD_FIN_FWD;
    return DQRM_APPLY_FWD_SEPARATE;
}

int dqrm_apply_fwd_is_one_launch(const dqrm_table_set* set, int num_ranks, int64_t cap_total, size_t workspace_bytes,
                                 const dqrm_batch* next, uint32_t fwd_flags) {
    const int f = dqrm_apply_fwd_form(set, num_ranks, cap_total, workspace_bytes, next, fwd_flags);
    return f < 0 ? f : (f == DQRM_APPLY_FWD_ONE_LAUNCH ? 1 : 0);
}

static int apply_update(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total, const void* payloads,
                        size_t payload_bytes, size_t rank_pitch, int num_ranks, int grad_bits, const float* s_avg,
                        float lr, int mode, int repack_bits, void* ws, size_t ws_bytes, const FwdArgs* nf,
                        void* stream) {
    return apply_update_ex(set, cap_base, cap_total, payloads, payload_bytes, rank_pitch, num_ranks, grad_bits, s_avg,
                           lr, mode, repack_bits, ws, ws_bytes, nf, nullptr, stream);
}

// fin_deferred (non-null): a flat apply's finalize launch is left to the caller (*fin_deferred = true),
// which runs it together with the next forward (k_finalize_fwd)
static int apply_update_ex(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total, const void* payloads,
                           size_t payload_bytes, size_t rank_pitch, int num_ranks, int grad_bits, const float* s_avg,
                           float lr, int mode, int repack_bits, void* ws, size_t ws_bytes, const FwdArgs* nf,
                           bool* fin_deferred, void* stream) {
    if (fin_deferred) *fin_deferred = false;
    int rc = check_set(set);
    if (rc) return rc;
    if (num_ranks <= 0 || num_ranks > DQRM_MAX_RANKS || !payloads || !cap_base)
        return set_error(DQRM_E_INVALID, "%s: bad ranks/payloads (%d)", "dqrm_apply_sparse_update", num_ranks);
    if (mode == DQRM_UPD_FP32 ? grad_bits != 32 : (grad_bits < 2 || grad_bits > 16 || !s_avg))
        return set_error(DQRM_E_INVALID, "%s: mode/grad_bits mismatch (%d)", "dqrm_apply_sparse_update", grad_bits);
    if (payload_bytes != dqrm_payload_bytes(set->num_tables, cap_total, set->dim, grad_bits))
        return set_error(DQRM_E_INVALID, "%s: payload_bytes mismatch", "dqrm_apply_sparse_update");
    if (rank_pitch < payload_bytes || (rank_pitch & 15) || (((uintptr_t)payloads) & 15))
        return set_error(DQRM_E_INVALID, "%s: rank pitch %zu / payload alignment", "dqrm_apply_sparse_update",
                         rank_pitch);
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_apply_sparse_update", repack_bits);
    ApplyArgs a;
    a.W = set->W; a.packed = set->packed; a.rowmax = set->rowmax; a.blkmax = set->blkmax;
    a.sblkmax = set->sblkmax; a.sdirty = set->sdirty; a.pscale = set->pscale; a.meta = set->meta;
    a.err = set->err; a.cap_base = cap_base; a.cap_total = cap_total;
    a.payloads = (const unsigned char*)payloads; a.payload_bytes = (int64_t)rank_pitch;  // rank stride
    a.N = num_ranks; a.T = set->num_tables; a.bits = grad_bits; a.s_avg = s_avg; a.nlr = -lr;
    a.mode = mode; a.repack = repack_bits == 4; a.bdirty = set->bdirty; a.tmax = set->tmax; a.sync = set->sync;
    a.fin_launch = finalize_launch(); a.wt = 1;
    hipStream_t st = (hipStream_t)stream;
    const int D = set->dim;
    const int kind = apply_kernel_kind();
    bool flat = false;
    // MERGE (AUTO for 1 < N <= 16 ranks, T <= 64 tables): the ranks' rows merged in LDS per
    // block-aligned row range, the hierarchy finalized in-launch (dqrm_apply_merge.hip)
    if (apply_uses_merge(set, num_ranks, cap_total, ws_bytes)) {
        dqrm_internal::MergeApplyArgs r{};
        r.W = a.W; r.packed = a.packed; r.rowmax = a.rowmax; r.blkmax = a.blkmax; r.sblkmax = a.sblkmax;
        r.sdirty = a.sdirty; r.bdirty = a.bdirty; r.tmax = a.tmax; r.sync = a.sync; r.pscale = a.pscale;
        r.meta = a.meta; r.err = a.err; r.cap_base = cap_base; r.cap_total = cap_total; r.payloads = a.payloads;
        r.rank_pitch = (int64_t)rank_pitch; r.N = num_ranks; r.T = a.T; r.D = D; r.bits = grad_bits; r.s_avg = s_avg;
        r.nlr = -lr; r.mode = mode; r.repack = a.repack;
        merge_plan(set, cap_total, num_ranks, r.kt, r.kbase);
        r.pos = reinterpret_cast<int32_t*>(ws);
        static const int diag = [] {  // timing experiments: phases of k_merge_pos skipped (results wrong)
            const char* e = getenv("DQRM_MERGE_DIAG");
            return e ? atoi(e) : 0;
        }();
        r.diag = diag;
        r.gx = merge_apply_gx(set, cap_total, num_ranks, D);
        if (nf) {  // the next batch's forward: the grid's last T * fwd_gx workgroups, behind each table's gate
            static const uint32_t spin = [] {  // DQRM_GATE_SPIN: gate polls before a forward flags a stall
                const char* e = getenv("DQRM_GATE_SPIN");
                return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 20);
            }();
            r.fwd_idx = nf->idx; r.fwd_B = nf->B; r.fwd_out = nf->out; r.fwd_ost_t = nf->ost_t; r.fwd_ost_b = nf->ost_b;
            r.fwd_scale = set->scale; r.fwd_bits = nf->bits; r.fwd_flags = nf->flags;
            r.fwd_gx = dqrm_internal::merge_forward_gx(nf->B); r.spin_limit = spin;
        }
        HIP_TRY(dqrm_internal::launch_apply_merge(r, st));
        return DQRM_OK;  // the |W| hierarchy is finalized inside the launch
    }
    if (nf) return set_error(DQRM_E_INVALID, "%s: a fused forward needs the merge kernel", "dqrm_apply_sparse_update");
    if (kind == DQRM_APPLY_RANGES) {
        // chunks per slot: the payload capacity of all ranks spread over the slots, ~48
        // entries per workgroup (at least 1, at most 64)
        const int64_t slots = (int64_t)a.T * SPLIT;
        int64_t K = ((int64_t)num_ranks * cap_total + slots * 48 - 1) / (slots * 48);
        K = K < 1 ? 1 : (K > 64 ? 64 : K);
        dqrm_internal::RangeApplyArgs r{a.W, a.packed, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax,
                                        a.sync, a.pscale, a.meta, a.err, cap_base, cap_total, a.payloads,
                                        (int64_t)rank_pitch, num_ranks, a.T, D, grad_bits, s_avg, -lr, mode,
                                        a.repack, (int)K};
        HIP_TRY(dqrm_internal::launch_apply_ranges(r, st));
        return DQRM_OK;  // the |W| hierarchy is finalized inside the launch
    }
    // AUTO: flat while each lane of a row's group searches at most one other rank
    // (num_ranks < D/4), slot beyond (tools/bench_apply_ranks.py)
    if (!apply_takes_flat(set, num_ranks, cap_total, ws_bytes)) {  // SLOT, or AUTO at num_ranks >= D/4
        DISPATCH_LPR(D, {
            if ((rc = allow_lds(k_table_apply<LPR>, SLOT_LDS))) return rc;
            hipLaunchKernelGGL(k_table_apply<LPR>, dim3(a.T * SPLIT), dim3(TWG), SLOT_LDS, st, a);
        });
    } else {
        flat = true;
        a.fin_launch = finalize_launch_flat();
        a.wt = !a.fin_launch;
        // grid (entry chunks, tables, ranks): twice the chunks of an average table (the
        // per-table capacities live on the device); larger tables grid-stride, chunks past
        // a table's count exit at once
        DISPATCH_LPR(D, {
            constexpr int G = FLAT_TPB / LPR;
            int64_t gx = 2 * ((cap_total + (int64_t)a.T * G - 1) / ((int64_t)a.T * G));
            const int64_t lim = (32768 + (int64_t)a.T * num_ranks - 1) / ((int64_t)a.T * num_ranks);
            if (gx > lim) gx = lim;
            if (gx < 1) gx = 1;
            // two entries per lane group when the tables hold enough entries to keep the chip busy
            // at half the workgroups (same box, TB: 2048 per rank 129 vs 142 us at N = 8, 44 vs 48 at
            // N = 2; 256 per rank slower: 20 vs 14 us at N = 2); DQRM_FLAT_DUAL=0/1 forces it
            const char* dual_e = getenv("DQRM_FLAT_DUAL");  // read per call (tests switch it)
            const int dual_env = dual_e ? atoi(dual_e) : -1;
            const bool dual = dual_env >= 0 ? dual_env != 0 : cap_total >= (int64_t)512 * a.T;
            if (a.fin_launch && dual && num_ranks > 1 && num_ranks <= FLAT_HDR_RANKS && dual_env == 4)
                hipLaunchKernelGGL((k_apply_flat2<LPR, (LPR >= 4 ? 4 : 2)>), dim3((unsigned)gx, (unsigned)a.T,
                                   (unsigned)num_ranks), dim3(FLAT_TPB), 0, st, a);  // (LDS: E = 4 needs LPR >= 4)
            else if (a.fin_launch && dual && num_ranks > 1 && num_ranks <= FLAT_HDR_RANKS)
                hipLaunchKernelGGL((k_apply_flat2<LPR, 2>), dim3((unsigned)gx, (unsigned)a.T, (unsigned)num_ranks),
                                   dim3(FLAT_TPB), 0, st, a);
            else if (a.fin_launch)
                hipLaunchKernelGGL((k_apply_flat<LPR, false>), dim3((unsigned)gx, (unsigned)a.T, (unsigned)num_ranks),
                                   dim3(FLAT_TPB), 0, st, a);
            else
                hipLaunchKernelGGL((k_apply_flat<LPR, true>), dim3((unsigned)gx, (unsigned)a.T, (unsigned)num_ranks),
                                   dim3(FLAT_TPB), 0, st, a);
        });
    }
    LAUNCH_CHECK();  // both kernels finalize the |W| hierarchy inside the launch
    if (a.fin_launch && flat && fin_deferred) {
        *fin_deferred = true;
        return DQRM_OK;
    }
    if (a.fin_launch) return launch_finalize(set, st, flat, flat);
    return DQRM_OK;
}

int dqrm_apply_sparse_update(const dqrm_table_set* set, const int64_t* cap_base, int64_t cap_total,
                             const void* payloads, size_t payload_bytes, int num_ranks, int grad_bits,
                             const float* s_avg, float lr, int mode, int repack_bits, void* stream) {
    return dqrm_apply_sparse_update_strided(set, cap_base, cap_total, payloads, payload_bytes, payload_bytes,
                                            num_ranks, grad_bits, s_avg, lr, mode, repack_bits, stream);
}

int dqrm_apply_local(const dqrm_table_set* set, const int64_t* ws_cap_base, int64_t ws_cap_total,
                     const int32_t* ws_rows, const float* ws_vals, const int32_t* ws_ucount,
                     const float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                     void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if (grad_bits < 2 || grad_bits > 16)
        return set_error(DQRM_E_INVALID, "%s: grad_bits must be 2..16 (got %d)", "dqrm_apply_local", grad_bits);
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !ws_absmax || !s_avg || ws_cap_total < 0)
        return set_error(DQRM_E_INVALID, "%s: null workspace pointer", "dqrm_apply_local");
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)", "dqrm_apply_local", repack_bits);
    ApplyArgs a{};
    a.W = set->W; a.packed = set->packed; a.rowmax = set->rowmax; a.blkmax = set->blkmax;
    a.sblkmax = set->sblkmax; a.sdirty = set->sdirty; a.bdirty = set->bdirty; a.tmax = set->tmax; a.pscale = set->pscale;
    a.sync = set->sync; a.fin_launch = finalize_launch_flat(); a.wt = !a.fin_launch;
    a.meta = set->meta; a.err = set->err; a.N = 1; a.T = set->num_tables; a.bits = grad_bits;
    a.s_avg = s_avg; a.nlr = -lr; a.mode = DQRM_UPD_DP; a.repack = repack_bits == 4;
    hipStream_t st = (hipStream_t)stream;
    const int D = set->dim;
    const int64_t slots = (int64_t)a.T * SPLIT;
    DISPATCH_LPR(D, {
        // grid (entry chunks, slots): enough chunks for a slot at its mean capacity, slots
        // with fewer entries exit at once, fuller ones grid-stride
        constexpr int G = FLAT_TPB / LPR;
        int64_t gx = (ws_cap_total / (slots > 0 ? slots : 1) + G - 1) / G;
        const int64_t lim = (32768 + slots - 1) / (slots > 0 ? slots : 1);
        if (gx > lim) gx = lim;
        if (gx < 1) gx = 1;
        if (a.fin_launch)
            hipLaunchKernelGGL((k_apply_local<LPR, false>), dim3((unsigned)gx, (unsigned)slots), dim3(FLAT_TPB), 0, st,
                               a, ws_cap_base, ws_rows, ws_vals, ws_ucount, ws_absmax, s_avg);
        else
            hipLaunchKernelGGL((k_apply_local<LPR, true>), dim3((unsigned)gx, (unsigned)slots), dim3(FLAT_TPB), 0, st,
                               a, ws_cap_base, ws_rows, ws_vals, ws_ucount, ws_absmax, s_avg);
    });
    LAUNCH_CHECK();  // the table's last working workgroup finalizes its |W| hierarchy
    if (a.fin_launch) return launch_finalize(set, st, true, true);
    return DQRM_OK;
}

// dqrm_emb_bwd_apply_local's choice: one launch for Criteo-form batches whose grid can be
// resident at once (device CUs, occupancy, the stream's CU mask), the two calls otherwise
static bool apply_local_one_launch(const dqrm_table_set* set, const dqrm_batch* batch, void* stream) {
    static const bool fused_off = [] {
        const char* e = getenv("DQRM_LOCAL_FUSED");
        return e && !strcmp(e, "0");
    }();
    return !fused_off && g_coalesce_kernel.load() == DQRM_COALESCE_AUTO && (batch->flags & DQRM_BATCH_POOLING_ONE) &&
           batch->num_bags <= dqrm_internal::kCoalesceMaxB && batch->max_lookups >= batch->num_bags &&
           set->total_rows <= 0xffffffffll && set->num_tables <= dqrm_internal::kCoalesceApplyMaxT &&
           dqrm_internal::coalesce_apply_resident(set->num_tables, (hipStream_t)stream);
}

// the next batch's forward runs inside the one-launch step when it is a Criteo-form batch of
// the same size on the exact FP32 rows (the INT4 packed path stays a launch of its own)
static bool fused_fwd_fits(const dqrm_batch* batch, const dqrm_batch* next, uint32_t flags) {
    static const bool off = [] {
        const char* e = getenv("DQRM_FUSED_FWD");
        return e && !strcmp(e, "0");
    }();
    return !off && next && (next->flags & DQRM_BATCH_POOLING_ONE) && next->num_bags == batch->num_bags &&
           next->max_lookups >= next->num_bags && !(flags & DQRM_FWD_USE_PACKED);
}

int dqrm_bwd_apply_local_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_bwd_apply_local_is_one_launch"))) return rc;
    return apply_local_one_launch(set, batch, stream) ? 1 : 0;
}

// The next batch's forward fused behind the one-launch update (nullptr: none)
struct FusedFwd {
    const dqrm_batch* next;
    int bits;
    uint32_t flags;
    float* out;
    int64_t ost_t, ost_b;
};

static int bwd_apply_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy, int64_t dy_stride_t,
                           int64_t dy_stride_b, int ste, const int64_t* ws_cap_base, int64_t ws_cap_total,
                           int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount, float* ws_absmax, int grad_bits,
                           float* s_avg, float lr, int repack_bits, void* workspace, size_t workspace_bytes,
                           const FusedFwd* ff, void* stream);

int dqrm_emb_bwd_apply_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                             int64_t dy_stride_t, int64_t dy_stride_b, int ste, const int64_t* ws_cap_base,
                             int64_t ws_cap_total, int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount,
                             float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                             void* workspace, size_t workspace_bytes, void* stream) {
    return bwd_apply_local(set, batch, dy, dy_stride_t, dy_stride_b, ste, ws_cap_base, ws_cap_total, ws_rows, ws_vals,
                           ws_ucount, ws_absmax, grad_bits, s_avg, lr, repack_bits, workspace, workspace_bytes, nullptr,
                           stream);
}

int dqrm_emb_bwd_apply_fwd_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                                 int64_t dy_stride_t, int64_t dy_stride_b, int ste, const int64_t* ws_cap_base,
                                 int64_t ws_cap_total, int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount,
                                 float* ws_absmax, int grad_bits, float* s_avg, float lr, int repack_bits,
                                 void* workspace, size_t workspace_bytes, const dqrm_batch* next, int fwd_bits,
                                 uint32_t fwd_flags, float* out, int64_t out_stride_t, int64_t out_stride_b,
                                 void* stream) {
    FwdArgs fa;  // the forward's arguments, validated as dqrm_emb_fwd validates them
    int rc = fwd_args(set, next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b, "dqrm_emb_bwd_apply_fwd_local", &fa);
    if (rc) return rc;
    const FusedFwd ff{next, fwd_bits, fwd_flags, out, out_stride_t, out_stride_b};
    return bwd_apply_local(set, batch, dy, dy_stride_t, dy_stride_b, ste, ws_cap_base, ws_cap_total, ws_rows, ws_vals,
                           ws_ucount, ws_absmax, grad_bits, s_avg, lr, repack_bits, workspace, workspace_bytes, &ff,
                           stream);
}

int dqrm_bwd_apply_fwd_local_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch,
                                           const dqrm_batch* next, uint32_t fwd_flags, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_bwd_apply_fwd_local_is_one_launch"))) return rc;
    if ((rc = check_batch(next, "dqrm_bwd_apply_fwd_local_is_one_launch"))) return rc;
    return apply_local_one_launch(set, batch, stream) && fused_fwd_fits(batch, next, fwd_flags) ? 1 : 0;
}

int dqrm_bwd_sgd_fwd_is_one_launch(const dqrm_table_set* set, const dqrm_batch* batch, const dqrm_batch* next,
                                   uint32_t fwd_flags) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_bwd_sgd_fwd_is_one_launch"))) return rc;
    if ((rc = check_batch(next, "dqrm_bwd_sgd_fwd_is_one_launch"))) return rc;
    return sgd_small_plan(set, batch, next, fwd_flags, nullptr) == 2 ? 1 : 0;
}

static int bwd_apply_local(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy, int64_t dy_stride_t,
                           int64_t dy_stride_b, int ste, const int64_t* ws_cap_base, int64_t ws_cap_total,
                           int32_t* ws_rows, float* ws_vals, int32_t* ws_ucount, float* ws_absmax, int grad_bits,
                           float* s_avg, float lr, int repack_bits, void* workspace, size_t workspace_bytes,
                           const FusedFwd* ff, void* stream) {
    int rc = check_set(set);
    if (rc) return rc;
    if ((rc = check_batch(batch, "dqrm_emb_bwd_apply_local"))) return rc;
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return set_error(DQRM_E_INVALID, "%s: dy must be 16-B aligned with strides %% 4 == 0", "dqrm_emb_bwd_apply_local");
    if (!ws_cap_base || !ws_rows || !ws_vals || !ws_ucount || !ws_absmax || !s_avg || ws_cap_total < 0 ||
        (((uintptr_t)ws_vals) & 15))
        return set_error(DQRM_E_INVALID, "%s: null/unaligned workspace", "dqrm_emb_bwd_apply_local");
    if (grad_bits < 2 || grad_bits > 16)
        return set_error(DQRM_E_INVALID, "%s: grad_bits must be 2..16 (got %d)", "dqrm_emb_bwd_apply_local", grad_bits);
    if (repack_bits && (repack_bits != 4 || !set->packed))
        return set_error(DQRM_E_INVALID, "%s: repack needs packed rows and bits == 4 (got %d)",
                         "dqrm_emb_bwd_apply_local", repack_bits);
    if (apply_local_one_launch(set, batch, stream)) {
        if (batch->num_bags <= 0)  // nothing to update; the next batch's forward still runs
            return ff ? dqrm_emb_fwd(set, ff->next, ff->bits, ff->flags, ff->out, ff->ost_t, ff->ost_b, stream)
                      : DQRM_OK;
        dqrm_internal::CoalesceArgs ca{};
        ca.meta = set->meta; ca.T = set->num_tables; ca.D = set->dim; ca.B = batch->num_bags; ca.idx = batch->idx;
        ca.dy = dy; ca.dst_t = dy_stride_t; ca.dst_b = dy_stride_b; ca.scale = set->scale; ca.ste = ste;
        ca.err = set->err; ca.ws_cap_base = ws_cap_base; ca.ws_rows = ws_rows; ca.ws_vals = ws_vals;
        ca.ws_ucount = ws_ucount; ca.ws_absmax = ws_absmax;
        dqrm_internal::LocalApplyArgs la{};
        la.W = set->W; la.packed = set->packed; la.rowmax = set->rowmax; la.blkmax = set->blkmax;
        la.sblkmax = set->sblkmax; la.sdirty = set->sdirty; la.bdirty = set->bdirty; la.tmax = set->tmax;
        la.pscale = set->pscale; la.sync = set->sync; la.s_avg = s_avg; la.bits = grad_bits; la.nlr = -lr;
        la.repack = repack_bits == 4;
        dqrm_internal::plan_sub_slots(set->num_rows_host, set->num_tables, &la);
        const bool fused_fwd = ff && fused_fwd_fits(batch, ff->next, ff->flags);
        if (fused_fwd) {
            la.fwd_idx = ff->next->idx; la.fwd_out = ff->out; la.fwd_ost_t = ff->ost_t; la.fwd_ost_b = ff->ost_b;
            la.fwd_scale = set->scale; la.fwd_bits = ff->bits; la.fwd_flags = ff->flags;
        }
        const hipError_t e = dqrm_internal::launch_coalesce_pool1(ca, &la, (hipStream_t)stream);
        if (e != hipSuccess)
            return set_error(DQRM_E_HIP, "dqrm_emb_bwd_apply_local: launch failed: %s (%d)", hipGetErrorString(e), (int)e);
        if (ff && !fused_fwd)
            return dqrm_emb_fwd(set, ff->next, ff->bits, ff->flags, ff->out, ff->ost_t, ff->ost_b, stream);
        return DQRM_OK;
    }
    if ((rc = dqrm_emb_bwd_coalesce(set, batch, dy, dy_stride_t, dy_stride_b, ste, ws_cap_base, ws_rows, ws_vals,
                                    ws_ucount, ws_absmax, workspace, workspace_bytes, stream)))
        return rc;
    if ((rc = dqrm_apply_local(set, ws_cap_base, ws_cap_total, ws_rows, ws_vals, ws_ucount, ws_absmax, grad_bits,
                               s_avg, lr, repack_bits, stream)))
        return rc;
    if (ff) return dqrm_emb_fwd(set, ff->next, ff->bits, ff->flags, ff->out, ff->ost_t, ff->ost_b, stream);
    return DQRM_OK;
}

int dqrm_read_errors(const dqrm_table_set* set, uint32_t* flags, int clear, void* stream) {
    if (!set || !set->err || !flags) return set_error(DQRM_E_INVALID, "%s: null pointer", "dqrm_read_errors");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(flags, set->err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (clear) HIP_TRY(hipMemsetAsync(set->err, 0, sizeof(uint32_t), st));
    return DQRM_OK;
}


// ---------------------------------------------------------------------------------
// Row-wise PTQ formats
// ---------------------------------------------------------------------------------
#define DISPATCH_G(D, ...)                                                               \
    switch ((D) % 8 ? 0 : (D) / 8) {                                                     \
        case 1: { constexpr int G = 1; __VA_ARGS__; } break;                             \
        case 2: { constexpr int G = 2; __VA_ARGS__; } break;                             \
        case 4: { constexpr int G = 4; __VA_ARGS__; } break;                             \
        case 8: { constexpr int G = 8; __VA_ARGS__; } break;                             \
        case 16: { constexpr int G = 16; __VA_ARGS__; } break;                           \
        case 32: { constexpr int G = 32; __VA_ARGS__; } break;                           \
        default: return set_error(DQRM_E_INVALID, "dqrm rowwise: dim %d unsupported", (int)(D)); \
    }

size_t dqrm_rowwise_row_bytes(int bits, int dim) {
    if ((bits != 4 && bits != 8) || dim < 8 || (dim & 7)) return 0;
    return (size_t)rowwise_row_bytes(bits, dim);
}

int dqrm_rowwise_prepack(int bits, const float* W, int64_t num_rows, int dim, uint8_t* packed, void* stream) {
    if (bits != 4 && bits != 8) return set_error(DQRM_E_INVALID, "dqrm_rowwise_prepack: bits must be 4 or 8");
    if (!W || !packed || num_rows < 0) return set_error(DQRM_E_INVALID, "dqrm_rowwise_prepack: bad arguments");
    if (((uintptr_t)W) & 15) return set_error(DQRM_E_INVALID, "dqrm_rowwise_prepack: W must be 16-byte aligned");
    if (num_rows == 0) return DQRM_OK;
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_G(dim, {
        const int rows_per_wg = 256 / G;
        const int grid = grid_for(num_rows, rows_per_wg, 65536);
        if (bits == 4)
            hipLaunchKernelGGL((k_rowwise_prepack<4, G>), dim3(grid), dim3(256), 0, st, W, num_rows, packed);
        else
            hipLaunchKernelGGL((k_rowwise_prepack<8, G>), dim3(grid), dim3(256), 0, st, W, num_rows, packed);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

int dqrm_rowwise_bag(int bits, const uint8_t* packed, int64_t num_rows, int dim, const int64_t* idx,
                     int64_t num_lookups, const int64_t* off, int64_t num_bags, int include_last_offset,
                     const float* per_sample_weights, float* out, uint32_t* err, void* stream) {
    if (bits != 4 && bits != 8) return set_error(DQRM_E_INVALID, "dqrm_rowwise_bag: bits must be 4 or 8");
    if (!packed || !off || !out || !err || (num_lookups > 0 && !idx) || num_rows < 0 || num_lookups < 0)
        return set_error(DQRM_E_INVALID, "dqrm_rowwise_bag: bad arguments");
    if (((uintptr_t)packed) & 3 || ((uintptr_t)out) & 15)
        return set_error(DQRM_E_INVALID, "dqrm_rowwise_bag: packed must be 4-B and out 16-B aligned");
    if (num_bags <= 0) return DQRM_OK;
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_G(dim, {
        const int bags_per_wg = 256 / G;
        const int grid = grid_for(num_bags, bags_per_wg, 65536);
        if (bits == 4)
            hipLaunchKernelGGL((k_rowwise_bag<4, G>), dim3(grid), dim3(256), 0, st, packed, num_rows, idx,
                               num_lookups, off, num_bags, per_sample_weights, include_last_offset, out, err);
        else
            hipLaunchKernelGGL((k_rowwise_bag<8, G>), dim3(grid), dim3(256), 0, st, packed, num_rows, idx,
                               num_lookups, off, num_bags, per_sample_weights, include_last_offset, out, err);
    });
    LAUNCH_CHECK();
    return DQRM_OK;
}

}  // extern "C"
