// dqrm_lookup.hip — the per-lookup sparse gradient of nn.EmbeddingBag(sparse=True) that the
// grad_mode="sparse" module hands torch.optim.SGD, with duplicate rows pre-summed so that the
// optimizer's scatter-add is deterministic.
//
// Reference: quant_modules_not_quantize_grad.py:288 (nn.EmbeddingBag(..., sparse=True)), the
// STE backward quant_utils.py:349-363, and the SGD step dlrm_s_pytorch_single_gpu.py:1736-1750,
// 1943-1950 (param.add_(grad, alpha=-lr) on an uncoalesced COO grad). On the GPU that add is
// ATen's atomic index_add_: with duplicate rows its summation order, hence W's last bits, vary
// run to run. Here the COO keeps the reference's shape (indices = the lookups' rows, one entry
// per lookup) but the FIRST lookup of every row carries the row's whole gradient, summed in
// lookup order (the order Tensor.coalesce sums duplicates), and every later lookup of the row
// carries +0.0. The scatter then adds one value per row (a zero adds -lr * +0 = -0.0, the exact
// identity, in any order), so W is bit-identical run to run and the COO still sums to the
// same per-row gradient.
//
// One 1024-thread workgroup per table (<= kPresumMaxL lookups; larger tables keep the plain
// per-lookup gradient): rows into an LDS hash (linear probing, arrival rank per lookup), the
// rows' lookup lists laid out by a block scan of their counts, each list put in lookup order
// by counting, then one lane group (LPR lanes x float4) per lookup writes its entry -- a
// row's first lookup sums the row's dy slices along its ordered list, PS_RUN loads in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "dqrm_device.h"
#include "dqrm_internal.h"

namespace {

constexpr int PS_TPB = 1024;
constexpr int PS_MAXL = dqrm_internal::kPresumMaxL;
constexpr int PS_HLOG = 12;                  // 4096 hash slots: load <= 1/2
constexpr int PS_HSIZE = 1 << PS_HLOG;
constexpr int PS_PER = PS_MAXL / PS_TPB;     // lookups per thread
constexpr int PS_RUN = 8;                    // dy rows of an owner's walk in flight
constexpr int PS_NW = PS_TPB / WAVE;
static_assert(PS_HSIZE % PS_TPB == 0 && PS_MAXL % PS_TPB == 0, "presum geometry");

DQRM_INLINE uint32_t ps_hash(uint32_t r) { return (r * 0x9E3779B1u) >> (32 - PS_HLOG); }

template <int LPR>
__global__ void __launch_bounds__(PS_TPB) k_lookup_grad_presum(dqrm_internal::PresumArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = PS_TPB / LPR;           // lane groups
    constexpr int HPT = PS_HSIZE / PS_TPB;    // hash slots per thread (scan)
    __shared__ uint32_t h_key[PS_HSIZE];      // row + 1 (0: empty)
    __shared__ int h_cnt[PS_HSIZE];           // lookups of the row
    __shared__ int h_base[PS_HSIZE];          // first list entry of the row
    __shared__ int s_slot[PS_MAXL];           // lookup -> hash slot (-1: no entry)
    __shared__ int s_bag[PS_MAXL];            // lookup -> bag (bag form; -1: before the first bag)
    __shared__ int s_arr[PS_MAXL];            // lookup -> arrival rank in its row
    __shared__ int s_list[PS_MAXL];           // the rows' lookups, arrival order
    __shared__ int s_olist[PS_MAXL];          // the rows' lookups, lookup order
    __shared__ int s_w[PS_NW + 1];
    const int t = blockIdx.x, tid = threadIdx.x;
    const float s = a.scale[t];
    const int64_t rowbase = a.meta[t], nrows = a.meta[a.T + t];
    const int64_t ibase = a.pool1 ? (int64_t)t * a.B : a.idx_base[t];
    const int L = (int)(a.pool1 ? a.B : a.idx_base[t + 1] - ibase);
    const int64_t B = a.B;
    if (L < 0 || L > PS_MAXL) {  // the caller understated max_lookups: the LDS lists cannot hold the
        if (tid == 0) flag_error(a.err, DQRM_ERRF_OVERFLOW);  // table; flagged, its entries zero rows
        for (int64_t j = tid; j < L; j += PS_TPB) a.rows[ibase + j] = rowbase;
        for (int64_t q = tid; q < (int64_t)L * (D / 4); q += PS_TPB)
            reinterpret_cast<float4*>(a.vals + ibase * D)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const bool p1 = a.pool1 && L == B;
    // 1. indices of this thread's lookups (all in flight); the hash cleared meanwhile
    int64_t r[PS_PER];
#pragma unroll
    for (int i = 0; i < PS_PER; ++i) {
        const int j = tid + PS_TPB * i;
        r[i] = j < L ? a.idx[ibase + j] : -1;
    }
    for (int q = tid; q < PS_HSIZE; q += PS_TPB) {
        h_key[q] = 0u;
        h_cnt[q] = 0;
    }
    if (!p1) {  // bag form: every lookup's bag from the offsets, validated as nn.EmbeddingBag does
        const int64_t* off = a.off + (int64_t)t * B;
        for (int j = tid; j < L; j += PS_TPB) s_bag[j] = -1;
        __syncthreads();
        for (int64_t b = tid; b < B; b += PS_TPB) {
            int64_t s0 = off[b], s1 = b + 1 < B ? off[b + 1] : L;
            if (s0 < 0 || s1 > L || s1 < s0 || (b == 0 && s0 != 0)) {
                flag_error(a.err, DQRM_ERRF_OFFSET);
                s0 = s0 < 0 ? 0 : (s0 > L ? L : s0);
                s1 = s1 < s0 ? s0 : (s1 > L ? L : s1);
            }
            for (int64_t j = s0; j < s1; ++j) s_bag[j] = (int)b;
        }
    }
    __syncthreads();
    // 2. insert: row -> slot, arrival rank within the row
#pragma unroll
    for (int i = 0; i < PS_PER; ++i) {
        const int j = tid + PS_TPB * i;
        if (j >= L) continue;
        int slot = -1;
        const bool valid = r[i] >= 0 && r[i] < nrows;
        if (!valid) flag_error(a.err, DQRM_ERRF_INDEX);  // the entry becomes a zero row on row 0
        if (valid && (p1 || s_bag[j] >= 0)) {
            const uint32_t key = (uint32_t)r[i] + 1u;
            uint32_t h = ps_hash((uint32_t)r[i]);
            for (;;) {
                const uint32_t old = atomicCAS(&h_key[h], 0u, key);
                if (old == 0u || old == key) break;
                h = (h + 1u) & (PS_HSIZE - 1);
            }
            slot = (int)h;
            s_arr[j] = atomicAdd(&h_cnt[h], 1);
        }
        s_slot[j] = slot;
    }
    __syncthreads();
    // 3. list bases: exclusive scan of the row counts (HPT consecutive slots per thread)
    {
        int c[HPT], sum = 0;
#pragma unroll
        for (int k = 0; k < HPT; ++k) {
            c[k] = h_cnt[tid * HPT + k];
            sum += c[k];
        }
        const int lane = tid % WAVE, w = tid / WAVE;
        int v = sum;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int y = __shfl_up(v, o, WAVE);
            if (lane >= o) v += y;
        }
        if (lane == WAVE - 1) s_w[w] = v;
        __syncthreads();
        if (tid == 0) {
            int run = 0;
            for (int q = 0; q < PS_NW; ++q) { const int x = s_w[q]; s_w[q] = run; run += x; }
        }
        __syncthreads();
        int base = s_w[w] + v - sum;
#pragma unroll
        for (int k = 0; k < HPT; ++k) {
            h_base[tid * HPT + k] = base;
            base += c[k];
        }
    }
    __syncthreads();
    // 4. every lookup to its row's list (arrival order), then to its place in lookup order
#pragma unroll
    for (int i = 0; i < PS_PER; ++i) {
        const int j = tid + PS_TPB * i;
        if (j < L && s_slot[j] >= 0) s_list[h_base[s_slot[j]] + s_arr[j]] = j;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PS_PER; ++i) {
        const int j = tid + PS_TPB * i;
        if (j >= L || s_slot[j] < 0) continue;
        const int b0 = h_base[s_slot[j]], n = h_cnt[s_slot[j]];
        int before = 0;
        for (int k = b0; k < b0 + n && n > 1; ++k) before += s_list[k] < j ? 1 : 0;
        s_olist[b0 + before] = j;
    }
    __syncthreads();
    // 5. entries: one lane group per lookup
    const int lane = tid % LPR, grp = tid / LPR;
    const float* dyt = a.dy + (int64_t)t * a.dst_t;
    auto bag_of = [&](int j) -> int64_t { return p1 ? j : s_bag[j]; };
    auto ste = [&](float4 g) -> float4 {
        if (a.ste) { g.x = (g.x * s) / s; g.y = (g.y * s) / s; g.z = (g.z * s) / s; g.w = (g.w * s) / s; }
        return g;
    };
    for (int j = grp; j < L; j += G) {
        const int slot = s_slot[j];
        const int64_t row = slot >= 0 ? (int64_t)h_key[slot] - 1 : 0;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (slot >= 0) {
            const int b0 = h_base[slot], n = h_cnt[slot];
            if (s_olist[b0] == j) {  // the row's first lookup: its whole gradient, in lookup order
                v = ste(reinterpret_cast<const float4*>(dyt + bag_of(j) * a.dst_b)[lane]);
                for (int k0 = 1; k0 < n; k0 += PS_RUN) {
                    float4 x[PS_RUN];
#pragma unroll
                    for (int k = 0; k < PS_RUN; ++k) {  // PS_RUN dy rows in flight (clamped addresses)
                        const int q = s_olist[b0 + (k0 + k < n ? k0 + k : n - 1)];
                        x[k] = reinterpret_cast<const float4*>(dyt + bag_of(q) * a.dst_b)[lane];
                    }
#pragma unroll
                    for (int k = 0; k < PS_RUN; ++k) {
                        if (k0 + k >= n) break;
                        const float4 g = ste(x[k]);
                        v.x = v.x + g.x; v.y = v.y + g.y; v.z = v.z + g.z; v.w = v.w + g.w;
                    }
                }
            }
        }
        if (lane == 0) a.rows[ibase + j] = rowbase + row;
        reinterpret_cast<float4*>(a.vals + (ibase + j) * D)[lane] = v;
    }
}

}  // namespace

namespace dqrm_internal {

hipError_t launch_lookup_grad_presum(const PresumArgs& a, hipStream_t stream) {
    switch (a.D) {
#define PS_CASE(Dd)                                                                                        \
    case Dd: hipLaunchKernelGGL(k_lookup_grad_presum<Dd / 4>, dim3(a.T), dim3(PS_TPB), 0, stream, a); break;
        PS_CASE(4) PS_CASE(8) PS_CASE(16) PS_CASE(32) PS_CASE(64) PS_CASE(128) PS_CASE(256)
#undef PS_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dqrm_internal

extern "C" int dqrm_internal_set_error(int code, const char* msg);  // dqrm_kernels.hip (hidden)

extern "C" int dqrm_emb_bwd_lookup_grad_presum(const dqrm_table_set* set, const dqrm_batch* batch, const float* dy,
                                               int64_t dy_stride_t, int64_t dy_stride_b, int ste, int64_t* rows,
                                               float* vals, void* stream) {
    const char* who = "dqrm_emb_bwd_lookup_grad_presum";
    char buf[256];
    auto err = [&](int code, const char* what) {
        snprintf(buf, sizeof(buf), "%s: %s", who, what);
        return dqrm_internal_set_error(code, buf);
    };
    if (!set || !batch || !set->meta || !set->scale || !set->err || set->num_tables <= 0)
        return err(DQRM_E_INVALID, "null table set / batch");
    const int D = set->dim;
    if (D < 4 || D > 256 || (D & 3) || ((D / 4) & (D / 4 - 1))) return err(DQRM_E_INVALID, "dim must be 4*2^k <= 256");
    if (!batch->idx || !batch->off || !batch->idx_base) return err(DQRM_E_INVALID, "null batch pointer");
    if (!dy || (((uintptr_t)dy) & 15) || (dy_stride_t & 3) || (dy_stride_b & 3))
        return err(DQRM_E_INVALID, "dy must be 16-B aligned with strides % 4 == 0");
    if (!rows || !vals || (((uintptr_t)vals) & 15)) return err(DQRM_E_INVALID, "rows / 16-B aligned vals required");
    if (batch->max_lookups > DQRM_PRESUM_MAX_LOOKUPS)
        return err(DQRM_E_CAPACITY, "a table has more than DQRM_PRESUM_MAX_LOOKUPS lookups (max_lookups)");
    if (batch->num_bags <= 0) return DQRM_OK;
    dqrm_internal::PresumArgs a{set->meta, set->scale, set->err, batch->idx, batch->off, batch->idx_base, dy,
                                dy_stride_t, dy_stride_b, batch->num_bags, rows, vals, set->num_tables, D, ste,
                                (batch->flags & DQRM_BATCH_POOLING_ONE) != 0};
    const hipError_t e = dqrm_internal::launch_lookup_grad_presum(a, (hipStream_t)stream);
    if (e != hipSuccess) return err(DQRM_E_HIP, hipGetErrorString(e));
    return DQRM_OK;
}
