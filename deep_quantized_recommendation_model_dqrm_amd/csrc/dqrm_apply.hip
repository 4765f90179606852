// dqrm_apply.hip — K6 for the N > 1 exchange: decode the N gathered payloads, sum each row's
// integer gradients over the ranks, dequantize, SGD, and keep the |W| hierarchy exact, in ONE
// launch (no finalize launch after it).
//
// Reference: sgd_quantized_gradients_parallel_comm.py quantize_emb_grad :873-885 (Gloo's
// sparse all_reduce: union of the ranks' rows, integer sum, * 1/N) and
// weight_update_parallel_comm :601-628 (W.add_(-lr * grad * s.item())); the table scale of
// the next forward is the full-table max|W| (quant_utils.py:141-194), kept incrementally.
//
// Work split: workgroup (table t, row-range slot s, chunk k) owns a block-aligned row range
// (the slot's blocks cut into K chunks). Every rank's entries of slot s arrive with rows
// ascending (dqrm_grad_quant_pack), so the chunk's entries are one contiguous run per rank,
// found by counting the slot's rows below the range's bounds (one cooperative load, no binary
// search chain). The lowest rank holding a row owns it and sums the ranks' values in ascending
// rank order. Because the workgroup owns every block of its range, a block whose max holder
// shrank is re-reduced right here (its other rows' stored maxima + the new ones); growth goes
// in by atomicMax; only a superblock whose holder block shrank is flagged, for the table's
// last-arriving workgroup (one arrival per workgroup, carrying "flagged"), which re-reduces
// flagged superblocks and, if needed, the table max -- the work of the separate
// k_table_finalize launch of the flat kernel, done only when some superblock needs it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dqrm_device.h"
#include "dqrm_internal.h"

namespace {

constexpr int SPLIT = DQRM_TABLE_SPLIT;
constexpr int AR_TPB = 256;
constexpr int AR_NW = AR_TPB / WAVE;
constexpr int AR_MAXN = 64;            // ranks
constexpr int AR_OWNQ = 128;           // shrunk block-max holders re-reduced in the workgroup
constexpr int AR_INFL = 4;             // entries per lane group with their loads in flight
constexpr uint32_t AR_DIRTY_ONE = 1u << 16;  // arrival word: arrivals | flagged arrivals << 16

template <int LPR>
__global__ void __launch_bounds__(AR_TPB) k_apply_ranges(dqrm_internal::RangeApplyArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = AR_TPB / LPR;    // lane groups
    __shared__ int s_pre[AR_MAXN];     // rank r: the slot's first entry in its table section
    __shared__ int s_cnt[AR_MAXN];     //   the slot's entries
    __shared__ int s_lo[AR_MAXN];      //   the chunk's first entry (within the slot)
    __shared__ int s_hi[AR_MAXN];      //   one past its last
    __shared__ int s_start[AR_MAXN + 1];  // prefix of the chunk's entries over the ranks
    __shared__ int s_oq_n;
    __shared__ uint32_t s_oq_blk[AR_OWNQ];
    __shared__ float s_oq_old[AR_OWNQ];
    __shared__ float s_oq_sold[AR_OWNQ];
    __shared__ int s_dirty;
    __shared__ int s_fin;
    const int K = a.K;
    const int slotk = (int)blockIdx.x / K, k = (int)blockIdx.x % K;
    const int t = slotk / SPLIT, s = slotk % SPLIT;
    const int tid = threadIdx.x, lane = tid % WAVE, w = tid / WAVE;
    const int T = a.T, N = a.N;
    const int64_t rb = a.meta[t], nrows = a.meta[T + t], bb = a.meta[2 * T + t], sbb = a.meta[3 * T + t];
    const uint32_t nblk = (uint32_t)((nrows + BLK - 1) / BLK);
    // this workgroup's blocks: the slot's (dqrm_emb_bwd_coalesce's row-range slots) cut in K
    // (32-bit arithmetic: a slot has < 2^26 blocks, K <= 64)
    auto slot0 = [&](int ss) { return (uint32_t)(((uint64_t)nblk * (uint32_t)ss) >> 3); };
    static_assert(SPLIT == 8, "slot bounds by shifts");
    const uint32_t s0 = slot0(s), nb = slot0(s + 1) - s0;
    const uint32_t b0 = s0 + nb * (uint32_t)k / (uint32_t)K, b1 = s0 + nb * (uint32_t)(k + 1) / (uint32_t)K;
    if (b0 >= b1) return;  // no rows (and no arrival: not counted below)
    // the table's workgroups with rows: a slot of nb blocks has min(nb, K) non-empty chunks
    uint32_t expected = 0;
#pragma unroll
    for (int ss = 0; ss < SPLIT; ++ss) {
        const uint32_t n_s = slot0(ss + 1) - slot0(ss);
        expected += n_s < (uint32_t)K ? n_s : (uint32_t)K;
    }
    const int64_t row_lo = (int64_t)b0 * BLK, row_hi = (int64_t)b1 * BLK < nrows ? (int64_t)b1 * BLK : nrows;
    const PayloadLayout pl = payload_layout(T, a.cap_total, D, a.bits);
    const int64_t cb = a.cap_base[t], cap = a.cap_base[t + 1] - cb;
    auto rows_of = [&](int r) {
        return reinterpret_cast<const int32_t*>(a.payloads + (int64_t)r * a.rank_pitch + pl.rows_off) + cb;
    };
    // 1. each rank's run of slot s in its table section (header counts, slot order, clamped)
    if (tid < N) {
        const int32_t* hdr = reinterpret_cast<const int32_t*>(a.payloads + (int64_t)tid * a.rank_pitch) + t * SPLIT;
        int c[SPLIT];
#pragma unroll
        for (int q = 0; q < SPLIT; ++q) c[q] = hdr[q];
        int run = 0, pre = 0, my = 0;
#pragma unroll
        for (int q = 0; q < SPLIT; ++q) {
            int x = c[q] < 0 ? 0 : c[q];
            x = x < cap - run ? x : (int)(cap - run);
            if (q == s) { pre = run; my = x; }
            run += x;
        }
        s_pre[tid] = pre;
        s_cnt[tid] = my;
        s_lo[tid] = 0;
        s_hi[tid] = K == 1 ? my : 0;
    }
    if (tid == 0) {
        s_oq_n = 0;
        s_dirty = 0;
    }
    __syncthreads();
    // 2. K > 1: the chunk's run in each rank = [#rows < row_lo, #rows < row_hi) of the slot's
    //    ascending rows (every rank's slot rows loaded once, counted with LDS adds)
    if (K > 1) {  // per rank: wave ballots, one LDS add per wave
        for (int r = 0; r < N; ++r) {
            const int32_t* rows = rows_of(r) + s_pre[r];
            const int n = s_cnt[r];
            for (int i0 = w * WAVE; i0 < n; i0 += AR_TPB) {
                const int i = i0 + lane;
                const int32_t x = i < n ? rows[i] : 0x7fffffff;
                const int nlo = __popcll(__ballot(x < row_lo)), nhi = __popcll(__ballot(x < row_hi));
                if (lane == 0) {
                    if (nlo) atomicAdd(&s_lo[r], nlo);
                    if (nhi) atomicAdd(&s_hi[r], nhi);
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        int run = 0;
        for (int r = 0; r < N; ++r) {
            s_start[r] = run;
            run += s_hi[r] - s_lo[r];
        }
        s_start[N] = run;
    }
    __syncthreads();
    const int M = s_start[N];
    // 3. the update: one LPR-lane group per entry; AR_INFL entries' loads in flight
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate upd{a.mode, (float)(1.0 / (double)N), sc, (float)((double)sc / (double)N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const float otm = a.tmax[t];
    const int sub = tid % LPR, grp = tid / LPR;
    const int gbase = lane - sub;  // first lane of this group in the wave
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    auto value = [&](int r, int e) -> float4 {  // rank r's entry e of slot s, widened to f32
        const unsigned char* p = a.payloads + (int64_t)r * a.rank_pitch + pl.vals_off;
        const int64_t q = cb + s_pre[r] + e;
        float4 v;
        if (pl.elem == 1) {
            const uint32_t x = reinterpret_cast<const uint32_t*>(p + q * D)[sub];
            v.x = (float)(int8_t)(x & 0xFF); v.y = (float)(int8_t)((x >> 8) & 0xFF);
            v.z = (float)(int8_t)((x >> 16) & 0xFF); v.w = (float)(int8_t)(x >> 24);
        } else if (pl.elem == 2) {
            const uint2 x = reinterpret_cast<const uint2*>(p + q * D * 2)[sub];
            v.x = (float)(int16_t)(x.x & 0xFFFF); v.y = (float)(int16_t)(x.x >> 16);
            v.z = (float)(int16_t)(x.y & 0xFFFF); v.w = (float)(int16_t)(x.y >> 16);
        } else {
            v = reinterpret_cast<const float4*>(p + q * D * 4)[sub];
        }
        return v;
    };
    // position of row x in rank j's chunk run [lo_j, hi_j) (ascending rows), or -1
    auto find = [&](int j, int32_t x) -> int {
        const int32_t* rows = rows_of(j) + s_pre[j];
        int lo = s_lo[j], hi = s_hi[j];
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (rows[mid] < x) lo = mid + 1; else hi = mid;
        }
        return (lo < s_hi[j] && rows[lo] == x) ? lo : -1;
    };
    bool dirty = false;
    for (int i0 = grp; i0 < M; i0 += G * AR_INFL) {
        int rk[AR_INFL], ee[AR_INFL];
        int32_t xx[AR_INFL];
        bool own[AR_INFL];
        float4 acc[AR_INFL], w0[AR_INFL];
        float ob[AR_INFL], osb[AR_INFL];
#pragma unroll
        for (int h = 0; h < AR_INFL; ++h) {  // the entries' rows
            const int i = i0 + h * G;
            int r = 0;
            if (i < M)
                while (i >= s_start[r + 1]) ++r;
            rk[h] = r;
            ee[h] = i < M ? s_lo[r] + (i - s_start[r]) : 0;
            xx[h] = i < M ? rows_of(r)[s_pre[r] + ee[h]] : -1;
        }
#pragma unroll
        for (int h = 0; h < AR_INFL; ++h) {  // ownership and the rank-ordered sum
            const int i = i0 + h * G;
            own[h] = i < M && xx[h] >= row_lo && xx[h] < row_hi;
            if (i < M && !own[h] && sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);  // cannot happen
            acc[h] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!own[h]) continue;
            if (N == 1) {
                acc[h] = value(0, ee[h]);
                continue;
            }
            // lane q of the group looks for the row in ranks q, q + LPR, ...: a lower rank
            // holding it owns the row
            bool lower = false;
            for (int j = sub; j < rk[h]; j += LPR) lower |= find(j, xx[h]) >= 0;
            if (__ballot(lower) & gmask) {
                own[h] = false;
                continue;
            }
            bool first = true;
            for (int j = rk[h]; j < N; ++j) {  // ascending rank order (FP32: Gloo's order)
                const int p = j == rk[h] ? ee[h] : find(j, xx[h]);
                if (p < 0) continue;
                const float4 v = value(j, p);
                if (first) { acc[h] = v; first = false; }
                else { acc[h].x += v.x; acc[h].y += v.y; acc[h].z += v.z; acc[h].w += v.w; }
            }
        }
#pragma unroll
        for (int h = 0; h < AR_INFL; ++h) {  // W rows and the maxima they are tested against
            w0[h] = make_float4(0.f, 0.f, 0.f, 0.f);
            ob[h] = osb[h] = 0.0f;
            if (!own[h]) continue;
            const int64_t x = xx[h];
            w0[h] = reinterpret_cast<const float4*>(a.W + (rb + x) * D)[sub];
            ob[h] = a.blkmax[bb + (x >> 8)];
            osb[h] = a.sblkmax[sbb + (x >> 16)];
        }
#pragma unroll
        for (int h = 0; h < AR_INFL; ++h) {
            if (!own[h]) continue;
            const int64_t x = xx[h], grow = rb + x, blk = x >> 8, sb = sbb + (x >> 16);
            float4 wn;
            wn.x = upd(w0[h].x, acc[h].x); wn.y = upd(w0[h].y, acc[h].y);
            wn.z = upd(w0[h].z, acc[h].z); wn.w = upd(w0[h].w, acc[h].w);
            reinterpret_cast<float4*>(a.W + grow * D)[sub] = wn;
            if (a.repack) pack4_row(wn, a.packed + grow * (D / 2), sub, r_pack);
            const float old_rm = group_max<LPR>(abs_max4(w0[h]));
            const float rm = group_max<LPR>(abs_max4(wn));
            if (sub != 0) continue;
            st_wt(a.rowmax + grow, rm);
            if (rm > ob[h]) {  // growth: order-free atomicMax on the non-negative float bits
                atomicMax(reinterpret_cast<unsigned int*>(a.blkmax) + bb + blk, __float_as_uint(rm));
                if (rm > osb[h]) {
                    atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sb, __float_as_uint(rm));
                    if (rm > otm) atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(rm));
                }
            }
            if (old_rm == ob[h] && rm < old_rm) {  // the block's max holder shrank: re-reduced below
                const int p = atomicAdd(&s_oq_n, 1);
                if (p < AR_OWNQ) {
                    s_oq_blk[p] = (uint32_t)blk;
                    s_oq_old[p] = ob[h];
                    s_oq_sold[p] = osb[h];
                } else {  // queue full: the table's last workgroup re-reduces it
                    flag_set(a.bdirty, bb + blk);
                    flag_set(a.sdirty, sb);
                    dirty = true;
                }
            }
        }
    }
    // 4. owned blocks whose max holder shrank: their 256 row maxima (this workgroup's new ones
    //    stored write-through; the untouched rows' unchanged), one wave per block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nq = s_oq_n < AR_OWNQ ? s_oq_n : AR_OWNQ;
    for (int q = w; q < nq; q += AR_NW) {
        const int64_t blk = s_oq_blk[q];
        float v[BLK / WAVE];
#pragma unroll
        for (int i = 0; i < BLK / WAVE; ++i) {
            const int64_t r = blk * BLK + lane + i * WAVE;
            v[i] = r < nrows ? ld_wt(a.rowmax + rb + r) : 0.0f;
        }
        float mv = 0.0f;
#pragma unroll
        for (int i = 0; i < BLK / WAVE; ++i) mv = fmaxf(mv, v[i]);
        mv = wave_max(mv);
        if (lane == 0) {
            st_wt(a.blkmax + bb + blk, mv);
            // it held the superblock's max before this step: the superblock may have shrunk
            if (mv < s_oq_old[q] && s_oq_old[q] == s_oq_sold[q]) {
                flag_set(a.sdirty, sbb + (blk >> 8));
                dirty = true;
            }
        }
    }
    if (dirty) s_dirty = 1;
    // 5. one arrival per workgroup after its stores landed (hand-off row 1 of the microarch
    //    guide); the last one re-reduces flagged superblocks / the table max, only if flagged
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        uint32_t* cnt = a.sync + (int64_t)t * DQRM_SYNC_STRIDE;
        const uint32_t add = 1u + (s_dirty ? AR_DIRTY_ONE : 0u);
        const uint32_t now = atomicAdd(cnt, add) + add;
        const bool last = (now & (AR_DIRTY_ONE - 1u)) == expected;
        if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_fin = last && (now >> 16) != 0u;
    }
    __syncthreads();
    if (s_fin)
        finalize_table<true>(make_meta(a.meta, T), t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty, a.tmax,
                             D, true, false);
}

}  // namespace

namespace dqrm_internal {

hipError_t launch_apply_ranges(const RangeApplyArgs& a, hipStream_t stream) {
    if (a.N < 1 || a.N > AR_MAXN || a.K < 1) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(a.T * SPLIT * a.K));
    switch (a.D) {
#define AR_CASE(Dd) \
    case Dd: hipLaunchKernelGGL(k_apply_ranges<Dd / 4>, grid, dim3(AR_TPB), 0, stream, a); break;
        AR_CASE(4) AR_CASE(8) AR_CASE(16) AR_CASE(32) AR_CASE(64) AR_CASE(128) AR_CASE(256)
#undef AR_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dqrm_internal
