// dqrm_apply_merge.hip — K6 for the N > 1 exchange (DQRM_APPLY_MERGE, opt-in; measured not faster
// than the flat kernel on the TB shape, so AUTO keeps the flat one -- DESIGN.md 6):
// decode the N gathered payloads, sum each row's gradients over the ranks, dequantize, SGD, keep
// the |W| hierarchy exact -- and, at the step boundary, the NEXT batch's forward -- in two
// launches, without the per-entry searches of the flat kernel.
//
// Reference: sgd_quantized_gradients_parallel_comm.py quantize_emb_grad :873-885 (Gloo's
// sparse all_reduce: union of the ranks' rows, integer sum, * 1/N) and
// weight_update_parallel_comm :601-628 (W.add_(-lr * grad * s.item())); the next forward's
// table scale is the full-table max|W| (quant_utils.py:141-194), kept incrementally; the next
// forward is apply_emb (dlrm_s_pytorch_single_gpu.py:609-674, q_m_n_q_g.py:317-398).
//
// Why: at N ranks every rank applies the union of all ranks' rows (weak scaling: ~N times one
// rank's rows). The flat kernel locates each entry's row in the other ranks' lists by binary
// searches in HBM and then reads the ranks' values one after another -- (N-1) chains of ~11
// dependent round trips plus N more per entry: 129 us at N = 8 on the TB shape
// (profiles/r6_apply_ranks_tb2048.txt). Here:
//   k_merge_pos   one workgroup per block-aligned row range of a row-range slot (~256 entries of
//                 all ranks): every rank's entries of the range are one contiguous run of its
//                 ascending rows, found by one pipelined ballot count, copied to LDS; every
//                 (entry, rank) pair is located by a binary search IN LDS, all pairs at once; the
//                 positions go to the caller's workspace (N ints per entry);
//   k_apply_pos   the flat kernel's shape (one lane group per entry, the whole chip) with the
//                 positions read in ONE load: an entry that a lower rank also holds is skipped,
//                 the owner loads every rank's value in one round trip (int8: 4 B per lane and
//                 rank) and sums them in ascending rank order (exact integer sums), then the SGD
//                 and the hierarchy (growth by atomicMax, a shrunk block-max holder flagged);
//                 the table's last arriving workgroup finalizes its hierarchy when it was
//                 flagged, then opens the table's gate for the forward plane: the grid's last
//                 slice of workgroups, which gather and fake-quantize the next batch's rows of
//                 that table (sc1 loads of the sc1-stored rows, MI355X_MICROARCH.md hand-off).
// At N = 1 (the forced collectives path) k_merge_pos is not needed: every entry owns its row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dqrm_device.h"
#include "dqrm_internal.h"

namespace {

constexpr int SPLIT = DQRM_TABLE_SPLIT;
constexpr int AM_TPB = 256;
constexpr int AM_MAXN = dqrm_internal::kMergeMaxRanks;  // ranks
constexpr int AM_KEYS = 4096;     // a chunk's rows of all ranks held in LDS (else searched in HBM)
constexpr int AM_MAP = 16384;     // dense-range map entries (int16): row span x ranks
constexpr int AP_TPB = 256;       // k_apply_pos
constexpr int AP_INFL = 4;        // entries per lane group with their loads in flight
static_assert(SPLIT == 8, "slot bounds by shifts");

constexpr int GATE_WORD = 8;       // a table's sync word: 1 = its update and |W| maxima are final (FWD)
constexpr int FCNT_WORD = 9;       //   arrivals of its forward workgroups (the last one re-arms both)
constexpr int FWD_UNR = 4;         // forward: bags per lane group with their loads in flight

// The next batch's forward of table t, workgroup bx of the table's a.fwd_gx (Criteo form: bag b
// = lookup b): once the table's last updating workgroup has opened the gate, the fake-quant
// EmbeddingBag of dqrm_emb_fwd (emb_fwd_table's arithmetic) with every handed-off byte (W rows,
// tmax) read by sc1 loads (MI355X_MICROARCH.md hand-off: the updates stored them sc1).
template <int LPR>
DQRM_INLINE void merge_forward(const dqrm_internal::MergeApplyArgs& a, int t, int bx) {
    constexpr int D = LPR * 4;
    constexpr int G = AM_TPB / LPR;
    uint32_t* gate = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + GATE_WORD;
    __shared__ int s_go;
    if (threadIdx.x == 0) {
        uint32_t n = 0;
        while (ld_wt(gate) == 0u) {  // bounded: a gate that never opens is flagged, not a hang
            if (++n > a.spin_limit) {
                flag_error(a.err, DQRM_ERRF_STALL);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        s_go = 1;
    }
    __syncthreads();
    (void)s_go;
    const bool fullp = (a.fwd_flags & DQRM_FWD_FULL_PRECISION) != 0;
    const bool refresh = (a.fwd_flags & DQRM_FWD_REFRESH_SCALE) != 0;
    float sv = 1.0f;
    if (!fullp) sv = refresh ? sym_scale(ld_wt(a.tmax + t), a.fwd_bits) : a.fwd_scale[t];
    if (refresh && !fullp && bx == 0 && threadIdx.x == 0) a.fwd_scale[t] = sv;
    const float rr = 1.0f / sv;
    const float qlo = -(float)(1 << (a.fwd_bits - 1)), qhi = (float)((1 << (a.fwd_bits - 1)) - 1);
    const int64_t rb = a.meta[t], nrows = a.meta[a.T + t];
    const int64_t B = a.fwd_B;
    const int64_t* idx = a.fwd_idx + (int64_t)t * B;
    float* out = a.fwd_out + (int64_t)t * a.fwd_ost_t;
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    for (int64_t b0 = (int64_t)bx * (G * FWD_UNR); b0 < B; b0 += (int64_t)a.fwd_gx * (G * FWD_UNR)) {
        int64_t x[FWD_UNR];
#pragma unroll
        for (int k = 0; k < FWD_UNR; ++k) {  // every index load in flight, then every row load
            const int64_t b = b0 + k * G + grp;
            x[k] = idx[b < B ? b : B - 1];
        }
        float4 v[FWD_UNR];
#pragma unroll
        for (int k = 0; k < FWD_UNR; ++k) {
            const bool ok = x[k] >= 0 && x[k] < nrows;
            v[k] = nrows > 0 ? ld4_wt(a.W + (rb + (ok ? x[k] : 0)) * D + sub * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < FWD_UNR; ++k) {
            const int64_t b = b0 + k * G + grp;
            if (b >= B) continue;
            const bool ok = x[k] >= 0 && x[k] < nrows;
            if (!ok && sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
            float4 y = ok ? v[k] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (!fullp) {
                y.x = fake_quant(y.x, rr, qlo, qhi) * sv;
                y.y = fake_quant(y.y, rr, qlo, qhi) * sv;
                y.z = fake_quant(y.z, rr, qlo, qhi) * sv;
                y.w = fake_quant(y.w, rr, qlo, qhi) * sv;
            }
            reinterpret_cast<float4*>(out + b * a.fwd_ost_b)[sub] = y;
        }
    }
    // every forward workgroup of the table has passed the gate once the last one arrives here:
    // it re-arms the gate and the count for the next launch
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t* fcnt = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FCNT_WORD;
        if (atomicAdd(fcnt, 1u) + 1u == (uint32_t)a.fwd_gx) {
            __hip_atomic_store(fcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gate, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}


// Positions of every entry's row in every rank's table section: workgroup (table t, slot s, chunk
// k) owns the block-aligned row range [row_lo, row_hi) of slot s (the slot's blocks cut in K_t
// chunks); for each rank's entry e of that range, pos[(r * cap_total + cap_base[t] + e) * N + j]
// = the entry of the same row in rank j's table section, or -1.
__global__ void __launch_bounds__(AM_TPB) k_merge_pos(dqrm_internal::MergeApplyArgs a) {
    __shared__ int s_pre[AM_MAXN];     // rank r: the slot's first entry in its table section
    __shared__ int s_cnt[AM_MAXN];     //   the slot's entries
    __shared__ int s_lo[AM_MAXN];      //   the chunk's first entry (within the slot)
    __shared__ int s_hi[AM_MAXN];      //   one past its last
    __shared__ int s_start[AM_MAXN + 1];  // prefix of the chunk's entries over the ranks
    __shared__ int32_t s_rows[AM_KEYS];   // the chunk's rows, rank by rank (when they fit)
    __shared__ int16_t s_map[AM_MAP];     // dense ranges: [rank][row - row_lo] -> entry in the run, -1
    const int tid = threadIdx.x, lane = tid % WAVE, w = tid / WAVE;
    const int T = a.T, N = a.N;
    int t = 0;  // workgroup -> (table, slot, chunk): table t owns [kbase[t], kbase[t+1]), K_t per slot
    while (t + 1 < T && (int)blockIdx.x >= a.kbase[t + 1]) ++t;
    const int K = a.kt[t];
    const int local = (int)blockIdx.x - a.kbase[t];
    const int s = local / K, k = local % K;
    const int64_t nrows = a.meta[T + t];
    const uint32_t nblk = (uint32_t)((nrows + BLK - 1) / BLK);
    auto slot0 = [&](int ss) { return (uint32_t)(((uint64_t)nblk * (uint32_t)ss) >> 3); };
    const uint32_t s0 = slot0(s), nb = slot0(s + 1) - s0;
    const uint32_t b0 = s0 + nb * (uint32_t)k / (uint32_t)K, b1 = s0 + nb * (uint32_t)(k + 1) / (uint32_t)K;
    if (b0 >= b1) return;  // no rows
    const int64_t row_lo = (int64_t)b0 * BLK, row_hi = (int64_t)b1 * BLK < nrows ? (int64_t)b1 * BLK : nrows;
    const PayloadLayout pl = payload_layout(T, a.cap_total, a.D, a.bits);
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
    __syncthreads();
    if (a.diag & 4) return;
    // 2. K > 1: the chunk's run in each rank = [#rows < row_lo, #rows < row_hi) of the slot's
    //    ascending rows (every rank's slot rows loaded in one sweep, counted by ballots)
    if (K > 1) {
        int tot = 0;
        for (int r = 0; r < N; ++r) tot += s_cnt[r];
        constexpr int CPT = 8;  // rows per thread with their loads in flight together
        for (int base = 0; base < tot; base += AM_TPB * CPT) {
            int32_t xs[CPT];
            int rs[CPT], es[CPT];
#pragma unroll
            for (int c = 0; c < CPT; ++c) {  // lanes of a wave take consecutive entries
                const int i = base + c * AM_TPB + w * WAVE + lane;
                int r = N - 1, e = 0;  // lanes past the end: the last rank (ranks ascend with the lane)
                if (i < tot) {
                    r = 0;
                    e = i;
                    while (e >= s_cnt[r]) { e -= s_cnt[r]; ++r; }
                }
                rs[c] = r;
                es[c] = e;
            }
#pragma unroll
            for (int c = 0; c < CPT; ++c)  // every row load in flight together (clamped: entry 0 of a rank)
                xs[c] = rows_of(rs[c])[s_pre[rs[c]] + es[c]];
#pragma unroll
            for (int c = 0; c < CPT; ++c)
                if (base + c * AM_TPB + w * WAVE + lane >= tot) xs[c] = 0x7fffffff;
#pragma unroll
            for (int c = 0; c < CPT; ++c) {  // count per rank with masked ballots
                const int i = base + c * AM_TPB + w * WAVE + lane;
                const uint64_t blo = __ballot(xs[c] < row_lo), bhi = __ballot(xs[c] < row_hi);
                const int rfirst = __shfl(rs[c], 0, WAVE), rlast = __shfl(rs[c], WAVE - 1, WAVE);
                for (int q = rfirst; q <= rlast; ++q) {  // wave-uniform
                    const uint64_t mq = __ballot(i < tot && rs[c] == q);
                    if (lane == 0 && mq) {
                        const int nlo = __popcll(blo & mq), nhi = __popcll(bhi & mq);
                        if (nlo) atomicAdd(&s_lo[q], nlo);
                        if (nhi) atomicAdd(&s_hi[q], nhi);
                    }
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
    // 3. the chunk's rows to LDS (rank-major, each run ascending) when they fit
    if (a.diag & 8) return;
    const bool in_lds = M <= AM_KEYS;
    if (in_lds) {
        constexpr int CPY = AM_KEYS / AM_TPB;  // rows per thread, loads in flight together
        int src[CPY];
#pragma unroll
        for (int c = 0; c < CPY; ++c) {
            const int i = tid + c * AM_TPB;
            int r = 0;
            if (i < M)
                while (i >= s_start[r + 1]) ++r;
            src[c] = i < M ? s_pre[r] + s_lo[r] + (i - s_start[r]) : -1;
            src[c] = src[c] < 0 ? -1 : (src[c] | (r << 24));  // rank in the top byte (entries < 2^24)
        }
        int32_t v[CPY];
#pragma unroll
        for (int c = 0; c < CPY; ++c)
            v[c] = src[c] >= 0 ? rows_of(src[c] >> 24)[src[c] & 0xFFFFFF] : 0;
#pragma unroll
        for (int c = 0; c < CPY; ++c)
            if (src[c] >= 0) s_rows[tid + c * AM_TPB] = v[c];
        __syncthreads();
    }
    auto row_at = [&](int r, int e) -> int32_t {  // entry e of rank r's chunk run
        return in_lds ? s_rows[s_start[r] + e] : rows_of(r)[s_pre[r] + s_lo[r] + e];
    };
    // 4. every (entry, rank) pair at once: the entry's row in rank j's run (binary search of an
    //    ascending run; LDS when it fits), written as the entry index in rank j's table section
    if (a.diag & 1) return;
    const int64_t span = row_hi - row_lo;
    if (in_lds && span * N <= AM_MAP) {
        // a dense range (few rows, most held by every rank: narrow and medium tables): a row ->
        // entry map per rank in LDS, one read per (entry, rank)
        for (int i = tid; i < (int)span * N; i += AM_TPB) s_map[i] = -1;
        __syncthreads();
        for (int i = tid; i < M; i += AM_TPB) {
            int r = 0;
            while (i >= s_start[r + 1]) ++r;
            s_map[r * (int)span + (int)(s_rows[i] - row_lo)] = (int16_t)(i - s_start[r]);
        }
        __syncthreads();
        for (int i = tid; i < M; i += AM_TPB) {
            int r = 0;
            while (i >= s_start[r + 1]) ++r;
            const int e = i - s_start[r];
            const int xo = (int)(s_rows[i] - row_lo);
            const int64_t ent = (int64_t)r * a.cap_total + cb + s_pre[r] + s_lo[r] + e;
            int p[AM_MAXN];
#pragma unroll
            for (int j = 0; j < AM_MAXN; ++j) p[j] = j < N ? s_map[j * (int)span + xo] : -1;
#pragma unroll
            for (int j = 0; j < AM_MAXN; ++j)
                if (j < N) a.pos[ent * N + j] = p[j] >= 0 ? s_pre[j] + s_lo[j] + p[j] : -1;
        }
        return;
    }
    // 4. every (entry, rank) pair at once: the entry's row in rank j's run (binary search of an
    //    ascending run; LDS when it fits), written as the entry index in rank j's table section
    for (int pq = tid; pq < M * N; pq += AM_TPB) {
        const int gi = pq / N, j = pq % N;
        int r = 0;
        while (gi >= s_start[r + 1]) ++r;
        const int e = gi - s_start[r];
        int p;
        if (j == r) {
            p = e;
        } else {
            const int32_t x = row_at(r, e);
            int lo = 0, hi = s_hi[j] - s_lo[j];
            const int n = hi;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (row_at(j, mid) < x) lo = mid + 1; else hi = mid;
            }
            p = (lo < n && row_at(j, lo) == x) ? lo : -1;
        }
        const int64_t ent = (int64_t)r * a.cap_total + cb + s_pre[r] + s_lo[r] + e;
        a.pos[ent * N + j] = p >= 0 ? s_pre[j] + s_lo[j] + p : -1;
    }
}

// The update: grid (entry chunks, T, N ranks [+ the forward plane]); lane group per entry of
// rank r's table-t section, AP_INFL entries in flight.
template <int LPR, bool FWD>
__global__ void __launch_bounds__(AP_TPB) k_apply_pos(dqrm_internal::MergeApplyArgs a) {
    constexpr int D = LPR * 4;
    constexpr int G = AP_TPB / LPR;
    const int t = blockIdx.y, r = blockIdx.z;
    const int T = a.T, N = a.N;
    if constexpr (FWD) {
        if (r == N) {  // the forward plane (the grid's last z slice: dispatched after every update)
            if ((int)blockIdx.x < a.fwd_gx) merge_forward<LPR>(a, t, blockIdx.x);
            return;
        }
    }
    const PayloadLayout pl = payload_layout(T, a.cap_total, D, a.bits);
    const int64_t cb = a.cap_base[t], cap = a.cap_base[t + 1] - cb;
    const unsigned char* pr = a.payloads + (int64_t)r * a.rank_pitch;
    // every rank's entry count of table t in ONE round trip: thread j*8+q loads rank j's slot-q
    // count, 8-lane sums (slot order), clamped to the table's capacity
    __shared__ int s_cnt[AM_MAXN];
    if ((int)threadIdx.x < N * SPLIT) {
        const int j = threadIdx.x / SPLIT, q = threadIdx.x % SPLIT;
        int c = reinterpret_cast<const int32_t*>(a.payloads + (int64_t)j * a.rank_pitch)[t * SPLIT + q];
        c = c > 0 ? c : 0;
        c += __shfl_xor(c, 1, WAVE);
        c += __shfl_xor(c, 2, WAVE);
        c += __shfl_xor(c, 4, WAVE);
        if (q == 0) s_cnt[j] = c < cap ? c : (int)cap;
    }
    __syncthreads();
    const int cnt_r = s_cnt[r];
    if ((int64_t)blockIdx.x * G * AP_INFL >= cnt_r) return;
    uint32_t expected = 0;  // the table's working workgroups over all ranks (each arrives once)
    for (int j = 0; j < N; ++j) {
        const uint32_t wgs = (uint32_t)((s_cnt[j] + G * AP_INFL - 1) / (G * AP_INFL));
        expected += wgs < gridDim.x ? wgs : gridDim.x;
    }
    const int64_t rb = a.meta[t], nrows = a.meta[T + t], bb = a.meta[2 * T + t], sbb = a.meta[3 * T + t];
    const float sc = (a.mode == DQRM_UPD_FP32) ? 1.0f : a.s_avg[t];
    const ApplyUpdate upd{a.mode, (float)(1.0 / (double)N), sc, (float)((double)sc / (double)N), a.nlr};
    const float r_pack = a.repack ? 1.0f / a.pscale[t] : 0.0f;
    const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
    const int gbase = (threadIdx.x % WAVE) - sub;
    const uint64_t gmask = (LPR >= WAVE ? ~0ull : ((1ull << LPR) - 1ull)) << gbase;
    const int32_t* rows_r = reinterpret_cast<const int32_t*>(pr + pl.rows_off) + cb;
    const bool fast8 = pl.elem == 1 && N <= 8 && N <= LPR;  // every rank's position in a lane of the group
    auto value = [&](int j, int64_t e) -> float4 {  // rank j's entry e of table t, widened to f32
        const unsigned char* p = a.payloads + (int64_t)j * a.rank_pitch + pl.vals_off;
        const int64_t q = cb + e;
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
    for (int e0 = blockIdx.x * G * AP_INFL + grp; e0 < cnt_r; e0 += gridDim.x * G * AP_INFL) {
        int32_t xx[AP_INFL];
        int pj[AP_INFL];    // lane sub < N: the entry of this row in rank sub (N = 1: the entry itself)
        int ee[AP_INFL];
#pragma unroll
        for (int h = 0; h < AP_INFL; ++h) {  // the rows and their positions, in flight together
            const int e = e0 + h * G;
            ee[h] = e;
            xx[h] = e < cnt_r ? rows_r[e] : -1;
            pj[h] = -1;
            if (e < cnt_r && sub < N)
                pj[h] = N == 1 ? e : a.pos[((int64_t)r * a.cap_total + cb + e) * N + sub];
        }
        float4 w0v[AP_INFL], acc[AP_INFL];
        float ob[AP_INFL], osb[AP_INFL], otm[AP_INFL];
#pragma unroll
        for (int h = 0; h < AP_INFL; ++h) {  // ownership: no lower rank holds the row (group-uniform)
            bool lower = sub < r && pj[h] >= 0;
            for (int j = sub + LPR; j < r && xx[h] >= 0; j += LPR)  // more ranks than lanes (rare)
                lower |= a.pos[((int64_t)r * a.cap_total + cb + ee[h]) * N + j] >= 0;
            if (__ballot(lower) & gmask) xx[h] = -1;
            if (xx[h] >= 0 && (xx[h] >= nrows)) {  // cannot happen for payloads this library packed
                if (sub == 0) flag_error(a.err, DQRM_ERRF_INDEX);
                xx[h] = -1;
            }
        }
#pragma unroll
        for (int h = 0; h < AP_INFL; ++h) {  // W rows and the maxima they are tested against
            w0v[h] = make_float4(0.f, 0.f, 0.f, 0.f);
            ob[h] = osb[h] = otm[h] = 0.0f;
            if (xx[h] < 0) continue;
            const int64_t x = xx[h];
            w0v[h] = reinterpret_cast<const float4*>(a.W + (rb + x) * D)[sub];
            ob[h] = a.blkmax[bb + (x >> 8)];
            osb[h] = a.sblkmax[sbb + (x >> 16)];
            otm[h] = a.tmax[t];
        }
        if (fast8) {  // int8: every rank's value of the rows in one round trip, summed in rank order
            uint32_t raw[AP_INFL][8];
#pragma unroll
            for (int h = 0; h < AP_INFL; ++h)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = __shfl(pj[h], gbase + (j < LPR ? j : 0), WAVE);  // lane j of the group
                    const bool ok = xx[h] >= 0 && j < N && j < LPR && p >= 0;
                    const int jj = ok ? j : 0;
                    const int64_t q = ok ? cb + p : 0;
                    raw[h][j] = reinterpret_cast<const uint32_t*>(a.payloads + (int64_t)jj * a.rank_pitch +
                                                                  pl.vals_off + q * D)[sub];
                    if (!ok) raw[h][j] = 0u;  // absent: +0 to an integer sum (never -0)
                }
#pragma unroll
            for (int h = 0; h < AP_INFL; ++h) {
                acc[h] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t x = raw[h][j];
                    acc[h].x += (float)(int8_t)(x & 0xFF); acc[h].y += (float)(int8_t)((x >> 8) & 0xFF);
                    acc[h].z += (float)(int8_t)((x >> 16) & 0xFF); acc[h].w += (float)(int8_t)(x >> 24);
                }
            }
        } else {  // int16 / FP32 / N > 8: ascending rank order, FP32 in Gloo's order
#pragma unroll
            for (int h = 0; h < AP_INFL; ++h) {
                acc[h] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (xx[h] < 0) continue;
                bool first = true;
                for (int j = r; j < N; ++j) {
                    const int p = j < LPR ? __shfl(pj[h], gbase + j, WAVE)
                                          : a.pos[((int64_t)r * a.cap_total + cb + ee[h]) * N + j];
                    if (p < 0) continue;
                    const float4 v = value(j, p);
                    if (first) { acc[h] = v; first = false; }
                    else { acc[h].x += v.x; acc[h].y += v.y; acc[h].z += v.z; acc[h].w += v.w; }
                }
            }
        }
#pragma unroll
        for (int h = 0; h < AP_INFL; ++h) {
            if (xx[h] < 0) continue;
            const int64_t x = xx[h], grow = rb + x, blk = x >> 8, sb = sbb + (x >> 16);
            float4 wn;
            wn.x = upd(w0v[h].x, acc[h].x); wn.y = upd(w0v[h].y, acc[h].y);
            wn.z = upd(w0v[h].z, acc[h].z); wn.w = upd(w0v[h].w, acc[h].w);
            // write-through: the forward plane and the finalize (narrow tables) read it in this launch
            if (FWD || nrows <= BLK)
                st4_wt(reinterpret_cast<float4*>(a.W + grow * D) + sub, wn);
            else
                reinterpret_cast<float4*>(a.W + grow * D)[sub] = wn;
            if (a.repack) pack4_row(wn, a.packed + grow * (D / 2), sub, r_pack);
            const float old_rm = group_max<LPR>(abs_max4(w0v[h]));
            const float rm = group_max<LPR>(abs_max4(wn));
            if (sub != 0) continue;
            st_wt(a.rowmax + grow, rm);
            if (rm > ob[h]) {  // growth: order-free atomicMax on the non-negative float bits
                atomicMax(reinterpret_cast<unsigned int*>(a.blkmax) + bb + blk, __float_as_uint(rm));
                if (rm > osb[h]) {
                    atomicMax(reinterpret_cast<unsigned int*>(a.sblkmax) + sb, __float_as_uint(rm));
                    if (rm > otm[h]) atomicMax(reinterpret_cast<unsigned int*>(a.tmax) + t, __float_as_uint(rm));
                }
            }
            if (old_rm == ob[h] && rm < old_rm) {  // the block's max holder shrank: the finalize re-reduces it
                flag_set(a.bdirty, bb + blk);
                flag_set(a.sdirty, sb);
                mark_table_flagged(a.sync, t);
            }
        }
    }
    // one arrival per working workgroup (hand-off row 1); the last one finalizes the table's
    // hierarchy if any workgroup flagged it, then opens the table's forward gate
    if (arrive_last(a.sync + (int64_t)t * DQRM_SYNC_STRIDE, expected)) {
        __shared__ int s_flag;
        if (threadIdx.x == 0) {
            uint32_t* fw = a.sync + (int64_t)t * DQRM_SYNC_STRIDE + FLAG_WORD;
            s_flag = ld_wt(fw) != 0u;
            if (s_flag) __hip_atomic_store(fw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (s_flag)
            finalize_table<true>(make_meta(a.meta, T), t, a.W, a.rowmax, a.blkmax, a.sblkmax, a.sdirty, a.bdirty,
                                 a.tmax, D, true, false);
        if constexpr (FWD) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the finalize's stores landed
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_store(a.sync + (int64_t)t * DQRM_SYNC_STRIDE + GATE_WORD, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

namespace dqrm_internal {

hipError_t launch_apply_merge(const MergeApplyArgs& a, hipStream_t stream) {
    if (a.N < 1 || a.N > AM_MAXN || a.T < 1 || a.T > kMergeMaxTables) return hipErrorInvalidValue;
    if (a.N > 1 && !a.pos) return hipErrorInvalidValue;
    const bool fwd = a.fwd_idx != nullptr;
    if (fwd && (a.fwd_gx < 1 || a.fwd_B < 1)) return hipErrorInvalidValue;
    if (a.N > 1) hipLaunchKernelGGL(k_merge_pos, dim3((unsigned)a.kbase[a.T]), dim3(AM_TPB), 0, stream, a);
    const dim3 grid((unsigned)(a.gx > (fwd ? a.fwd_gx : 0) ? a.gx : a.fwd_gx), (unsigned)a.T,
                    (unsigned)(a.N + (fwd ? 1 : 0)));
    switch (a.D) {
#define AP_CASE(Dd)                                                                                        \
    case Dd:                                                                                               \
        if (fwd) hipLaunchKernelGGL((k_apply_pos<Dd / 4, true>), grid, dim3(AP_TPB), 0, stream, a);      \
        else hipLaunchKernelGGL((k_apply_pos<Dd / 4, false>), grid, dim3(AP_TPB), 0, stream, a);         \
        break;
        AP_CASE(4) AP_CASE(8) AP_CASE(16) AP_CASE(32) AP_CASE(64) AP_CASE(128) AP_CASE(256)
#undef AP_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int merge_forward_gx(int64_t B) {  // forward workgroups per table: ~128 bags each, 1..64
    constexpr int bags = (AM_TPB / 16) * FWD_UNR * 2;
    int64_t g = (B + bags - 1) / bags;
    return (int)(g < 1 ? 1 : (g > 64 ? 64 : g));
}

size_t apply_workspace_bytes(int num_ranks, int64_t cap_total) {
    return num_ranks > 1 ? (size_t)num_ranks * (size_t)num_ranks * (size_t)cap_total * sizeof(int32_t) : 0;
}

}  // namespace dqrm_internal
