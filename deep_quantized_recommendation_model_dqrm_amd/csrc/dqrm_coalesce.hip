// dqrm_coalesce.hip — K4 coalesce for Criteo-form batches (gfx950).
//
//   STE backward        SymmetricQuantFunction.backward   quant_utils.py:349-363
//   sparse backward     nn.EmbeddingBag(mode="sum", sparse=True), one lookup per bag
//   grad.coalesce()     + per-table max|grad| for the local scale   s_q_g_p_c.py:859-861
//
// One 1024-thread workgroup per (table, row-range slot), exactly the general kernel's
// workspace contract (include/dqrm.h, dqrm_emb_bwd_coalesce), for batches in the Criteo
// form (DQRM_BATCH_POOLING_ONE, B <= 4096 lookups per table): bag b is lookup b, so a
// lookup's dy row is known from its position alone. The kernel is built for latency: at
// 2048 lookups per table every workgroup does a few hundred keys, so what costs is the
// chain of dependent steps and the instructions each wave issues, not bandwidth.
//   1. every thread's lookups (b = tid + 1024 i) are loaded at once;
//   2. a dimension-split table (fewer than 8 row blocks: every workgroup sees all lookups
//      and owns D/8 of the dimensions) issues its dy slice of every lookup right behind the
//      index loads (a row-split slot issues as many placeholder loads, so the compiler waits
//      for the index loads alone); the slot's lookups are compacted in lookup order (ballots
//      + a DPP scan), keys = (row - r0) << 32 | gather index << 12 | lookup; a row-split
//      slot then issues its lookups' dy rows, in flight across the sort;
//   3. rows are COUNTED, not compared, for row spans up to CSPAN rows: spans <= 256 by
//      per-wave row counters + bit-sliced same-row ballots (a stable radix pass), larger
//      ones by LDS row counters (arrival rank) re-ranked inside each row's bucket by lookup
//      order; one block scan of the per-row (lookups, distinct rows, multi-lookup rows)
//      prefixes then gives every segment's start, output entry and stage place directly.
//      Wider spans: an MSD bucket sort; a crowded bucket (hot row) falls back to the stable
//      LSD radix sort. Either way the order is the reference's: rows ascending, a row's
//      lookups in lookup order;
//   4. single-lookup segments are stored straight from registers; the others land in a
//      DIMENSION-MAJOR stage at their sorted positions and item (segment, dimension) = one
//      lane sums its column strictly in lookup order (16 LDS values in flight ahead of the
//      adds). Slots too large for the stage stream it in chunks (the same lane carries a
//      segment across chunks).
// A table's 8 slots run on one XCD (block map below), so dy lines shared by the slices of a
// dimension-split table come from one L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdint.h>

#include "../../include/dqrm.h"
#include "dqrm_device.h"
#include "dqrm_internal.h"

namespace {

// Diagnostic build only (-DDQRM_DIAG_CLOCK, tools/diag_coalesce.py): thread 0 of every
// workgroup stamps the 100 MHz wall clock at phase boundaries.
#ifdef DQRM_DIAG_CLOCK
__device__ unsigned long long g_coal_clk[8192 * 32];
#define CDIAG(ph) do { if (threadIdx.x == 0) g_coal_clk[kd * 32 + (ph)] = wall_clock64(); } while (0)
#define CDIAG_W(ph) do { __builtin_amdgcn_s_waitcnt(0); CDIAG(ph); } while (0)
#else
#define CDIAG(k) do { } while (0)
#define CDIAG_W(k) do { } while (0)
#endif

#ifndef DQRM_COAL_TPB
#define DQRM_COAL_TPB 1024
#endif
#ifndef DQRM_COAL_PFR
#define DQRM_COAL_PFR 6
#endif
constexpr int TPB = DQRM_COAL_TPB;
constexpr int NW = TPB / WAVE;
constexpr int SPLIT = DQRM_TABLE_SPLIT;
static_assert(SPLIT == 8, "the XCD-aware block map puts a table's SPLIT slots on one XCD");
constexpr int MAXB = (int)dqrm_internal::kCoalesceMaxB;
constexpr int MAXI = MAXB / TPB;  // lookups per thread
constexpr int PFR = DQRM_COAL_PFR;  // prefetched float4 per thread
constexpr int DBMAX = TPB >= 512 ? 9 : 8;  // radix digit bits per pass (one digit per thread in the scan)
static_assert(TPB >= 256, "the MSD pass gives each of its 256 buckets a thread");
constexpr int FIX_MAX = 64;       // largest bucket the MSD pass finishes by ranking
#ifndef DQRM_COAL_CSPAN
#define DQRM_COAL_CSPAN 4096
#endif
constexpr int CSPAN = DQRM_COAL_CSPAN;  // largest row span sorted by counting rows (0: never)
#ifndef DQRM_COAL_UNIQ
#define DQRM_COAL_UNIQ 1  // 0: an A/B build without the one-launch step's distinct-rows fast path
#endif
constexpr int UNIQ_MAXN = TPB;      // fast path: at most one lookup per thread
constexpr int UNIQ_HLOG = 12;       // its LDS hash: 4096 slots
constexpr int UNIQ_HASH = 1 << UNIQ_HLOG;
constexpr int RPT = CSPAN > 0 ? (CSPAN + TPB - 1) / TPB : 1;  // rows per thread in the row scan
constexpr int LDS_BYTES = 156 * 1024;
// dynamic LDS: keys u64[MAXB] | while sorting: ping-pong u64[MAXB] + digit counters
// i32[NW << DBMAX]; after it: sorted position of each lookup u16[MAXB] | segment heads
// u16[MAXB+8] | multi-lookup segments u16[MAXB+8] | output entry of each sorted position
// i32[MAXB] (-1: part of a multi-lookup segment) | dimension-major stage f32
constexpr int OFF_SCR = MAXB * 8;
constexpr int OFF_POS = OFF_SCR;
constexpr int OFF_HPOS = OFF_POS + MAXB * 2;
constexpr int OFF_MLIST = OFF_HPOS + (MAXB + 8) * 2;
constexpr int OFF_SDEST = OFF_MLIST + (MAXB + 8) * 2;
constexpr int OFF_STAGE = OFF_SDEST + MAXB * 4;
constexpr int STAGE_FLOATS = (LDS_BYTES - OFF_STAGE) / 4;
static_assert(OFF_STAGE % 16 == 0, "stage alignment");
// counting path: per-row packed prefix (lookups | distinct rows << 16) and multi-lookup
// prefix, [CSPAN + 1] each, at the start of the stage (which is filled only after them)
constexpr int OFF_INFO = OFF_STAGE;
constexpr int OFF_MINFO = OFF_INFO + (CSPAN + 4) * 4;
static_assert(OFF_MINFO + (CSPAN + 4) * 4 <= LDS_BYTES, "row counters");
static_assert(MAXB < 65536 && CSPAN < 65536, "16-bit packed row prefixes");
static_assert(OFF_SCR + MAXB * 8 + (NW << DBMAX) * 4 <= LDS_BYTES, "sort scratch");
static_assert(MAXI * NW <= WAVE, "one prefix lane per (item, wave)");
// key = (row - r0) << 32 | gather index << 12 | lookup: unique, and gather order = lookup order
constexpr uint32_t LK_BITS = 12;
constexpr uint32_t LK_MASK = (1u << LK_BITS) - 1u;
static_assert(MAXB <= (1 << LK_BITS), "lookup index field");

__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << (threadIdx.x % WAVE)) - 1ull; }
// the wave index as a scalar (uniform) value, for v_readlane broadcasts
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE)); }
__device__ __forceinline__ int lane_of(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// inclusive prefix sum over the 64 lanes by DPP row shifts and row broadcasts (no LDS
// permutes); every lane must be active
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ uint32_t krow(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint32_t kgat(uint64_t x) { return (uint32_t)x >> LK_BITS; }
__device__ __forceinline__ uint32_t kbag(uint64_t x) { return (uint32_t)x & LK_MASK; }
// 16-B load of bytes another workgroup of the launch stored write-through (sc1): an sc1
// buffer load (L2-served, past this CU's L1), tracked by the compiler's vmcnt accounting
__device__ __forceinline__ float4 ld4_sc1(const float* base, uint32_t byte_off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16 /* sc1 */);
    return make_float4(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]), __uint_as_float(x[3]));
}

// Items (i, tid), i < ni, in the order i * TPB + tid: the ones whose pred holds get
// consecutive positions in that order (emit(i, position)); every item also sees the
// position the next hit would get and whether it hit (all(i, rank, hit)). Returns the count.
template <class Pred, class Emit, class All>
__device__ __forceinline__ int ordered_compact(int ni, int* s_cnt, Pred pred, Emit emit, All all) {
    const int lane = threadIdx.x % WAVE, w = wave_id();
    uint64_t m[MAXI];
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
        m[i] = 0;
        if (i < ni) m[i] = __ballot(pred(i));
    }
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < MAXI; ++i)
            if (i < ni) s_cnt[i * NW + w] = (int)__popcll(m[i]);
    __syncthreads();
    const int v = lane < ni * NW ? s_cnt[lane] : 0;
    const int incl = wave_incl_scan(v);
    const int excl = incl - v;
    const int total = lane_of(incl, WAVE - 1);
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
        const int base = lane_of(excl, (i * NW + w) & (WAVE - 1));
        const bool hit = (m[i] >> lane) & 1ull;
        const int rank = base + (int)__popcll(m[i] & lt);
        if (i < ni) {
            if (hit) emit(i, rank);
            all(i, rank, hit);
        }
    }
    return total;
}

// exclusive prefix of one int per thread over the workgroup; *total = the sum
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int* total) {
    const int lane = threadIdx.x % WAVE, w = wave_id();
    const int incl = wave_incl_scan(v);
    if (lane == WAVE - 1) s_w[w] = incl;
    __syncthreads();
    if (w == 0) {
        const int x = lane < NW ? s_w[lane] : 0;
        const int y = wave_incl_scan(x);
        if (lane < NW) s_w[lane] = y - x;
        if (lane == NW - 1) s_w[NW] = y;
    }
    __syncthreads();
    *total = s_w[NW];
    return s_w[w] + incl - v;
}

// block_excl_scan of two ints at once (shared barriers)
__device__ __forceinline__ void block_excl_scan2(int v1, int v2, int* s_w, int* s_w2, int& e1, int& e2,
                                                 int& t1, int& t2) {
    const int lane = threadIdx.x % WAVE, w = wave_id();
    const int i1 = wave_incl_scan(v1), i2 = wave_incl_scan(v2);
    if (lane == WAVE - 1) { s_w[w] = i1; s_w2[w] = i2; }
    __syncthreads();
    if (w == 0) {
        const int x1 = lane < NW ? s_w[lane] : 0, x2 = lane < NW ? s_w2[lane] : 0;
        const int y1 = wave_incl_scan(x1), y2 = wave_incl_scan(x2);
        if (lane < NW) { s_w[lane] = y1 - x1; s_w2[lane] = y2 - x2; }
        if (lane == NW - 1) { s_w[NW] = y1; s_w2[NW] = y2; }
    }
    __syncthreads();
    t1 = s_w[NW];
    t2 = s_w2[NW];
    e1 = s_w[w] + i1 - v1;
    e2 = s_w2[w] + i2 - v2;
}

// Stable LSD radix sort of keys[0, n) by the row field (bits [0, nbits)), passes of at
// most DBMAX bits (a dimension-split table's rows: one pass). Wave w owns keys
// [w*64*kpl, (w+1)*64*kpl), 64 at a time; same-digit lanes from bit-slice ballots;
// [digit][wave] counters, one workgroup scan per pass.
__device__ void radix_sort(uint64_t* keys, uint64_t* tmp, int* hist, int* s_w, int n, int nbits) {
    const int tid = threadIdx.x, lane = tid % WAVE, w = tid / WAVE;
    const int kpl = (n + TPB - 1) / TPB;
    const int i0 = w * WAVE * kpl + lane;
    const uint64_t lt = lanemask_lt();
    const int passes = (nbits + DBMAX - 1) / DBMAX;
    uint64_t* src = keys;
    uint64_t* dst = tmp;
    int sh = 0;
    for (int ps = 0; ps < passes; ++ps) {
        const int db = (nbits - sh + (passes - ps) - 1) / (passes - ps);
        const uint32_t dm = (1u << db) - 1u;
        const int nd = 1 << db;
        for (int j = tid; j < (NW << db); j += TPB) hist[j] = 0;
        __syncthreads();
        auto peers_of = [&](uint32_t d, bool v) {
            uint64_t m = __ballot(v);
            for (int q = 0; q < db; ++q) {
                const uint64_t bq = __ballot((d >> q) & 1u);
                m &= ((d >> q) & 1u) ? bq : ~bq;
            }
            return m;
        };
        for (int kk = 0; kk < kpl; ++kk) {
            const int i = i0 + kk * WAVE;
            const bool v = i < n;
            const uint32_t d = v ? (krow(src[i]) >> sh) & dm : 0u;
            const uint64_t pm = peers_of(d, v);
            if (v && (pm & lt) == 0) hist[w * nd + d] += (int)__popcll(pm);
        }
        __syncthreads();
        {  // exclusive scan in (digit, wave) order: thread d owns digit d's NW counters
            int c[NW];
            int sum = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                c[q] = tid < nd ? hist[q * nd + tid] : 0;
                sum += c[q];
            }
            int tot;
            int ex = block_excl_scan(sum, s_w, &tot);
            if (tid < nd)
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    hist[q * nd + tid] = ex;
                    ex += c[q];
                }
        }
        __syncthreads();
        for (int kk = 0; kk < kpl; ++kk) {
            const int i = i0 + kk * WAVE;
            const bool v = i < n;
            const uint64_t x = v ? src[i] : 0ull;
            const uint32_t d = (krow(x) >> sh) & dm;
            const uint64_t pm = peers_of(d, v);
            if (v) {
                int* hp = hist + w * nd + d;
                const int p = *hp + (int)__popcll(pm & lt);
                dst[p] = x;
                if ((pm & lt) == 0) *hp = p + (int)__popcll(pm);
            }
        }
        __syncthreads();
        uint64_t* tt = src;
        src = dst;
        dst = tt;
        sh += db;
    }
    if (src != keys) {
        for (int i = tid; i < n; i += TPB) keys[i] = src[i];
        __syncthreads();
    }
}

// Keys over a row span of more than 8 bits: one counting pass on the top 8 bits of the row
// into 256 buckets (rank inside a bucket from an LDS atomic: any order), then every key's
// place inside its bucket = the number of smaller keys there (the keys are unique, so this
// is THE sorted order; a bucket is read by its own keys only, all reads independent). A
// bucket above FIX_MAX keys (hot rows) -> radix_sort.
__device__ void msd_sort(uint64_t* keys, uint64_t* tmp, int* hist, int* s_w, int n, int nbits) {
    const int tid = threadIdx.x;
    const int sh = nbits - 8;
    int* cnt = hist;          // [256]
    int* start = hist + 256;  // [257]
    int* flag = hist + 520;
    if (tid < 256) cnt[tid] = 0;
    if (tid == 0) *flag = 0;
    __syncthreads();
    uint64_t x[MAXI];
    int d[MAXI], rk[MAXI];
#pragma unroll
    for (int j = 0; j < MAXI; ++j) {
        const int i = tid + TPB * j;
        d[j] = -1;
        x[j] = 0;
        rk[j] = 0;
        if (i < n) {
            x[j] = keys[i];
            d[j] = (int)((krow(x[j]) >> sh) & 255u);
            rk[j] = atomicAdd(&cnt[d[j]], 1);
        }
    }
    __syncthreads();
    const int c = tid < 256 ? cnt[tid] : 0;
    int tot;
    const int ex = block_excl_scan(c, s_w, &tot);
    if (tid < 256) {
        start[tid] = ex;
        if (c > FIX_MAX) *flag = 1;
    }
    if (tid == 0) start[256] = tot;
    __syncthreads();
    const bool crowded = *flag != 0;
    __syncthreads();
    if (crowded) {
        radix_sort(keys, tmp, hist, s_w, n, nbits);
        return;
    }
#pragma unroll
    for (int j = 0; j < MAXI; ++j)
        if (d[j] >= 0) tmp[start[d[j]] + rk[j]] = x[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXI; ++j)
        if (d[j] >= 0) {
            const int b0 = start[d[j]], b1 = start[d[j] + 1];
            int below = 0;
            for (int i = b0; i < b1; ++i) below += tmp[i] < x[j] ? 1 : 0;
            keys[b0 + below] = x[j];
        }
    __syncthreads();
}

// row-range slot of a row (slot_rows' inverse): the largest s with floor(nblk*s/SPLIT) <= blk
__device__ __forceinline__ int slot_of_row(int64_t row, int64_t nblk) {
    const uint32_t blk = (uint32_t)(row >> 8), nb = (uint32_t)nblk;
    return (int)((SPLIT * (blk + 1) + nb - 1) / nb) - 1;
}

#ifndef DQRM_COAL_CH
#define DQRM_COAL_CH 16
#endif
constexpr int CH4 = DQRM_COAL_CH / 4;  // float4 of an ordered chain in flight

// acc + col[p] + col[p+1] + ... + col[pe-1], strictly in order; 16-B reads, the next
// 4*CH4 values in flight while the current 4*CH4 are added (col 16-B aligned)
__device__ __forceinline__ float chain_sum(const float* col, int p, int pe, float acc) {
    for (; p < pe && (p & 3); ++p) acc = acc + col[p];
    if (p + 4 * CH4 <= pe) {
        float4 x[CH4];
#pragma unroll
        for (int j = 0; j < CH4; ++j) x[j] = reinterpret_cast<const float4*>(col + p)[j];
        p += 4 * CH4;
        while (p + 4 * CH4 <= pe) {
            float4 y[CH4];
#pragma unroll
            for (int j = 0; j < CH4; ++j) y[j] = reinterpret_cast<const float4*>(col + p)[j];
#pragma unroll
            for (int j = 0; j < CH4; ++j) {
                acc = acc + x[j].x; acc = acc + x[j].y; acc = acc + x[j].z; acc = acc + x[j].w;
                x[j] = y[j];
            }
            p += 4 * CH4;
        }
#pragma unroll
        for (int j = 0; j < CH4; ++j) {
            acc = acc + x[j].x; acc = acc + x[j].y; acc = acc + x[j].z; acc = acc + x[j].w;
        }
    }
    for (; p + 4 <= pe; p += 4) {
        const float4 v = *reinterpret_cast<const float4*>(col + p);
        acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
    }
    for (; p < pe; ++p) acc = acc + col[p];
    return acc;
}

// the same sum over a ROW-MAJOR stage: c[p * stride], p in [p, pe), strictly in order, G LDS
// reads in flight while the previous G are added (measured: G = 16 / 32, or batches predicated
// to the chain's end, were slower on the 680-long chains of the 3-row tables)
#ifndef DQRM_COAL_RMG
#define DQRM_COAL_RMG 8
#endif
__device__ __forceinline__ float chain_sum_rm(const float* c, int p, int pe, int stride, float acc) {
    constexpr int G = DQRM_COAL_RMG;
    if (p + G <= pe) {
        float x[G];
#pragma unroll
        for (int j = 0; j < G; ++j) x[j] = c[(p + j) * stride];
        p += G;
        while (p + G <= pe) {
            float y[G];
#pragma unroll
            for (int j = 0; j < G; ++j) y[j] = c[(p + j) * stride];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                acc = acc + x[j];
                x[j] = y[j];
            }
            p += G;
        }
#pragma unroll
        for (int j = 0; j < G; ++j) acc = acc + x[j];
    }
    for (; p < pe; ++p) acc = acc + c[p * stride];
    return acc;
}

// Stage layout. Row-major: sorted position / entry p's SW floats contiguous, so a float4 lands
// with one conflict-free ds_write_b128 and a chain's 64 dimensions are 64 consecutive dwords;
// dimension-major: column d holds dimension d of every position, so a float4 is 4 stores 4*SP
// floats apart (8-way bank conflicts at SW = 64) but a chain is read 16 B at a time -- what
// the long chains of a dimension-split table (a few rows, hundreds of lookups each) want; at
// SW = 16 the dimension-major stores conflict only 2-way. Measured (same box, bench step):
// row-major -1.0 us at D = 64 (terabyte), +2 us at D = 16 (kaggle). The layout is a template
// parameter of the kernel (a per-workgroup runtime choice cost more than either layout):
// DQRM_COAL_ROWMAJOR 1 (default) row-major for D >= 32; 0 never, 2 always (A/B builds).
#ifndef DQRM_COAL_ROWMAJOR
#define DQRM_COAL_ROWMAJOR 1
#endif
// A dimension-split table's workgroup stages its slice (SW = D/8 floats per position) for a
// few rows with hundreds of lookups each: its cost is the ordered chains, which read 16 B at a
// time from a dimension-major stage (4 positions per LDS read) but 4 B from a row-major one.
// DQRM_COAL_DSDM 1: such workgroups take the dimension-major stage under RM too -- in the
// N > 1 coalesce (APPLY false; TB forced-collectives step 60.4 -> 56.5 us, A/B r5j). In the
// one-launch step the runtime layout choice cost every table ~1.5 us (38.4 -> 40.7 us/step),
// so that kernel keeps the compile-time layout.
#ifndef DQRM_COAL_DSDM
#define DQRM_COAL_DSDM 1
#endif

#ifndef DQRM_COAL_WPF
#define DQRM_COAL_WPF 4
#endif
#ifndef DQRM_FWD_EARLY_IDX
#define DQRM_FWD_EARLY_IDX 0
#endif
#ifndef DQRM_COAL_WLATE
#define DQRM_COAL_WLATE 0  // 1: an A/B build issuing the W prefetch after the land phase
#endif
#ifndef DQRM_COAL_CAND
#define DQRM_COAL_CAND 0  // A/B builds: 1 prefetch candidate blocks' row maxima during the rendezvous,
#endif                    // 2 the same unless the table already met
constexpr int WPF = DQRM_COAL_WPF;  // fused update: W float4 per thread loaded during the segment phase
constexpr int WPFA = WPF > 0 ? WPF : 1;  // array extent (WPF = 0: no early W loads, an A/B build)
constexpr int OWN_Q = 64;           // fused update: shrunk block-max holders re-reduced in the launch
constexpr int SBC = 256;            // fused update: superblock maxima of the slot's rows cached in LDS
constexpr int CAND_SLOTS = 2 * (MAXB * 2) / (BLK * 4);  // row-max caches of candidate blocks (pos + mlist regions)
static_assert(CAND_SLOTS == 16 && CAND_SLOTS <= NW, "one candidate-block cache per wave");
constexpr int GRAN_WORD = 32;       // the table's 16 slot granules (8 slots x 2 sub-slots) in its sync words
static_assert(GRAN_WORD + 2 * SPLIT * 2 <= DQRM_SYNC_STRIDE, "granules fit the table's sync words");
constexpr uint32_t DIRTY_ONE = 1u << 16;  // arrival counter (sync word 0): arrivals | dirty arrivals << 16

// Sub-slots (APPLY only). The grid has (T+7)/8*8 groups of 8 workgroups (one XCD each); group
// g < T is table g's 8 row-range slots, and the spare groups g >= T each give one of the
// largest row-split tables a SECOND workgroup per slot (la.sub_table / la.sub_mask, planned on
// the host from the tables' row counts: >= 16 row blocks, by row blocks, ties by index):
// slot s's blocks are halved, sub-slot 0 takes the lower half, the spare group's workgroup s
// (sub-slot 1) the upper. The big tables' slots are bound by the bytes one CU moves (dy rows
// in, W rows read and written), so halving them shortens the launch; the workspace contract
// (DQRM_TABLE_SPLIT slots per table) is unchanged: after the rendezvous the sub-slots' counts
// (carried in their granules) place sub-slot 1's rows after sub-slot 0's.

// granule of a slot: {max|grad| bits, distinct rows (13 bits), launch epoch (19 bits)}, one 8-B
// sc1 store (data-tagged: no ordering needed for its contents)
constexpr uint32_t GR_EPOCH_MASK = (1u << 19) - 1u;
__device__ __forceinline__ uint32_t gr_epoch(uint64_t g) { return (uint32_t)(g >> 45); }
__device__ __forceinline__ int gr_count(uint64_t g) { return (int)((g >> 32) & 0x1FFFu); }
__device__ __forceinline__ uint64_t gr_make(float m, int count, uint32_t epoch) {
    return (uint64_t)__float_as_uint(m) | ((uint64_t)((uint32_t)count & 0x1FFFu) << 32) |
           ((uint64_t)(epoch & GR_EPOCH_MASK) << 45);
}
static_assert(MAXB < (1 << 13), "distinct-row count field of a granule");


constexpr int STALL_WORD = 3;  // a table's sync word: bit (s + 8 j) = workgroup (slot s, sub-slot j) stalled
// fused next-batch forward: sync words 4-5 hold the table's final |W| max as a granule
// {max bits, launch epoch}, stored by the table's last arriver after its finalize
constexpr int FWD_WORD = 4;
static_assert(FWD_WORD % 2 == 0 && FWD_WORD + 2 <= GRAN_WORD, "8-B word below the slot granules");

// The table's last-arriving workgroup, when some of the table's workgroups gave up waiting at
// the rendezvous (stall_mask): every workgroup published its granule before it arrived, so the
// table scale is known now; the stalled workgroups' entries (left in the workspace: rows, and
// values the stalled workgroup spilled or a dimension-split table's workgroups stored) are
// quantized and applied here with dqrm_apply_local's arithmetic, their blocks flagged for the
// finalize that follows (the rows are not this workgroup's). The table's update is then
// complete -- never half-applied; DQRM_ERRF_STALL still reports the stall.
__device__ __forceinline__ void recover_stalled(const dqrm_internal::CoalesceArgs& a, const dqrm_internal::LocalApplyArgs& la,
                                             int t, uint32_t stall_mask, const uint64_t* gran, int NG, int K,
                                             bool dsplit, int NA, int64_t nblk, const int64_t* s_cb) {
    __shared__ float s_sv;
    __shared__ int s_cnt_g[2 * SPLIT];
    const int tid = threadIdx.x;
    if (tid < WAVE) {  // the table scale from every granule (all published by now)
        const uint64_t g = tid < NG ? __hip_atomic_load(gran + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const float am = wave_max(tid < NG ? __uint_as_float((uint32_t)g) : 0.0f);
        if (tid < NG) s_cnt_g[tid] = gr_count(g);
        if (tid == 0) {
            s_sv = sym_scale(am, la.bits) * (float)(1.0 / 1.0);
            la.s_avg[t] = s_sv;
        }
        if (K == 2 && tid < SPLIT && ((stall_mask >> tid) & 1u)) {  // sub-slot 0 stalled: its slot's count / max
            const uint64_t g1 = __hip_atomic_load(gran + SPLIT + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int c = gr_count(g) + gr_count(g1);
            const int64_t cap = s_cb[tid + 1] - s_cb[tid];
            c = c < cap ? c : (int)cap;
            a.ws_ucount[t * SPLIT + tid] = c;
            a.ws_absmax[t * SPLIT + tid] = fmaxf(__uint_as_float((uint32_t)g), __uint_as_float((uint32_t)g1));
        }
    }
    __syncthreads();
    const float sv = s_sv, rr = 1.0f / sv;
    const float qlo = -(float)(1 << (la.bits - 1)), qhi = (float)((1 << (la.bits - 1)) - 1);
    const ApplyUpdate upd{DQRM_UPD_DP, 1.0f, sv, sv, la.nlr};
    const float r_pack = la.repack ? 1.0f / la.pscale[t] : 0.0f;
    const int D = a.D, LPR = D / 4, lpr_sh = __ffs(LPR) - 1;
    const int64_t rb = a.meta[t], nrows = a.meta[a.T + t], bb = a.meta[2 * a.T + t], sbb = a.meta[3 * a.T + t];
    (void)nblk;
    auto apply_range = [&](int64_t e0, int64_t e1) {  // workspace entries [e0, e1)
        for (int64_t q = tid; q < ((e1 - e0) << lpr_sh); q += TPB) {
            const int64_t e = e0 + (q >> lpr_sh);
            const int sub = (int)(q & (LPR - 1));
            const int64_t x = (int64_t)(int32_t)ld_wt(reinterpret_cast<const uint32_t*>(a.ws_rows + e));
            const float4 v = ld4_sc1(a.ws_vals + e * D, (uint32_t)sub * 16u);
            const bool ok = x >= 0 && x < nrows;
            const int64_t grow = rb + (ok ? x : 0);
            const float4 w0 = reinterpret_cast<const float4*>(la.W + grow * D)[sub];
            float4 acc, wn;
            acc.x = fake_quant(v.x, rr, qlo, qhi) + 0.0f; acc.y = fake_quant(v.y, rr, qlo, qhi) + 0.0f;
            acc.z = fake_quant(v.z, rr, qlo, qhi) + 0.0f; acc.w = fake_quant(v.w, rr, qlo, qhi) + 0.0f;
            wn.x = upd(w0.x, acc.x); wn.y = upd(w0.y, acc.y); wn.z = upd(w0.z, acc.z); wn.w = upd(w0.w, acc.w);
            if (ok) {  // write-through: a fused forward may read the row from another CU
                st4_wt(reinterpret_cast<float4*>(la.W + grow * D) + sub, wn);
                if (la.repack) pack4_row(wn, la.packed + grow * (D / 2), sub, r_pack);
            }
            float old_rm = abs_max4(w0), rm = abs_max4(wn);
            for (int o = 1; o < LPR; o <<= 1) {
                old_rm = fmaxf(old_rm, __shfl_xor(old_rm, o, WAVE));
                rm = fmaxf(rm, __shfl_xor(rm, o, WAVE));
            }
            if (sub != 0 || !ok) continue;
            st_wt(la.rowmax + grow, rm);
            const int64_t blk = x >> 8, sb = sbb + (blk >> 8);
            const float oblk = la.blkmax[bb + blk];
            if (rm > oblk) {
                atomicMax(reinterpret_cast<unsigned int*>(la.blkmax) + bb + blk, __float_as_uint(rm));
                atomicMax(reinterpret_cast<unsigned int*>(la.sblkmax) + sb, __float_as_uint(rm));
                atomicMax(reinterpret_cast<unsigned int*>(la.tmax) + t, __float_as_uint(rm));
            }
            if (old_rm == oblk && rm < old_rm) {  // held its block's max: the finalize re-reduces it
                flag_set(la.bdirty, bb + blk);
                flag_set(la.sdirty, sb);
            }
        }
    };
    for (uint32_t m = stall_mask; m; m &= m - 1) {  // uniform
        const int gi = __ffs((int)m) - 1, sg = gi % SPLIT, jg = gi / SPLIT;
        if (dsplit) {  // the row-range slots this workgroup would have updated
            for (int sl = sg; sl < SPLIT; sl += NA) {
                int c = (int)ld_wt(reinterpret_cast<const uint32_t*>(a.ws_ucount + t * SPLIT + sl));
                const int64_t cap = s_cb[sl + 1] - s_cb[sl];
                c = c < 0 ? 0 : (c > cap ? (int)cap : c);
                apply_range(s_cb[sl], s_cb[sl] + c);
            }
        } else {
            int c = s_cnt_g[gi];
            const int64_t cap = s_cb[sg + 1] - s_cb[sg];
            c = c < cap ? c : (int)cap;
            if (K == 1 || jg == 0) apply_range(s_cb[sg], s_cb[sg] + c);
            else apply_range(s_cb[sg + 1] - c, s_cb[sg + 1]);
        }
    }
}

// APPLY (dqrm_emb_bwd_apply_local, world size 1): after the coalesce, the table's workgroups
// meet once (each publishes its max|grad|, then waits for the table's others: all of them are
// resident, one per CU), and each updates the rows of its row-range slot exactly as
// k_apply_local does -- quantize with the table scale, SGD, rowmax, block maxima it owns
// re-reduced here, superblock / table growth by atomicMax, shrunk superblocks flagged for the
// table's last workgroup. The W rows are loaded before the segment phase, so the update's
// random-row latency hides behind the coalesce.
// FWD (APPLY only; dqrm_emb_bwd_apply_fwd_local): the next batch's forward behind the update,
// its own instantiation so the update-only kernel keeps its registers.
template <bool APPLY, bool RM, bool FWD>
__global__ void __launch_bounds__(TPB) k_coalesce_p1(dqrm_internal::CoalesceArgs a, dqrm_internal::LocalApplyArgs la) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int s_cnt[MAXI * NW];
    __shared__ int s_cnt2[MAXI * NW];
    __shared__ int s_w[NW + 1];
    __shared__ int s_w2[NW + 1];
    __shared__ int s_crowd;
    __shared__ int64_t s_cb[SPLIT + 1];
    __shared__ int s_uf[SPLIT + 1];
    __shared__ int s_ucnt[SPLIT];
    __shared__ float s_red[NW];
    __shared__ float s_am;
    __shared__ int s_stall;
    __shared__ int s_upart;
    __shared__ uint32_t s_epoch;
    __shared__ float s_sbm[SBC];            // fused update: sblkmax of the slot's superblocks
    __shared__ int s_cand_blk[CAND_SLOTS];  // fused update: block cached by wave w's row-max slot (-1: none)
    __shared__ int s_oq_n;
    __shared__ int s_dirty;
    __shared__ int s_fin;
    __shared__ int s_stallmask;
    __shared__ int s_lastarr;
    __shared__ float s_ftm;
    __shared__ int s_fok;
    __shared__ int s_pub;
    __shared__ uint32_t s_oq_blk[OWN_Q];
    __shared__ float s_oq_old[OWN_Q];
    __shared__ float s_oq_sold[OWN_Q];
    uint64_t* keys = reinterpret_cast<uint64_t*>(lds);
    uint16_t* pos = reinterpret_cast<uint16_t*>(lds + OFF_POS);
    uint16_t* hpos = reinterpret_cast<uint16_t*>(lds + OFF_HPOS);
    uint16_t* mlist = reinterpret_cast<uint16_t*>(lds + OFF_MLIST);
    int* sdest = reinterpret_cast<int*>(lds + OFF_SDEST);
    float* stage = reinterpret_cast<float*>(lds + OFF_STAGE);

    // XCD-aware placement: blocks b and b + 8 share an XCD (and its L2), so table t's 8 slots
    // are blocks (t/8)*64 + s*8 + t%8. A dimension-split table's slots read 32-B slices of
    // the same dy lines; on one XCD a line is fetched from HBM once, not once per slot.
    const int grp = (int)(blockIdx.x >> 6) * 8 + (int)(blockIdx.x & 7), s = (int)(blockIdx.x >> 3) & 7;
    int t = (APPLY && la.group_perm && grp < a.T) ? (int)la.table_of_group[grp] : grp, j = 0;
    if (grp >= a.T) {  // a spare group: sub-slot 1 of a big table's slots, or idle
        const int e = grp - a.T;
        if (!APPLY || e >= dqrm_internal::kSubTables || la.sub_table[e] < 0) return;
        t = la.sub_table[e];
        j = 1;
    }
    const int k = t * SPLIT + s;
    const int kd = k + j * a.T * SPLIT;  // diagnostic stamp row (sub-slot 1 after all of sub-slot 0)
    (void)kd;
    const int tid = threadIdx.x, w = tid / WAVE;
    // dy float4 prefetched per thread: 4 in the fused kernel (its update needs the registers;
    // a Criteo slot of <= 256 lookups x 16 float4 still lands in one round)
    constexpr int PF = APPLY ? (PFR < 4 ? PFR : 4) : PFR;
    const int B = (int)a.B;
    CDIAG(0);
    // 1. the table's uniform values (scalar loads), then this thread's lookups
    //    b = tid + TPB*i, all in flight. Every global load below is unconditional (indices
    //    clamped), so the compiler can count them and wait for exactly the one it needs.
    const int64_t nrows = a.meta[a.T + t];
    const float sc = a.scale[t];
    // this slot's workspace region (scalar), and the table's slot bases (lane q < 9) for LDS
    const int64_t cb_s = a.ws_cap_base[k], cb_e = a.ws_cap_base[k + 1];
    const int64_t cbl = a.ws_cap_base[t * SPLIT + (tid <= SPLIT ? tid : SPLIT)];
    const int ni = (B + TPB - 1) / TPB;
    int64_t r[MAXI];
    const int64_t* ti = a.idx + (int64_t)t * a.B;
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
        const int b = tid + TPB * i;
        r[i] = -1;
        if (i < ni) r[i] = ti[b < B ? b : B - 1];
    }
    const int64_t nblk = (nrows + BLK - 1) / BLK;
    const bool dsplit = nblk < SPLIT;
    const int LPR = a.D / 4;
    const int DS = LPR < SPLIT ? LPR : SPLIT;
    const int LG = dsplit ? LPR / DS : LPR;  // float4 of a row this workgroup owns
    const int lg_sh = __ffs(LG) - 1;
    const int SW = LG * 4;                   // dimensions this workgroup owns
    const int sw_sh = lg_sh + 2;
    const int q0 = dsplit ? s * LG : 0;
    // sub-slots of this table's slots: 2 if a spare group serves it
    const int K = (j == 1 || (APPLY && !dsplit && ((la.sub_mask >> t) & 1u))) ? 2 : 1;
    int64_t r0 = 0, r1 = nrows;
    if (!dsplit) {
        int64_t b0 = nblk * s / SPLIT, b1 = nblk * (s + 1) / SPLIT;
        if (K == 2) {  // halves of the slot's blocks: sub-slot 0 the lower, 1 the upper
            const int64_t bm = (b0 + b1) / 2;
            if (j == 0) b1 = bm; else b0 = bm;
        }
        r0 = b0 * BLK;
        r1 = b1 * BLK;
        r1 = r1 < nrows ? r1 : nrows;
    }
    const bool active = dsplit ? s < DS : r0 < r1;
    const int SP = (STAGE_FLOATS / SW) & ~3;  // stage entries (dimension-major: the column pitch, 16-B columns)
    const int CE = SP - 4;                    // stage entries per chunk
    const bool rmaj = RM && !(DQRM_COAL_DSDM && !APPLY && dsplit);
    // stage index of (entry p, dimension d)
    auto sx = [&](int p, int d) -> int { return rmaj ? p * SW + d : d * SP + p; };
    const float* dyt = a.dy + (int64_t)t * a.dst_t;
    // fused update: this launch's epoch = this slot's previous granule epoch + 1 (every slot
    // of a table publishes once per launch, so the table's granules always agree)
    uint64_t* gran = reinterpret_cast<uint64_t*>(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + GRAN_WORD);
    uint32_t epoch = 0;
    if (APPLY && tid < WAVE)
        epoch = (gr_epoch(__hip_atomic_load(gran + s + SPLIT * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u) &
                GR_EPOCH_MASK;
    if (DQRM_COAL_CAND == 2 && APPLY && tid == 0) s_epoch = epoch;  // (read after the barriers below)
    auto fetch = [&](int b, int sub) -> float4 {
        return reinterpret_cast<const float4*>(dyt + (int64_t)b * a.dst_b)[q0 + sub];
    };
    auto finish = [&](float4 g) -> float4 {  // g' = (g * s) / s
        if (a.ste) {
            g.x = (g.x * sc) / sc; g.y = (g.y * sc) / sc; g.z = (g.z * sc) / sc; g.w = (g.w * sc) / sc;
        }
        return g;
    };
    CDIAG(1);
    if (!active) {  // a dimension slice beyond D (D < 32): no work; the counts come from slot 0
        if (tid == 0) a.ws_absmax[k] = 0.0f;
        return;
    }
    // A dimension-split table combines its slice of EVERY lookup: those dy loads depend on
    // nothing and go out now, in flight with the index loads and across the compaction and
    // sort. A row-split slot issues the same number of placeholder loads (one hot 16-B line,
    // overwritten after the compaction), so on both paths the compiler waits for the index
    // loads alone.
    float4 pf[PF];
    {
        const int lim = B > 0 ? (B << lg_sh) - 1 : 0;
#pragma unroll
        for (int f = 0; f < PF; ++f) {
            const int q = min(tid + TPB * f, lim);
            const float4* src = dsplit && B > 0
                                    ? reinterpret_cast<const float4*>(dyt + (int64_t)(q >> lg_sh) * a.dst_b) + q0 + (q & (LG - 1))
                                    : reinterpret_cast<const float4*>(a.ws_cap_base);
            pf[f] = *src;
        }
    }
    if (tid <= SPLIT) s_cb[tid] = cbl;
    if (tid < SPLIT) s_ucnt[tid] = 0;
#pragma unroll
    for (int i = 0; i < MAXI; ++i)
        if (tid + TPB * i >= B) r[i] = -1;
    CDIAG(8);
    // Row spans of at most CSPAN rows are sorted by counting rows: the per-row counts give
    // every segment's start, number and kind directly (no comparison sort, no head pass).
    // A lookup's place among its row's lookups (lookup order) comes from
    //   ranked (span <= 256): per-wave row counters + same-row lanes by ballots, as one
    //     stable radix pass does;
    //   atomic (256 < span <= CSPAN): the row counter's arrival rank, then re-ranked inside
    //     its bucket by lookup order (a bucket above FIX_MAX -> the comparison sort)
    const uint32_t span = (uint32_t)(r1 - r0);
    const int nbits = span <= 1 ? 0 : 32 - __clz(span - 1);
    const bool ranked = CSPAN > 0 && nbits <= 8;
    const bool atomic_mode = nbits > 8 && span <= (uint32_t)CSPAN;
    int* info = reinterpret_cast<int*>(lds + OFF_INFO);
    int* minfo = reinterpret_cast<int*>(lds + OFF_MINFO);
    int* whist = reinterpret_cast<int*>(lds + OFF_SCR);  // ranked: [NW][span] row counters
    if (atomic_mode) {
        for (int q = tid; q < (int)span; q += TPB) info[q] = 0;
        if (tid == 0) s_crowd = 0;
    }
    if (ranked)
        for (int q = tid; q < NW * (int)span; q += TPB) whist[q] = 0;
    // 2. the slot's lookups, compacted in lookup order (counting path: each one's arrival
    //    rank in its row's counter, in any order)
    auto none = [](int, int, bool) {};
    uint64_t kx[MAXI];
    int krk[MAXI];
    const int n = ordered_compact(
        ni, s_cnt, [&](int i) { return r[i] >= r0 && r[i] < r1; },
        [&](int i, int p) {
            const uint32_t b = tid + TPB * i;
            const uint32_t g = dsplit ? b : (uint32_t)p;
            kx[i] = ((uint64_t)(r[i] - r0) << 32) | (g << LK_BITS) | b;
            keys[p] = kx[i];
            if (atomic_mode) krk[i] = atomicAdd(&info[r[i] - r0], 1);
        },
        none);
    CDIAG(9);
    if (j == 0 && (dsplit ? s == 0 : s == SPLIT - 1)) {  // out-of-range indices: flagged once per table
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MAXI; ++i)
            if (tid + TPB * i < B && (r[i] < 0 || r[i] >= nrows)) bad = true;
        if (bad) atomicOr(a.err, DQRM_ERRF_INDEX);
    }
    __syncthreads();
    CDIAG(10);
    // the dy values this workgroup will combine, in flight across the sort (a dimension-
    // split table: its slice of every lookup; a row split: its lookups' rows). Nothing
    // between here and their use waits for global memory.
    if (!dsplit) {
#pragma unroll
        for (int f = 0; f < PF; ++f) {
            const int q = tid + TPB * f;
            if (q < (n << lg_sh)) pf[f] = fetch((int)kbag(keys[q >> lg_sh]), q & (LG - 1));
        }
    }
    CDIAG(2);
    uint64_t* tmp = reinterpret_cast<uint64_t*>(lds + OFF_SCR);
    int U, NS, M;
    bool counted = false;
    int ta = 0, tm = 0;
    // 3u. one-launch step: a wide row-split slot whose rows are all distinct (a big table's
    //     slot, nearly always) needs no sort -- every lookup is its own segment, in compaction
    //     (= lookup) order, and the update keeps no order. Distinctness from one LDS hash insert
    //     per lookup. (The N > 1 coalesce keeps the sort: its payload rows must be ascending.)
    bool uniq = false;
    if (APPLY && DQRM_COAL_UNIQ && !dsplit && !ranked && !atomic_mode && n <= UNIQ_MAXN) {
        uint32_t* hk = reinterpret_cast<uint32_t*>(stage);  // the stage is not used before the land phase
        for (int q = tid; q < UNIQ_HASH; q += TPB) hk[q] = 0u;
        if (tid == 0) s_crowd = 0;
        __syncthreads();
        if (tid < n) {
            const uint32_t key = krow(keys[tid]) + 1u;
            uint32_t h = (key * 2654435761u) >> (32 - UNIQ_HLOG);
            for (;;) {  // linear probing, load <= 1/4
                const uint32_t old = atomicCAS(&hk[h], 0u, key);
                if (old == 0u) break;
                if (old == key) {
                    s_crowd = 1;  // a repeated row: the sorting path
                    break;
                }
                h = (h + 1u) & (UNIQ_HASH - 1);
            }
        }
        __syncthreads();
        uniq = s_crowd == 0;
        if (uniq) {
            for (int p = tid; p < n; p += TPB) {
                pos[kgat(keys[p])] = (uint16_t)p;
                hpos[p] = (uint16_t)p;
                sdest[p] = (int)((j ? cb_e - n : cb_s) + p);
            }
            if (tid == 0) hpos[n] = (uint16_t)n;
            U = n;
            M = 0;
            NS = n;
        }
    }
    if (ranked) {
        // 3a'. wave w ranks keys [w*64*kpl, (w+1)*64*kpl) in order: same-row lanes by
        //      bit-slice ballots, earlier keys of the wave by its row counters
        const int lane = tid % WAVE, wu = wave_id();
        const int kpl = (n + TPB - 1) / TPB;
        const int i0 = wu * WAVE * kpl + lane;
        const uint64_t lt = lanemask_lt();
        uint64_t xr[MAXI];
        int wr[MAXI];
#pragma unroll
        for (int kk = 0; kk < MAXI; ++kk) {
            if (kk >= kpl) break;
            const int i = i0 + kk * WAVE;
            const bool v = i < n;
            xr[kk] = v ? keys[i] : 0ull;
            const uint32_t d = krow(xr[kk]);
            uint64_t pm = __ballot(v);
            for (int q = 0; q < nbits; ++q) {
                const uint64_t bq = __ballot((d >> q) & 1u);
                pm &= ((d >> q) & 1u) ? bq : ~bq;
            }
            int* hc = whist + wu * (int)span + d;
            wr[kk] = v ? *hc + (int)__popcll(pm & lt) : 0;
            if (v && (pm & lt) == 0) *hc += (int)__popcll(pm);
        }
        __syncthreads();
        // 3b'. per row (thread = row): its count over the waves, the row prefixes, and each
        //      wave's first place in the row's bucket
        int cw[NW];
        int c = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            cw[q] = tid < (int)span ? whist[q * (int)span + tid] : 0;
            c += cw[q];
        }
        int ea, em;
        block_excl_scan2(c | (c > 0 ? 1 << 16 : 0), c > 1 ? 1 : 0, s_w, s_w2, ea, em, ta, tm);
        if (tid < (int)span) {
            info[tid] = ea;
            minfo[tid] = em;
            int o = ea & 0xFFFF;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                whist[q * (int)span + tid] = o;
                o += cw[q];
            }
        }
        if (tid == 0) {
            info[span] = ta;
            minfo[span] = tm;
        }
        __syncthreads();
        // 3c'. every key to its place (each place written once; all keys are in registers)
#pragma unroll
        for (int kk = 0; kk < MAXI; ++kk) {
            if (kk >= kpl) break;
            if (i0 + kk * WAVE < n) keys[whist[wu * (int)span + krow(xr[kk])] + wr[kk]] = xr[kk];
        }
        __syncthreads();
        counted = true;
    } else if (atomic_mode) {
        // 3a. row scan: per row, the lookups and distinct rows before it (packed) and the
        //     multi-lookup rows before it; thread tid owns rows [tid*RPT, tid*RPT + RPT)
        int c[RPT];
        int va = 0, vm = 0;
        bool crowd = false;
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
            const int q = tid * RPT + j;
            c[j] = q < (int)span ? info[q] : 0;
            va += c[j] | (c[j] > 0 ? 1 << 16 : 0);
            vm += c[j] > 1 ? 1 : 0;
            crowd |= c[j] > FIX_MAX;
        }
        if (crowd) s_crowd = 1;
        int ea, em;
        block_excl_scan2(va, vm, s_w, s_w2, ea, em, ta, tm);
        if (s_crowd == 0) {
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const int q = tid * RPT + j;
                if (q < (int)span) {
                    info[q] = ea;
                    minfo[q] = em;
                }
                ea += c[j] | (c[j] > 0 ? 1 << 16 : 0);
                em += c[j] > 1 ? 1 : 0;
            }
            if (tid == 0) {
                info[span] = ta;
                minfo[span] = tm;
            }
            __syncthreads();
            // 3b. every lookup to its row's bucket (arrival order), 3c. then to its place in
            //     the bucket = the number of the bucket's keys before it in lookup order
#pragma unroll
            for (int i = 0; i < MAXI; ++i)
                if (i < ni && r[i] >= r0 && r[i] < r1) tmp[(info[r[i] - r0] & 0xFFFF) + krk[i]] = kx[i];
            __syncthreads();
#pragma unroll
            for (int i = 0; i < MAXI; ++i)
                if (i < ni && r[i] >= r0 && r[i] < r1) {
                    const int q = (int)(r[i] - r0);
                    const int st = info[q] & 0xFFFF, len = (info[q + 1] & 0xFFFF) - st;
                    int below = 0;
                    for (int j = st; j < st + len && len > 1; ++j) below += tmp[j] < kx[i] ? 1 : 0;
                    keys[st + below] = kx[i];
                }
            __syncthreads();
            counted = true;
        }
    }
    if (counted) {
            CDIAG(3);
            // 3d. per sorted position: gather -> position map, segment heads, multi-lookup
            //     segment list and output entries, all from the row prefixes
            for (int p = tid; p < n; p += TPB) {
                const uint64_t x = keys[p];
                const int q = (int)krow(x);
                const int inf = info[q], st = inf & 0xFFFF, u = inf >> 16;
                const int len = (info[q + 1] & 0xFFFF) - st, mp = minfo[q];
                pos[kgat(x)] = (uint16_t)p;
                if (p == st) {
                    hpos[u] = (uint16_t)p;
                    if (len > 1) mlist[mp] = (uint16_t)u;
                }
                int e = -(p - (u - mp)) - 1;
                if (len == 1) {
                    if (dsplit) {
                        const int sl = slot_of_row(q, nblk);
                        const int rs = (int)(nblk * sl / SPLIT * BLK);
                        e = (int)(s_cb[sl] + (u - (info[rs] >> 16)));
                    } else {
                        e = (int)((j ? cb_e - (ta >> 16) : cb_s) + u);
                    }
                }
                sdest[p] = e;
            }
            U = ta >> 16;
            M = tm;
            NS = U - M;
            if (tid == 0) hpos[U] = (uint16_t)n;
            if (dsplit && tid <= SPLIT) {  // first segment of every row-range slot, and counts
                auto uf = [&](int sl) {
                    const int64_t rs = nblk * sl / SPLIT * BLK;
                    return rs < (int64_t)span ? info[rs] >> 16 : U;
                };
                s_uf[tid] = uf(tid);
                if (tid < SPLIT) s_ucnt[tid] = uf(tid + 1) - uf(tid);
            }
    }
    if (dsplit) {  // invalid lookups have no key: their prefetched slices are dropped
#pragma unroll
        for (int i = 0; i < MAXI; ++i)
            if (tid + TPB * i < B && !(r[i] >= 0 && r[i] < nrows)) pos[tid + TPB * i] = 0xFFFF;
    }
    if (counted || uniq) __syncthreads();
    else {
    // 3. sort by row
    {
        int* hist = reinterpret_cast<int*>(lds + OFF_SCR + MAXB * 8);
        if (nbits > 8)
            msd_sort(keys, tmp, hist, s_w, n, nbits);
        else
            radix_sort(keys, tmp, hist, s_w, n, nbits);
    }
    CDIAG(3);
    for (int p = tid; p < n; p += TPB) pos[kgat(keys[p])] = (uint16_t)p;
    if (dsplit) {  // invalid lookups have no key: their prefetched slices are dropped
#pragma unroll
        for (int i = 0; i < MAXI; ++i)
            if (tid + TPB * i < B && !(r[i] >= 0 && r[i] < nrows)) pos[tid + TPB * i] = 0xFFFF;
    }
    // segment heads (first sorted position of every distinct row) and single-lookup
    // segments, both prefix-counted in one pass. sdest[p]: a single-lookup segment's output
    // entry (dimension-split: its segment number, fixed up below), else -(stage index) - 1,
    // the stage holding only the lookups of multi-lookup segments, in sorted order
    {
        const int lane = tid % WAVE;
        const int np = (n + TPB - 1) / TPB;
        uint64_t mh[MAXI], ms[MAXI];
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int p = tid + TPB * i;
            bool h = false, sg = false;
            if (i < np && p < n) {
                const uint32_t rw = krow(keys[p]);
                h = p == 0 || krow(keys[p - 1]) != rw;
                sg = h && (p + 1 == n || krow(keys[p + 1]) != rw);
            }
            mh[i] = __ballot(h);
            ms[i] = __ballot(sg);
        }
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < MAXI; ++i)
                if (i < np) {
                    s_cnt[i * NW + w] = (int)__popcll(mh[i]);
                    s_cnt2[i * NW + w] = (int)__popcll(ms[i]);
                }
        __syncthreads();
        const int vh = lane < np * NW ? s_cnt[lane] : 0, vs = lane < np * NW ? s_cnt2[lane] : 0;
        const int ih = wave_incl_scan(vh), is = wave_incl_scan(vs);
        U = lane_of(ih, WAVE - 1);
        NS = lane_of(is, WAVE - 1);
        const int eh = ih - vh, es = is - vs;
        const uint64_t lt = lanemask_lt();
        const int wu = wave_id();
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int p = tid + TPB * i;
            const int rh = lane_of(eh, (i * NW + wu) & (WAVE - 1)) + (int)__popcll(mh[i] & lt);
            const int rs = lane_of(es, (i * NW + wu) & (WAVE - 1)) + (int)__popcll(ms[i] & lt);
            if (i < np && p < n) {
                const bool h = (mh[i] >> lane) & 1ull, sg = (ms[i] >> lane) & 1ull;
                if (h) {
                    hpos[rh] = (uint16_t)p;
                    if (dsplit) atomicAdd(&s_ucnt[slot_of_row(krow(keys[p]), nblk)], 1);
                }
                const int u = h ? rh : rh - 1;
                sdest[p] = sg ? (dsplit ? u : (int)((j ? cb_e - U : cb_s) + u)) : -(p - rs) - 1;
            }
        }
    }
    if (tid == 0) hpos[U] = (uint16_t)n;
    __syncthreads();
    if (dsplit && tid <= SPLIT) {  // first segment of every row-range slot
        int c = 0;
        for (int q = 0; q < tid; ++q) c += s_ucnt[q];
        s_uf[tid] = c;
    }
    // segments of more than one lookup (the rest are copied straight from registers)
    M = ordered_compact(
        (U + TPB - 1) / TPB, s_cnt,
        [&](int i) {
            const int u = tid + TPB * i;
            return u < U && hpos[u + 1] - hpos[u] > 1;
        },
        [&](int i, int m) { mlist[m] = (uint16_t)(tid + TPB * i); }, none);
    if (dsplit) {  // single-lookup segment -> its row-range slot's entry
        for (int p = tid; p < n; p += TPB) {
            const int u = sdest[p];
            if (u >= 0) {
                const int sl = slot_of_row(krow(keys[p]), nblk);
                sdest[p] = (int)(s_cb[sl] + (u - s_uf[sl]));
            }
        }
        __syncthreads();
    }
    }  // comparison sort
    CDIAG(4);
    // fused update: the entries of row-range slot sl are segments [ua, ua + nu) (a dimension-
    // split table: its rows in that range; a row split: all of the slot's), entry s_cb[sl] +
    // (u - ua). Workgroup s updates slots s, s + NA, ... (NA = the table's active workgroups).
    const int NA = dsplit ? DS : SPLIT;
    const int NG = NA * K;  // the table's workgroups (granules)
    const int lpr_sh = __ffs(LPR) - 1;
    // this workgroup's entries in its slot's workspace region: sub-slot 0 (or a whole slot) from
    // its start, sub-slot 1 packed at its end (its values are scratch; its rows are written at
    // their final place, after sub-slot 0's, once the rendezvous has told it sub-slot 0's count)
    auto ebase = [&]() -> int64_t { return j ? s_cb[s + 1] - U : s_cb[s]; };  // (LDS reads, not a live register)
    auto slot_entries = [&](int sl, int& ua, int& nu) {
        ua = dsplit ? s_uf[sl] : 0;
        nu = dsplit ? s_uf[sl + 1] - ua : U;
        const int cap = (int)(s_cb[sl + 1] - s_cb[sl]);
        nu = nu < cap ? nu : cap;
    };
    // a row-split slot whose entries fit beside the stage's multi-lookup values keeps its
    // coalesced values in the stage (entry u, dimension d at column d, index vb0 + u) instead
    // of the workspace: no HBM round trip for them (the workspace values are then not written)
    const int vb0 = n - NS;
    const bool lds_vals = APPLY && !dsplit && vb0 + U <= CE && U <= (int)(s_cb[s + 1] - s_cb[s]);
    int64_t rb = 0, bb = 0, sbb = 0;
    int ua0 = 0, nu0 = 0;
    float4 wpf[WPFA];
    float bpf[WPFA];
    float otm = 0.0f;
    if constexpr (APPLY) {
        rb = a.meta[t];
        bb = a.meta[2 * a.T + t];
        sbb = a.meta[3 * a.T + t];
        slot_entries(s, ua0, nu0);
        if (tid == 0) {
            s_oq_n = 0;
            s_dirty = 0;
        }
        otm = la.tmax[t];
    }
    // the W rows and block maxima of the entries this workgroup will update, in flight across
    // the land and segment phases and the wait for the table's other workgroups: issued before
    // the land phase (the default; at WPF = 4 both register sets fit the 128-VGPR budget), or
    // once the dy prefetch registers are free (DQRM_COAL_WLATE=1, an A/B build)
    auto issue_w = [&]() {
        if constexpr (APPLY) {
#pragma unroll
            for (int jj = 0; jj < WPF; ++jj) {
                const int q = tid + TPB * jj;
                wpf[jj] = make_float4(0.f, 0.f, 0.f, 0.f);
                bpf[jj] = 0.0f;
                if (q < (nu0 << lpr_sh)) {
                    const int64_t x = r0 + krow(keys[hpos[ua0 + (q >> lpr_sh)]]);
                    wpf[jj] = reinterpret_cast<const float4*>(la.W + (rb + x) * a.D)[q & (LPR - 1)];
                    bpf[jj] = la.blkmax[bb + (x >> 8)];
                }
            }
        }
    };
    // the superblock maxima of the slot's rows (a row-split slot spans a few hundred at most),
    // read by the update's growth / holder checks from LDS instead of a dependent HBM load each.
    // Read before the update: a stale-low value (another slot's growth) only costs a redundant
    // atomicMax or superblock re-reduction, never a wrong maximum.
    const int64_t sb0 = r0 >> 16;
    const int nsbc = APPLY && !dsplit && r1 > r0 && ((r1 - 1) >> 16) - sb0 < SBC ? (int)(((r1 - 1) >> 16) - sb0 + 1) : 0;
    float sbv = 0.0f;
    if (APPLY && tid < nsbc) sbv = la.sblkmax[sbb + sb0 + tid];
    CDIAG_W(17);  // (diagnostic build: the dy prefetch landed -- before the W rows are issued)
    if (!DQRM_COAL_WLATE || n - NS > CE) issue_w();
    float amax = 0.0f;
    auto emit = [&](int u, int d, float acc) {  // segment u's sum in dimension q0*4 + d
        const int64_t row = r0 + krow(keys[hpos[u]]);
        int sl = s;
        int64_t e = ebase() + u;
        if (dsplit) {
            sl = slot_of_row(row, nblk);
            e = s_cb[sl] + (u - s_uf[sl]);
        }
        if (e < s_cb[sl + 1]) {
            if (lds_vals) stage[sx(vb0 + u, d)] = acc;
            else if (APPLY && dsplit) st_wt(a.ws_vals + e * a.D + q0 * 4 + d, acc);
            else a.ws_vals[e * a.D + q0 * 4 + d] = acc;
            if (j == 0 && q0 == 0 && d == 0) a.ws_rows[e] = (int32_t)row;
        }
        amax = fmaxf(amax, fabsf(acc));
    };
    auto put = [&](int p, int sub, float4 v) {  // entry p, dimensions 4*sub .. 4*sub+3
        if (rmaj) {
            *reinterpret_cast<float4*>(stage + p * SW + sub * 4) = v;
        } else {
            float* col = stage + (sub * 4) * SP + p;
            col[0] = v.x; col[SP] = v.y; col[2 * SP] = v.z; col[3 * SP] = v.w;
        }
    };
    // strictly ordered sum of dimension d over entries [p, pe), starting from acc
    auto chain = [&](int d, int p, int pe, float acc) -> float {
        return rmaj ? chain_sum_rm(stage + d, p, pe, SW, acc) : chain_sum(stage + d * SP, p, pe, acc);
    };
    if (n - NS <= CE) {
        // 4. one chunk. Every value first goes where it belongs -- a single-lookup segment's
        //    value IS its output row (kept in registers), the others land in the stage at
        //    their sorted positions -- and only then are the output rows stored, so no wait
        //    for a load ever waits for a store as well
        const int nitems = (dsplit ? B : n) << lg_sh;
        auto land = [&](int q, float4 v) -> int {  // v finished; returns the output entry or -1
            const int p = pos[q >> lg_sh];
            if (p == 0xFFFF) return -1;
            const int e = sdest[p];
            if (e < 0) put(-e - 1, q & (LG - 1), v);
            return e;
        };
        auto store = [&](int q, int e, float4 v) {  // a single-lookup segment's output row
            if (e < 0 || e >= s_cb[SPLIT]) return;
            if (lds_vals) {
                put(vb0 + (int)(e - ebase()), q & (LG - 1), v);
            } else {
                float4* dst = reinterpret_cast<float4*>(a.ws_vals + (int64_t)e * a.D) + q0 + (q & (LG - 1));
                if (APPLY && dsplit) st4_wt(dst, v);
                else *dst = v;
            }
            if (j == 0 && q0 == 0 && (q & (LG - 1)) == 0) a.ws_rows[e] = (int32_t)(r0 + krow(keys[pos[q >> lg_sh]]));
            amax = fmaxf(amax, abs_max4(v));
        };
        int q = tid;
        {
            int de[PF];
#pragma unroll
            for (int f = 0; f < PF; ++f) {
                de[f] = -1;
                if (q + TPB * f < nitems) {  // the STE division only where a value exists
                    pf[f] = finish(pf[f]);
                    de[f] = land(q + TPB * f, pf[f]);
                }
            }
#pragma unroll
            for (int f = 0; f < PF; ++f) store(q + TPB * f, de[f], pf[f]);
            q += TPB * PF;
        }
        if (DQRM_COAL_WLATE) issue_w();
        for (; q < nitems; q += TPB) {  // beyond the register budget (or no prefetch)
            const int p = pos[q >> lg_sh];
            if (p == 0xFFFF) continue;
            const float4 v = finish(fetch(kbag(keys[p]), q & (LG - 1)));
            store(q, land(q, v), v);
        }
        __syncthreads();
        CDIAG(5);
        for (int i = tid; i < (M << sw_sh); i += TPB) {
            const int u = mlist[i >> sw_sh], d = i & (SW - 1);
            const int h = hpos[u], len = hpos[u + 1] - h;
            const int st = -sdest[h] - 1;  // the segment's first stage entry
            emit(u, d, chain(d, st, st + len, -0.0f));  // -0 + x == x for every x: the first value exactly
        }
    } else {
        // a slot larger than the stage: chunks of CE sorted lookups, loaded after the sort;
        // item (u, d) belongs to thread (u*SW + d) % TPB in every chunk, so the segment that
        // crosses a chunk boundary continues in the same lane (carry)
        float carry = 0.0f;
        for (int c0 = 0; c0 < n; c0 += CE) {
            const int ce = n - c0 < CE ? n - c0 : CE;
            for (int q = tid; q < (ce << lg_sh); q += TPB) {
                const int p = c0 + (q >> lg_sh), sub = q & (LG - 1);
                put(p - c0, sub, finish(fetch(kbag(keys[p]), sub)));
            }
            __syncthreads();
            auto seg_of = [&](int p) {  // segment holding sorted position p
                int lo = 0, hi = U - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((int)hpos[mid] <= p) lo = mid; else hi = mid - 1;
                }
                return lo;
            };
            const int ua = seg_of(c0), ub = seg_of(c0 + ce - 1);
            const int first = ua << sw_sh;
            for (int i = first + ((tid - first) % TPB + TPB) % TPB; i < ((ub + 1) << sw_sh); i += TPB) {
                const int u = i >> sw_sh, d = i & (SW - 1);
                const int h = hpos[u], e1 = hpos[u + 1];
                const int pe = e1 < c0 + ce ? e1 : c0 + ce;
                const float acc = h >= c0 ? chain(d, h - c0, pe - c0, -0.0f) : chain(d, 0, pe - c0, carry);
                if (e1 > c0 + ce) {
                    carry = acc;
                    continue;
                }
                emit(u, d, acc);
            }
            __syncthreads();
        }
    }
    CDIAG_W(6);
    // the workgroup's max|grad| (dimension-split: its slice's) and the slot counts
    for (int o = WAVE / 2; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, WAVE));
    if (tid % WAVE == 0) s_red[w] = amax;
    // a dimension-split table's values are read by its other workgroups: every wave's value
    // stores land before the granule below signals them (hand-off row 1, sc1 stores)
    if (APPLY && dsplit) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        float m = 0.0f;
        for (int q = 0; q < NW; ++q) m = fmaxf(m, s_red[q]);
        if (K == 1) a.ws_absmax[k] = m;  // sub-slots: sub-slot 0 writes the slot's, after the rendezvous
        // publish this slot's max|grad| (and distinct rows) as ONE 8-B sc1 store (a data-tagged
        // granule: no counter, no ordering needed for the value itself)
        if constexpr (APPLY) {
            __hip_atomic_store(gran + s + SPLIT * j, gr_make(m, dsplit ? 0 : U, epoch), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            // a slot served alone this launch also advances its sub-slot-1 granule, so both
            // sub-slots derive the same epoch in a later launch that splits the slot (a parent
            // set and a one-table view of it plan sub-slots differently; nobody polls it now)
            if (K == 1 && !dsplit)
                __hip_atomic_store(gran + s + SPLIT, gr_make(0.0f, 0, epoch), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if constexpr (APPLY) {
        if (tid < nsbc) s_sbm[tid] = sbv;
        // While wave 0 waits for the table's other workgroups, every other wave looks for a block
        // whose row-max holder is one of its (prefetched) rows -- the blocks the update may have
        // to re-reduce -- and copies the first such block's 256 stored row maxima into its LDS
        // cache (the pos / mlist regions, dead by now). Rows of a block are updated only by this
        // workgroup, so the copy stays exact for the untouched rows.
        if (DQRM_COAL_CAND && !dsplit && w > 0) {
            int cb = -1;
            bool met = false;
            if (DQRM_COAL_CAND == 2) {  // the table already met (this workgroup came last): nothing to hide behind
                const int l = tid % WAVE;
                const bool ok = l >= NG || gr_epoch(__hip_atomic_load(gran + l, __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT)) == s_epoch;
                met = __all(ok);
            }
#pragma unroll
            for (int jj = 0; jj < WPF && !met; ++jj) {
                const int q = tid + TPB * jj;
                const bool in = q < (nu0 << lpr_sh);
                float orm = in ? abs_max4(wpf[jj]) : -1.0f;
                for (int o = 1; o < LPR; o <<= 1) orm = fmaxf(orm, __shfl_xor(orm, o, WAVE));
                const bool cand = in && (q & (LPR - 1)) == 0 && orm == bpf[jj];
                const uint64_t cm = __ballot(cand);
                if (cb < 0 && cm) {
                    const int l = __ffsll((unsigned long long)cm) - 1;
                    const int qq = __builtin_amdgcn_readlane(q, l);
                    cb = (int)((r0 + krow(keys[hpos[ua0 + (qq >> lpr_sh)]])) >> 8);
                }
            }
            const int lane = tid % WAVE;
            if (cb >= 0) {
                float* cache = reinterpret_cast<float*>(w < 8 ? (unsigned char*)pos : (unsigned char*)mlist) + (w & 7) * BLK;
                float v[BLK / WAVE];
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) {
                    const int64_t r = (int64_t)cb * BLK + lane + i * WAVE;
                    v[i] = r < nrows ? la.rowmax[rb + r] : 0.0f;
                }
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) cache[lane + i * WAVE] = v[i];
            }
            if (lane == 0) s_cand_blk[w] = cb;
        }
        if (w == 0 && tid < CAND_SLOTS) {
            if (tid == 0 || dsplit || !DQRM_COAL_CAND) s_cand_blk[tid] = -1;
        }
    }
    if (APPLY && tid < WAVE) {  // wave 0: lane j polls slot j's granule until it shows this launch's epoch
        uint64_t g = 0;
        bool ok = tid >= NG;
        bool stalled = false;
        for (int spin = 0;; ++spin) {
            if (!ok) {
                g = __hip_atomic_load(gran + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = gr_epoch(g) == epoch;
            }
            if (__all(ok)) break;
            // the table's workgroups were not all resident (the host checks the device's CUs,
            // the occupancy and the stream's CU mask before it launches this form; another
            // stream's kernels can still hold CUs): flagged, no hang -- this workgroup does
            // not update its rows itself (the table scale would come from stale maxima); it
            // leaves them in the workspace for the table's last-arriving workgroup, which has
            // every slot's maximum by then (all-or-nothing per table)
            if (spin > (int)la.spin_limit) {
                if (tid == 0) flag_error(a.err, DQRM_ERRF_STALL);
                stalled = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const float am = wave_max(tid < NG ? __uint_as_float((uint32_t)g) : 0.0f);
        if (K == 2) {  // the partner sub-slot's count and maximum (uniform: readlane)
            const int p = j ? s : SPLIT + s;
            const int upart = __builtin_amdgcn_readlane(gr_count(g), p);
            const float mself = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g, s + SPLIT * j));
            const float mpart = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)g, p));
            if (tid == 0) {
                s_upart = upart;
                if (j == 0 && !stalled) {  // the slot's count and partial maximum, as one workgroup would write them
                    int c = U + upart;
                    const int64_t cap = s_cb[s + 1] - s_cb[s];
                    if (c > cap) {
                        atomicOr(a.err, DQRM_ERRF_OVERFLOW);
                        c = (int)cap;
                    }
                    a.ws_ucount[k] = c;
                    a.ws_absmax[k] = fmaxf(mself, mpart);
                }
            }
        }
        if (tid == 0) {
            s_am = am;
            s_stall = stalled ? 1 : 0;
        }
    }
    if (K == 1 && (!dsplit ? tid == 0 : (s == 0 && tid < SPLIT))) {
        const int sl = dsplit ? tid : s;
        int c = dsplit ? s_ucnt[sl] : U;
        const int64_t cap = s_cb[sl + 1] - s_cb[sl];
        if (c > cap) {
            atomicOr(a.err, DQRM_ERRF_OVERFLOW);
            c = (int)cap;
        }
        a.ws_ucount[t * SPLIT + sl] = c;
    }
    CDIAG_W(7);
    if constexpr (APPLY) {
        __syncthreads();
        CDIAG(11);
        // (A/B DQRM_FWD_EARLY_IDX=1: the fused forward's next-batch indices issued here, in
        // flight across the update, instead of after the arrival)
        int64_t nxe[(FWD && DQRM_FWD_EARLY_IDX) ? MAXI : 1];
        if constexpr (FWD && DQRM_FWD_EARLY_IDX) {
#pragma unroll
            for (int i = 0; i < MAXI; ++i) {
                const int b = tid + TPB * i;
                nxe[i] = b < B ? la.fwd_idx[(int64_t)t * B + b] : -1;
            }
        }
        CDIAG_W(16);  // (diagnostic build: every load of the workgroup landed, the W prefetch included)
        // the update of dqrm_apply_local: s = clamp(max|g|, 1e-8) / (2^(bits-1)-1) (* 1/N,
        // N = 1), q = clamp(round(g/s)), W += -lr * ((q * 1) * s)
        const float sv = sym_scale(s_am, la.bits) * (float)(1.0 / 1.0);
        const bool go = s_stall == 0;  // a stalled workgroup leaves its rows to the last arriver
        if (go && s == 0 && j == 0 && tid == 0) la.s_avg[t] = sv;
        const float rr = 1.0f / sv;
        const float qlo = -(float)(1 << (la.bits - 1)), qhi = (float)((1 << (la.bits - 1)) - 1);
        const ApplyUpdate upd{DQRM_UPD_DP, 1.0f, sv, sv, la.nlr};
        const float r_pack = la.repack ? 1.0f / la.pscale[t] : 0.0f;
        bool dirty = false;
        // a workgroup that updates ONE row-range slot keeps its rows' new maxima in LDS (the
        // stage, free by now): a shrunk block is then re-reduced from the other rows' stored
        // maxima (untouched this launch) and these, with no wait for its own stores
        const bool one_slot = NA == SPLIT;
        // (LDS dead by now: the gather map sdest and the multi-lookup list mlist)
        float* s_newrm = reinterpret_cast<float*>(sdest);  // [nu0]
        float* s_blkrm = stage;  // [RRW][BLK] per-wave block scratch (the update's values are dead by then)
        constexpr int RRW = 8;                             // waves re-reducing blocks at a time
        static_assert(RRW * BLK <= STAGE_FLOATS, "block scratch in the stage region");
        // item (entry u - ua, float4 sub) of slot sl: w0 = the row's old values, oblk its
        // block's max before this step (a stale-low superblock or table max only costs a
        // redundant atomicMax: within the launch they only grow)
        auto update = [&](int ua, int q, float4 w0, float oblk, float4 v) {
            const int u = ua + (q >> lpr_sh), sub = q & (LPR - 1);
            const int64_t x = r0 + krow(keys[hpos[u]]), grow = rb + x;
            float4 acc;  // + 0.0f: the payload's integer round trip turns -0 into +0
            acc.x = fake_quant(v.x, rr, qlo, qhi) + 0.0f; acc.y = fake_quant(v.y, rr, qlo, qhi) + 0.0f;
            acc.z = fake_quant(v.z, rr, qlo, qhi) + 0.0f; acc.w = fake_quant(v.w, rr, qlo, qhi) + 0.0f;
            float4 wn;
            wn.x = upd(w0.x, acc.x); wn.y = upd(w0.y, acc.y); wn.z = upd(w0.z, acc.z); wn.w = upd(w0.w, acc.w);
            reinterpret_cast<float4*>(la.W + grow * a.D)[sub] = wn;
            if (la.repack) pack4_row(wn, la.packed + grow * (a.D / 2), sub, r_pack);
            float old_rm = abs_max4(w0), rm = abs_max4(wn);
            for (int o = 1; o < LPR; o <<= 1) {
                old_rm = fmaxf(old_rm, __shfl_xor(old_rm, o, WAVE));
                rm = fmaxf(rm, __shfl_xor(rm, o, WAVE));
            }
            if (sub != 0) return;
            st_wt(la.rowmax + grow, rm);
            if (one_slot) s_newrm[u - ua] = rm;
            const int64_t blk = x >> 8, sb = sbb + (blk >> 8);
            const int64_t sbl = (blk >> 8) - sb0;  // superblock index relative to the slot's first
            const float osb = !(rm > oblk || old_rm == oblk) ? 0.0f  // the superblock's max
                              : (sbl >= 0 && sbl < nsbc) ? s_sbm[sbl] : la.sblkmax[sb];
            if (rm > oblk) {  // growth: order-free atomicMax on the non-negative float bits
                atomicMax(reinterpret_cast<unsigned int*>(la.blkmax) + bb + blk, __float_as_uint(rm));
                if (rm > osb) {
                    atomicMax(reinterpret_cast<unsigned int*>(la.sblkmax) + sb, __float_as_uint(rm));
                    if (rm > otm) atomicMax(reinterpret_cast<unsigned int*>(la.tmax) + t, __float_as_uint(rm));
                }
            }
            if (old_rm == oblk && rm < old_rm) {  // the block's max holder shrank: this slot owns the block
                const int p = atomicAdd(&s_oq_n, 1);
                if (p < OWN_Q) {
                    s_oq_blk[p] = (uint32_t)blk;
                    s_oq_old[p] = oblk;
                    s_oq_sold[p] = osb;
                } else {  // queue full: the finalize re-reduces it
                    flag_set(la.bdirty, bb + blk);
                    flag_set(la.sdirty, sb);
                    dirty = true;
                }
            }
        };
        // the values: from the LDS stage (lds_vals), else a row split reads back its own values
        // (plain loads after the workgroup barrier) and a dimension-split table's rows hold the
        // slices of all its workgroups (sc1 loads)
        auto lds_val = [&](int q) -> float4 {  // entry q >> lpr_sh, float4 q & (LPR-1)
            if (rmaj)
                return *reinterpret_cast<const float4*>(stage + (vb0 + (q >> lpr_sh)) * SW + (q & (LPR - 1)) * 4);
            const float* c = stage + (q & (LPR - 1)) * 4 * SP + vb0 + (q >> lpr_sh);
            return make_float4(c[0], c[SP], c[2 * SP], c[3 * SP]);
        };
        auto mem_val = [&](const float* vb, int q) -> float4 {
            return dsplit ? ld4_sc1(vb, (uint32_t)q * 16u) : reinterpret_cast<const float4*>(vb)[q];
        };
        auto load_val = [&](const float* vb, int q) -> float4 { return lds_vals ? lds_val(q) : mem_val(vb, q); };
        if (!go && !dsplit) {
            // a row-split slot's entries [ebase, ebase + nu0) re-stored write-through (sc1: the
            // last arriver may run on another XCD, whose L2 never saw this one's plain stores):
            // values from the LDS stage or back from this workgroup's own workspace stores, rows
            // from its keys (a dimension-split table's values are stored write-through already,
            // its workgroups' hand-off; they share one XCD with their rows' writer)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            for (int q = tid; q < (nu0 << lpr_sh); q += TPB) {
                const int u = q >> lpr_sh, sub = q & (LPR - 1);
                const int64_t e = ebase() + u;
                float4* dst = reinterpret_cast<float4*>(a.ws_vals + e * a.D) + sub;
                st4_wt(dst, lds_vals ? lds_val(q) : *dst);
                if (sub == 0)
                    __hip_atomic_store(reinterpret_cast<uint32_t*>(a.ws_rows + e),
                                       (uint32_t)(r0 + krow(keys[hpos[u]])), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!go && tid == 0)  // recorded before this workgroup's arrival (ordered by its vmcnt(0))
            atomicOr(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + STALL_WORD, 1u << (s + SPLIT * j));
        // vmcnt counts loads and stores in issue order: a load still pending when the update's
        // stores have been issued is waited for with vmcnt(0), i.e. after every one of them. So
        // the prefetched W rows and block maxima (landed during the rendezvous) are waited for
        // here, once (a real s_waitcnt vmcnt(0) the compiler's wait tracking sees; they landed
        // during the rendezvous), and values read from memory likewise before their updates.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt / lgkmcnt not waited
        for (int sl = s, j0 = 0; go && sl < SPLIT; sl += NA, j0 = 1) {  // uniform
            int ua, nu;
            slot_entries(sl, ua, nu);
            const int nit = nu << lpr_sh;
            const float* vb = a.ws_vals + (dsplit ? s_cb[sl] : ebase()) * a.D;  // the entries, D floats each
            int q = tid;
            if (j0 == 0) {  // the prefetched rows: value loads two at a time in flight, then the updates
#pragma unroll
                for (int jh = 0; jh < WPF; jh += 2) {
                    float4 v[2];
                    if (lds_vals) {
#pragma unroll
                        for (int j = jh; j < jh + 2 && j < WPF; ++j)
                            v[j - jh] = q + TPB * j < nit ? lds_val(q + TPB * j) : make_float4(0.f, 0.f, 0.f, 0.f);
                    } else {  // landed before the updates' stores (else every later use waits for them too)
#pragma unroll
                        for (int j = jh; j < jh + 2 && j < WPF; ++j)
                            v[j - jh] = q + TPB * j < nit ? mem_val(vb, q + TPB * j) : make_float4(0.f, 0.f, 0.f, 0.f);
                        __builtin_amdgcn_s_waitcnt(0x0F70);
                    }
#pragma unroll
                    for (int j = jh; j < jh + 2 && j < WPF; ++j)
                        if (q + TPB * j < nit) update(ua, q + TPB * j, wpf[j], bpf[j], v[j - jh]);
                }
                q += TPB * WPF;
                CDIAG(14);
            }
            for (; q < nit; q += TPB) {
                const int64_t x = r0 + krow(keys[hpos[ua + (q >> lpr_sh)]]);
                const float4 w0 = reinterpret_cast<const float4*>(la.W + (rb + x) * a.D)[q & (LPR - 1)];
                const float ob = la.blkmax[bb + (x >> 8)];
                update(ua, q, w0, ob, load_val(vb, q));
            }
        }
        // owned blocks whose max holder shrank: re-reduce their 256 row maxima
        __syncthreads();
        CDIAG(15);
        const int nq = s_oq_n < OWN_Q ? s_oq_n : OWN_Q;
        if (nq > 0 && !one_slot) {  // uniform: the stored maxima (write-through), once they have landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        const int lane = tid % WAVE;
        for (int qi = w; qi < nq && (w < RRW || !one_slot); qi += one_slot ? RRW : NW) {  // one wave per block
            const int64_t blk = s_oq_blk[qi];
            float mv = 0.0f;
            if (one_slot) {
                // the block's untouched rows keep their stored maxima; its touched rows (the
                // slot's entries [e0, e1), ascending rows) take their new maxima from LDS
                float* sc = s_blkrm + w * BLK;
                int ci = -1;  // a wave's cache holds this block's stored row maxima already
                for (int c = 1; c < CAND_SLOTS; ++c)
                    if (ci < 0 && s_cand_blk[c] == (int)blk) ci = c;
                if (ci >= 0) {
                    sc = reinterpret_cast<float*>(ci < 8 ? (unsigned char*)pos : (unsigned char*)mlist) + (ci & 7) * BLK;
                } else {
#pragma unroll
                    for (int i = 0; i < BLK / WAVE; ++i) {
                        const int64_t r = blk * BLK + lane + i * WAVE;
                        sc[lane + i * WAVE] = r < nrows ? la.rowmax[rb + r] : 0.0f;
                    }
                }
                if (nu0 <= 16 * WAVE) {  // every lane tests its entries (independent LDS reads, no search)
                    for (int e = lane; e < nu0; e += WAVE) {
                        const int64_t x = r0 + krow(keys[hpos[ua0 + e]]);
                        if ((x >> 8) == blk) sc[x & (BLK - 1)] = s_newrm[e];
                    }
                } else {
                    auto first_at_least = [&](int64_t row) {  // first entry with a row >= `row`
                        int lo = 0, hi = nu0;
                        while (lo < hi) {
                            const int mid = (lo + hi) >> 1;
                            if (r0 + (int64_t)krow(keys[hpos[ua0 + mid]]) < row) lo = mid + 1; else hi = mid;
                        }
                        return lo;
                    };
                    const int e0 = first_at_least(blk * BLK), e1 = first_at_least((blk + 1) * BLK);
                    for (int e = e0 + lane; e < e1; e += WAVE)
                        sc[(r0 + krow(keys[hpos[ua0 + e]])) & (BLK - 1)] = s_newrm[e];
                }
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) mv = fmaxf(mv, sc[lane + i * WAVE]);
            } else {
#pragma unroll
                for (int i = 0; i < BLK / WAVE; ++i) {
                    const int64_t r = blk * BLK + lane + i * WAVE;
                    if (r < nrows) mv = fmaxf(mv, ld_wt(la.rowmax + rb + r));
                }
            }
            mv = wave_max(mv);
            if (lane == 0) {
                st_wt(la.blkmax + bb + blk, mv);
                // it held the superblock's max before this step: the finalize re-reduces the
                // superblock (exact whatever grew meanwhile)
                if (mv < s_oq_old[qi] && s_oq_old[qi] == s_oq_sold[qi]) {
                    flag_set(la.sdirty, sbb + (blk >> 8));
                    dirty = true;
                }
            }
        }
        if (dirty) s_dirty = 1;
        if (j == 1 && go) {  // sub-slot 1's rows, at their place after sub-slot 0's entries (stalled: left for the recovery)
            const int nr = U < (int)(s_cb[s + 1] - s_cb[s]) - s_upart ? U : (int)(s_cb[s + 1] - s_cb[s]) - s_upart;
            for (int u = tid; u < nr; u += TPB) a.ws_rows[s_cb[s] + s_upart + u] = (int32_t)(r0 + krow(keys[hpos[u]]));
        }
        CDIAG(12);
        // one arrival per workgroup after all its stores landed, carrying whether it flagged
        // a superblock (hand-off row 1 of MI355X_MICROARCH.md: sc1 stores / atomics, vmcnt(0),
        // barrier, one lane's agent-scope add; the last arriver reads with sc1 loads only).
        // The last one re-reduces the flagged superblocks and the table max -- only if some
        // workgroup flagged one -- and re-arms the counter.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            uint32_t* cnt = la.sync + (int64_t)t * DQRM_SYNC_STRIDE;
            const uint32_t add = 1u + (s_dirty ? DIRTY_ONE : 0u);
            const uint32_t now = atomicAdd(cnt, add) + add;
            const bool last = (now & (DIRTY_ONE - 1u)) == (uint32_t)NG;
            uint32_t sm = 0u;
            if (last) {
                __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sm = ld_wt(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + STALL_WORD);
                if (sm) __hip_atomic_store(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + STALL_WORD, 0u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
            s_stallmask = (int)sm;
            s_lastarr = last ? 1 : 0;
            s_fin = last && ((now >> 16) != 0u || sm != 0u);
            s_pub = 0;
            if (FWD && last && !s_fin) {
                // fused forward: nothing to finalize or recover, so the table max is final now
                // (every workgroup's growth atomics landed before its arrival): published at
                // once, the table's other workgroups wait on it (step 9)
                const float tm = ld_wt(la.tmax + t);
                s_ftm = tm;
                s_fok = 1;
                s_pub = 1;
                __hip_atomic_store(reinterpret_cast<uint64_t*>(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + FWD_WORD),
                                   gr_make(tm, 0, epoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (s_stallmask) {  // uniform, rare: apply the stalled workgroups' rows (then finalize)
            recover_stalled(a, la, t, (uint32_t)s_stallmask, gran, NG, K, dsplit, NA, nblk, s_cb);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (s_fin)
            finalize_table<true>(make_meta(a.meta, a.T), t, la.W, la.rowmax, la.blkmax, la.sblkmax, la.sdirty,
                                 la.bdirty, la.tmax, a.D, true, false);
        CDIAG_W(13);
        // 9. the NEXT batch's forward (dqrm_emb_bwd_apply_fwd_local): emb_fwd_table's
        //    arithmetic for pooling 1, y[b] = fake-quant(W[row_b]) with the scale of the updated
        //    table. The table's last arriver publishes its final max (FWD_WORD granule, after
        //    the finalize); the others wait for it. Which workgroup gathers which lookup: a row
        //    split the rows of its own range -- updated by itself (or untouched) -- so its row
        //    loads go out before the wait; a dimension-split table (one XCD, no sub-slots) deals
        //    the lookups round-robin and reads after the wait, from the XCD's L2. Out-of-range
        //    rows: workgroup (0, 0) writes zeros and flags them. A stalled workgroup's share (its
        //    rows were applied by the last arriver) is the last arriver's.
        if constexpr (FWD) {
            const bool refresh = (la.fwd_flags & DQRM_FWD_REFRESH_SCALE) != 0;
            const bool fullp = (la.fwd_flags & DQRM_FWD_FULL_PRECISION) != 0;
            uint64_t* fword = reinterpret_cast<uint64_t*>(la.sync + (int64_t)t * DQRM_SYNC_STRIDE + FWD_WORD);
            if (s_lastarr && !s_pub) {  // after the recovery / finalize: the final max, then published
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    const float tm = ld_wt(la.tmax + t);
                    s_ftm = tm;
                    s_fok = 1;
                    __hip_atomic_store(fword, gr_make(tm, 0, epoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // (i) this workgroup's lookups of the next batch -- they do not depend on the table's
            //     final max -- as per-wave LDS lists {row | 0xFFFFFFFF, b} in lookup order (the
            //     key region is dead by now). A dimension-split table deals its lookups round-robin
            //     over its NA workgroups (every wave gets some); a row split takes the rows of its
            //     own range; the last arriver also the stalled workgroups' shares.
            int64_t nx[MAXI];
#pragma unroll
            for (int i = 0; i < MAXI; ++i) {
                const int b = tid + TPB * i;
                if constexpr (DQRM_FWD_EARLY_IDX) nx[i] = nxe[i];
                else nx[i] = b < B ? la.fwd_idx[(int64_t)t * B + b] : -1;
            }
            const int me = s + SPLIT * j;
            const uint32_t smask = s_lastarr ? (uint32_t)s_stallmask : 0u;
            const int lane = tid % WAVE;
            uint64_t* lst = keys + w * (WAVE * MAXI);
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < MAXI; ++i) {
                const int b = tid + TPB * i;
                const int64_t x = nx[i];
                const bool okr = x >= 0 && x < nrows;
                int own = 0;
                if (dsplit) {
                    own = b % NA;
                } else if (okr) {
                    const int sl = slot_of_row(x, nblk);
                    int jj = 0;
                    if (K == 2) {
                        const int64_t b0 = nblk * sl / SPLIT, b1 = nblk * (sl + 1) / SPLIT;
                        jj = (x >> 8) >= (b0 + b1) / 2 ? 1 : 0;
                    }
                    own = sl + SPLIT * jj;
                }
                const bool mine = b < B && ((own == me && go) || ((smask >> own) & 1u));
                const uint64_t m = __ballot(mine);
                if (mine) {
                    const int p = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    lst[p] = ((uint64_t)(okr ? (uint32_t)x : 0xFFFFFFFFu) << 32) | (uint32_t)b;
                    if (!okr) flag_error(a.err, DQRM_ERRF_INDEX);
                }
                cnt += __popcll(m);
            }
            CDIAG(20);
            // (ii) a row split reads only rows it updated itself (or untouched ones): its first
            //      rows go out now, in flight across the wait for the table's final max. Plain
            //      loads: a workgroup's own stores are visible to it, and a dimension-split
            //      table's rows (other workgroups' stores, one XCD) were never loaded by this CU
            //      in this launch -- its slot ranges are block-aligned, no line is shared -- so
            //      they come from the XCD's L2, once the wait below has ordered them.
            const int G = LPR < WAVE ? WAVE / LPR : 1;  // rows per wave pass
            const int gl = lane / LPR, sub = lane % LPR;
            constexpr int FU = 4;  // rows per lane group in flight
            uint64_t e[FU];
            float4 v[FU];
            auto issue = [&](int p0) {
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const int ix = p0 + gl + G * u;
                    e[u] = ix < cnt && lane < G * LPR ? lst[ix] : ~0ull;
                }
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    const uint32_t x = (uint32_t)(e[u] >> 32);
                    v[u] = nrows > 0 ? reinterpret_cast<const float4*>(la.W + (rb + (x != 0xFFFFFFFFu ? x : 0u)) * a.D)[sub]
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            };
            if (!dsplit && cnt > 0) issue(0);
            // (iii) the table's final max: published by the last arriver (above, or at its
            //       arrival), the others wait for it
            if (!s_lastarr && tid == 0) {
                // a workgroup that stalled at the rendezvous leaves its share to the last arriver
                // and does not wait (its CU may be what a late workgroup of the table needs);
                // the others met every workgroup of the table there, so all of them arrive
                uint64_t g = 0;
                int ok = go ? 1 : 0;
                for (uint32_t spin = 0; ok; ++spin) {
                    g = __hip_atomic_load(fword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (gr_epoch(g) == epoch) break;
                    if (spin > (1u << 20)) {  // (never, all resident) flagged, this share skipped
                        flag_error(a.err, DQRM_ERRF_STALL);
                        ok = 0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                s_ftm = __uint_as_float((uint32_t)g);
                s_fok = ok;
            }
            __syncthreads();
            CDIAG(19);
            if (!s_fok) cnt = 0;  // (uniform)
            const float sf = fullp ? 1.0f : (refresh ? sym_scale(s_ftm, la.fwd_bits) : la.fwd_scale[t]);
            if (refresh && !fullp && s_lastarr && tid == 0) la.fwd_scale[t] = sf;
            const float rf = 1.0f / sf;
            const float fqlo = -(float)(1 << (la.fwd_bits - 1)), fqhi = (float)((1 << (la.fwd_bits - 1)) - 1);
            float* outt = la.fwd_out + (int64_t)t * la.fwd_ost_t;
            for (int p0 = 0; p0 < cnt; p0 += G * FU) {  // uniform per wave
                if (p0 > 0 || dsplit) issue(p0);  // (the first rows of a row split went out before the wait)
                if (p0 == 0) CDIAG_W(21);
#pragma unroll
                for (int u = 0; u < FU; ++u) {
                    if (e[u] == ~0ull) continue;
                    float4 y = (uint32_t)(e[u] >> 32) != 0xFFFFFFFFu ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
                    if (!fullp) {
                        y.x = fake_quant(y.x, rf, fqlo, fqhi) * sf;
                        y.y = fake_quant(y.y, rf, fqlo, fqhi) * sf;
                        y.z = fake_quant(y.z, rf, fqlo, fqhi) * sf;
                        y.w = fake_quant(y.w, rf, fqlo, fqhi) * sf;
                    }
                    reinterpret_cast<float4*>(outt + (int64_t)(uint32_t)e[u] * la.fwd_ost_b)[sub] = y;
                }
            }
            CDIAG_W(18);  // (diagnostic build: the next batch's forward done)
        }
    }
}

}  // namespace

namespace {
// the attribute is per function, process-wide: set once (thread-safe), re-checked each call
hipError_t allow_coalesce_lds() {
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
        const void* fns[] = {reinterpret_cast<const void*>(k_coalesce_p1<false, false, false>),
                             reinterpret_cast<const void*>(k_coalesce_p1<false, true, false>),
                             reinterpret_cast<const void*>(k_coalesce_p1<true, false, false>),
                             reinterpret_cast<const void*>(k_coalesce_p1<true, true, false>),
                             reinterpret_cast<const void*>(k_coalesce_p1<true, false, true>),
                             reinterpret_cast<const void*>(k_coalesce_p1<true, true, true>)};
        for (const void* f : fns)
            if (attr == hipSuccess) attr = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    });
    return attr;
}
}  // namespace

namespace dqrm_internal {

int coalesce_apply_grid(int T) { return (T + 7) / 8 * 64; }

void plan_table_groups(const int64_t* num_rows_host, int T, LocalApplyArgs* la);

void plan_sub_slots(const int64_t* num_rows_host, int T, LocalApplyArgs* la) {
    static const bool off = [] {
        const char* e = getenv("DQRM_SUBSLOTS");
        return e && !strcmp(e, "0");
    }();
    la->sub_mask = 0;
    for (int e = 0; e < kSubTables; ++e) la->sub_table[e] = -1;
    if (off || !num_rows_host || T <= 0 || T > kCoalesceApplyMaxT) return;
    const int nextra = coalesce_apply_grid(T) / SPLIT - T;  // spare groups of 8 workgroups
    // eligible: row-split tables of >= 16 row blocks (each half-slot keeps >= 1 block), by row
    // blocks descending, ties by table index
    int order[kCoalesceApplyMaxT];
    int64_t nb[kCoalesceApplyMaxT];
    int ne = 0;
    for (int t = 0; t < T; ++t) {
        nb[t] = (num_rows_host[t] + BLK - 1) / BLK;
        if (nb[t] >= 2 * SPLIT) order[ne++] = t;
    }
    // DQRM_SUBSLOT_ORDER=small (A/B): the smallest eligible tables first (their slots hold
    // duplicate-heavy lookups: sort, ordered sums, block re-reductions), not the largest
    static const bool small_first = [] {
        const char* e = getenv("DQRM_SUBSLOT_ORDER");
        return e && !strcmp(e, "small");
    }();
    if (small_first) std::stable_sort(order, order + ne, [&](int x, int y) { return nb[x] < nb[y]; });
    else std::stable_sort(order, order + ne, [&](int x, int y) { return nb[x] > nb[y]; });
    for (int e = 0; e < nextra && e < ne && e < kSubTables; ++e) {
        la->sub_table[e] = (int8_t)order[e];
        la->sub_mask |= 1u << order[e];
    }
    plan_table_groups(num_rows_host, T, la);
}

// DQRM_TABLE_GROUPS=critical (A/B): the groups a table's 8 slots run in, XCD by XCD (group g's
// workgroups share XCD g % 8), filled with the tables expected to end last first -- uneven
// row-split slots (8 < blocks < 16, not a multiple of 8), then a few-row tables' long ordered
// chains, then medium tables, the big distinct-row tables last
void plan_table_groups(const int64_t* num_rows_host, int T, LocalApplyArgs* la) {
    static const bool crit = [] {
        const char* e = getenv("DQRM_TABLE_GROUPS");
        return e && !strcmp(e, "critical");
    }();
    la->group_perm = 0;
    for (int g = 0; g < kSubTables; ++g) la->table_of_group[g] = (int8_t)g;
    if (!crit || !num_rows_host || T <= 0 || T > kCoalesceApplyMaxT) return;
    int score[kCoalesceApplyMaxT], tabs[kCoalesceApplyMaxT], groups[kCoalesceApplyMaxT];
    for (int t = 0; t < T; ++t) {
        const int64_t n = num_rows_host[t], nb = (n + BLK - 1) / BLK;
        score[t] = n >= (1 << 20) ? 0 : (nb > SPLIT && nb < 2 * SPLIT && nb % SPLIT) ? 3 : (nb < SPLIT && n <= 64) ? 2 : 1;
        tabs[t] = t;
    }
    std::stable_sort(tabs, tabs + T, [&](int x, int y) { return score[x] > score[y]; });
    int ng = 0;
    for (int x = 0; x < SPLIT; ++x)
        for (int g = x; g < T; g += SPLIT) groups[ng++] = g;
    for (int i = 0; i < T; ++i) la->table_of_group[groups[i]] = (int8_t)tabs[i];
    la->group_perm = 1;
}

bool coalesce_apply_resident(int T, hipStream_t stream) {
    if (T <= 0 || T > kCoalesceApplyMaxT) return false;
    // per device, once: CUs x workgroups of k_coalesce_p1<true> a CU holds (1024 threads,
    // 156 KiB LDS: one). A query that fails counts as "does not fit".
    struct Dev { std::once_flag once; int cus = 0, occ = 0; };
    static Dev devs[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    Dev& d = devs[dev];
    std::call_once(d.once, [&d, dev] {
        int cus = 0, occ = 0;
        if (allow_coalesce_lds() != hipSuccess) return;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return;
        for (const void* f : {reinterpret_cast<const void*>(k_coalesce_p1<true, false, false>),
                              reinterpret_cast<const void*>(k_coalesce_p1<true, true, false>),
                              reinterpret_cast<const void*>(k_coalesce_p1<true, false, true>),
                              reinterpret_cast<const void*>(k_coalesce_p1<true, true, true>)}) {
            int o = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, TPB, LDS_BYTES) != hipSuccess) return;
            occ = occ == 0 || o < occ ? o : occ;
        }
        d.cus = cus;
        d.occ = occ;
    });
    const int grid = coalesce_apply_grid(T);
    if ((int64_t)d.occ * d.cus < grid) return false;  // e.g. a CPX partition (32 CUs)
    // the stream's CU mask (hipExtStreamCreateWithCUMask): every CU of the device must be
    // enabled, since the hardware deals the grid over the XCDs whatever the mask leaves
    uint32_t mask[32] = {};
    const int words = (d.cus + 31) / 32;
    if (words > 32) return false;
    if (stream == nullptr) {  // the legacy default stream has no mask of its own; a process-wide one
        const char* g = getenv("ROC_GLOBAL_CU_MASK");  // (HIP's global CU mask) is not assumed full
        const char* h = getenv("HSA_CU_MASK");
        return !(g && *g) && !(h && *h);
    }
    if (hipExtStreamGetCUMask(stream, (uint32_t)words, mask) != hipSuccess) return false;
    int on = 0;
    for (int i = 0; i < words; ++i) on += __builtin_popcount(mask[i]);
    return on >= d.cus;
}

hipError_t launch_coalesce_pool1(const CoalesceArgs& a, const LocalApplyArgs* la, hipStream_t stream) {
    const hipError_t attr = allow_coalesce_lds();
    if (attr != hipSuccess) return attr;
    const dim3 grid((a.T + 7) / 8 * 64);
    const bool rm = DQRM_COAL_ROWMAJOR == 2 || (DQRM_COAL_ROWMAJOR == 1 && a.D >= 32);  // stage layout
    if (la) {
        if (!coalesce_apply_resident(a.T, stream)) return hipErrorInvalidValue;  // not all resident at once
        static const uint32_t spin = [] {  // DQRM_STALL_SPIN: rendezvous polls before a stall (tests)
            const char* e = getenv("DQRM_STALL_SPIN");
            return e ? (uint32_t)strtoul(e, nullptr, 10) : (1u << 20);
        }();
        LocalApplyArgs l2 = *la;
        l2.spin_limit = spin;
        const bool fwd = l2.fwd_idx != nullptr;
        if (rm && fwd) hipLaunchKernelGGL((k_coalesce_p1<true, true, true>), grid, dim3(TPB), LDS_BYTES, stream, a, l2);
        else if (fwd) hipLaunchKernelGGL((k_coalesce_p1<true, false, true>), grid, dim3(TPB), LDS_BYTES, stream, a, l2);
        else if (rm) hipLaunchKernelGGL((k_coalesce_p1<true, true, false>), grid, dim3(TPB), LDS_BYTES, stream, a, l2);
        else hipLaunchKernelGGL((k_coalesce_p1<true, false, false>), grid, dim3(TPB), LDS_BYTES, stream, a, l2);
    } else {
        if (rm) hipLaunchKernelGGL((k_coalesce_p1<false, true, false>), grid, dim3(TPB), LDS_BYTES, stream, a, LocalApplyArgs{});
        else hipLaunchKernelGGL((k_coalesce_p1<false, false, false>), grid, dim3(TPB), LDS_BYTES, stream, a, LocalApplyArgs{});
    }
    return hipGetLastError();
}

}  // namespace dqrm_internal

#ifdef DQRM_DIAG_CLOCK
extern "C" int dqrm_diag_coal_read(unsigned long long* host, int n) {
    if (hipDeviceSynchronize() != hipSuccess) return DQRM_E_HIP;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_coal_clk), (size_t)n * sizeof(unsigned long long)) != hipSuccess)
        return DQRM_E_HIP;
    return DQRM_OK;
}
#endif
