// dqrm_device.h — device helpers shared by the translation units of libdqrm (not part
// of the C ABI): table metadata, the quantization arithmetic, write-through stores and
// dirty flags of the |W| hierarchy, the in-launch hand-off and the table finalize.
#pragma once

#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "../../include/dqrm.h"

#define DQRM_INLINE __device__ __forceinline__

namespace {

constexpr int WAVE = 64;
constexpr int BLK = DQRM_BLOCK_ROWS;     // 256
constexpr int SBLK_BLOCKS = 256;         // blocks per superblock

// ------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------
struct Meta {
    const int64_t* row_base;
    const int64_t* num_rows;
    const int64_t* blk_base;
    const int64_t* sblk_base;
};

DQRM_INLINE Meta make_meta(const int64_t* m, int T) {
    return Meta{m, m + T, m + 2 * T, m + 3 * T};
}

DQRM_INLINE int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// largest t with base[t] <= x (base ascending, base[0] == 0)
DQRM_INLINE int find_table(const int64_t* base, int T, int64_t x) {
    int lo = 0, hi = T - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (base[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// symmetric scale: clamp(absmax, min=1e-8) / (2^(bits-1)-1)      quant_utils.py:189-192
DQRM_INLINE float sym_scale(float absmax, int bits) {
    const float n = (float)((1 << (bits - 1)) - 1);
    float a = absmax < 1e-8f ? 1e-8f : absmax;
    return a / n;
}

// linear_quantize + clamp: clamp(round(1/s * x + 0), -n-1, n)  quant_utils.py:101,343
// r = 1/s is precomputed by the caller with an IEEE division (torch: reciprocal(s)*1.0).
DQRM_INLINE float fake_quant(float x, float r, float lo, float hi) {
    float t = r * x;
    t = t + 0.0f;          // `+ zero_point` (zero_point = 0): turns -0 products into +0
    t = rintf(t);          // torch.round: half to even
    t = fmaxf(t, lo);      // torch.clamp(min) then (max)
    t = fminf(t, hi);
    return t;
}

DQRM_INLINE float abs_max4(float4 v) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}

// max over a group of `G` consecutive lanes (G power of two <= 64)
template <int G>
DQRM_INLINE float group_max(float v) {
#pragma unroll
    for (int m = 1; m < G; m <<= 1) v = fmaxf(v, __shfl_xor(v, m, WAVE));
    return v;
}

DQRM_INLINE float wave_max(float v) { return group_max<WAVE>(v); }

// pack 4 quantized values (ints in [-8,7] held as float) into 2 offset-binary bytes
DQRM_INLINE uint16_t pack4_int4(float q0, float q1, float q2, float q3) {
    uint32_t n0 = (uint32_t)((int)q0 + 8), n1 = (uint32_t)((int)q1 + 8);
    uint32_t n2 = (uint32_t)((int)q2 + 8), n3 = (uint32_t)((int)q3 + 8);
    return (uint16_t)(n0 | (n1 << 4) | (n2 << 8) | (n3 << 12));
}

DQRM_INLINE void flag_error(uint32_t* err, uint32_t f) { atomicOr(err, f); }

// ------------------------------------------------------------------------------------
// In-launch hand-off of the |W| hierarchy to a table's last workgroup (no finalize launch).
// MI355X_MICROARCH.md "inter-workgroup visibility", hand-off row 1: every byte the last
// workgroup reads was stored write-through (sc1 stores, or device-scope atomics), every
// storing wave waits vmcnt(0), a workgroup barrier, then ONE lane adds to the table's
// arrival counter; the workgroup whose add returns expected-1 reads with sc1 loads only.
// No L2 write-back (release fence) and no L1 invalidate (acquire) on either side.
// ------------------------------------------------------------------------------------
DQRM_INLINE void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DQRM_INLINE float ld_wt(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DQRM_INLINE uint32_t ld_wt(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 bytes another workgroup of the launch stored write-through, as two 8-B agent-scope loads
// (global_load_dwordx2 ... sc1: past this CU's L1, tracked by the compiler's vmcnt accounting;
// a 64-bit address, unlike a buffer load's 32-bit offset). p 16-B aligned.
DQRM_INLINE float4 ld4_wt(const float* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)),
                       __uint_as_float((uint32_t)hi), __uint_as_float((uint32_t)(hi >> 32)));
}
// 16-B write-through store (global_store_dwordx4 ... sc1)
DQRM_INLINE void st4_wt(float4* p, float4 v) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}
// W stores of a narrow table (<= 256 rows: finalize rebuilds its maxima from W) go write-through
DQRM_INLINE void st4_w(float4* p, float4 v, bool wt) {
    if (wt) st4_wt(p, v); else *p = v;
}
DQRM_INLINE void st_w(float* p, float v, bool wt) {
    if (wt) st_wt(p, v); else *p = v;
}

// dirty flags (u8 arrays sdirty / bdirty) are set / cleared by device-scope atomics on their
// aligned 32-bit word and read with sc1 word loads (the arrays are padded to whole words)
// (the word pointer is derived from f by pointer arithmetic, not through an integer, so the
// compiler keeps f's global address space: global atomics, not flat ones -- a pending flat
// atomic makes every later LDS access wait for all of the wave's stores, vmcnt(0) lgkmcnt(0))
DQRM_INLINE uint32_t* flag_word(const uint8_t* f, int64_t i, int* sh) {
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(f + i) & 3u);
    *sh = (int)mis * 8;
    return reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(f + i - mis));
}
DQRM_INLINE void flag_set(uint8_t* f, int64_t i) {
    int sh;
    uint32_t* w = flag_word(f, i, &sh);
    atomicOr(w, 1u << sh);
}
DQRM_INLINE void flag_clear(uint8_t* f, int64_t i) {
    int sh;
    uint32_t* w = flag_word(f, i, &sh);
    atomicAnd(w, ~(0xFFu << sh));
}
DQRM_INLINE bool flag_get(const uint8_t* f, int64_t i) {
    int sh;
    const uint32_t* w = flag_word(f, i, &sh);
    return ((ld_wt(w) >> sh) & 0xFFu) != 0u;
}

// Word FLAG_WORD of a table's sync words: set (atomicOr) by the flat apply kernels whenever
// they flag a block / superblock of the table; the finalize launch that follows them skips a
// table whose word is clear (its |W| maxima are exact already: growth went in by atomicMax)
// and clears it otherwise.
constexpr int FLAG_WORD = 2;
DQRM_INLINE void mark_table_flagged(uint32_t* sync, int t) {
    atomicOr(sync + (int64_t)t * DQRM_SYNC_STRIDE + FLAG_WORD, 1u);
}

// loads of the finalize: sc1 inside the updating launch (WT), plain in a launch of its own
template <bool WT> DQRM_INLINE float ld_h(const float* p) { if constexpr (WT) return ld_wt(p); else return *p; }
template <bool WT> DQRM_INLINE uint32_t ld_h(const uint32_t* p) { if constexpr (WT) return ld_wt(p); else return *p; }
template <bool WT> DQRM_INLINE bool flag_get_h(const uint8_t* f, int64_t i) {
    int sh;
    const uint32_t* w = flag_word(f, i, &sh);
    return ((ld_h<WT>(w) >> sh) & 0xFFu) != 0u;
}

// All threads of the workgroup call this after their last store for table t; returns
// (uniformly) whether this is the last of the `expected` arriving workgroups. The last one
// re-arms the counter for the next launch.
DQRM_INLINE bool arrive_last(uint32_t* cnt, uint32_t expected) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores and atomics have landed
    __syncthreads();                                   // ... and every other wave's
    if (threadIdx.x == 0) {
        const uint32_t old = atomicAdd(cnt, 1u);
        const bool last = old + 1u == expected;
        if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last ? 1 : 0;
    }
    __syncthreads();
    return s_last != 0;
}

// INT4-pack the 4 dims of float4 number idx4 of a row (prow = the row's packed bytes)
DQRM_INLINE void pack4_row(const float4 w, uint8_t* __restrict__ prow, int idx4, float r) {
    float q0 = fake_quant(w.x, r, -8.0f, 7.0f), q1 = fake_quant(w.y, r, -8.0f, 7.0f);
    float q2 = fake_quant(w.z, r, -8.0f, 7.0f), q3 = fake_quant(w.w, r, -8.0f, 7.0f);
    reinterpret_cast<uint16_t*>(prow)[idx4] = pack4_int4(q0, q1, q2, q3);
}

// Per table, after its slot workgroups: re-reduce flagged superblocks, then tmax over all
// superblocks. Narrow tables (<= 256 rows, dimension-split in the slot kernels) get their
// rowmax, block, superblock and table maxima rebuilt from W here (<= 256 rows x D floats),
// unless rebuild_narrow is false (the updating kernel kept them exact like any table's).
// WTS: the table max is stored write-through (read by other workgroups of the launch); U4:
// loads in flight per thread in the flag and superblock scans; FB: flagged superblocks a wave
// fixes at once (> 1: 3 KiB more LDS, for the finalize launches, not the in-launch finalizes). on_final() is called once by every
// thread of the workgroup as soon as the table max is final: with `tracked`, right after the flag
// scan when no flagged superblock held the table max (the rest only fixes lower levels), else at
// the end (k_finalize_fwd opens the table's forward gate there).
struct NoFinal {
    DQRM_INLINE void operator()() const {}
};
template <bool WT, bool WTS = WT, int U4 = 4, int FB = 1, class OnFinal = NoFinal>
DQRM_INLINE void finalize_table(const Meta& m, int t, const float* __restrict__ W, float* __restrict__ rowmax,
                               float* __restrict__ blkmax, float* __restrict__ sblkmax,
                               uint8_t* __restrict__ sdirty, uint8_t* __restrict__ bdirty, float* __restrict__ tmax,
                               int D, bool tracked, bool rebuild_narrow = true, OnFinal on_final = OnFinal()) {
    // Every load below is an sc1 (write-through) load: this runs either as its own launch or
    // in the table's last workgroup of the updating kernel (arrive_last), whose producers
    // stored the hierarchy write-through.
    __shared__ float red[16];
    __shared__ int s_rescan;
    if (rebuild_narrow && m.num_rows[t] <= BLK) {
        const int64_t grow = m.row_base[t] + threadIdx.x;
        float v = 0.0f;
        if (threadIdx.x < m.num_rows[t]) {
            const float* wr = W + grow * D;
            if constexpr (WT) {
                for (int k0 = 0; k0 < D; k0 += 16) {  // 16 loads in flight
                    float x[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) x[j] = k0 + j < D ? ld_h<WT>(wr + k0 + j) : 0.0f;
#pragma unroll
                    for (int j = 0; j < 16; ++j) v = fmaxf(v, fabsf(x[j]));
                }
            } else {
                for (int k = 0; k < D / 4; ++k) v = fmaxf(v, abs_max4(reinterpret_cast<const float4*>(wr)[k]));
            }
            rowmax[grow] = v;
        }
        v = wave_max(v);
        if (threadIdx.x % WAVE == 0) red[threadIdx.x / WAVE] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float r = 0.0f;
            for (int k = 0; k < (int)(blockDim.x / WAVE); ++k) r = fmaxf(r, red[k]);
            blkmax[m.blk_base[t]] = r;
            sblkmax[m.sblk_base[t]] = r;
            if (flag_get_h<WT>(sdirty, m.sblk_base[t])) flag_clear(sdirty, m.sblk_base[t]);
            if (flag_get_h<WT>(bdirty, m.blk_base[t])) flag_clear(bdirty, m.blk_base[t]);
            if constexpr (WTS) st_wt(tmax + t, r); else tmax[t] = r;  // WT: read by other workgroups
        }
        on_final();
        return;
    }
    const int64_t nblk = ceil_div(m.num_rows[t], BLK);
    const int64_t ns = ceil_div(nblk, SBLK_BLOCKS);
    const int64_t sbb = m.sblk_base[t], bb = m.blk_base[t];
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    // tracked (flat apply kernels): tmax already holds every grown row max (atomicMax), so
    // the table-wide rescan is needed only if a rescanned superblock held the table max
    const float tmax0 = tracked ? ld_h<WT>(tmax + t) : 0.0f;
    if (threadIdx.x == 0) s_rescan = tracked ? 0 : 1;
    __syncthreads();
    // the table's superblock flags, 4 per 32-bit word (word 0 holds superblock 0 at byte sh0)
    int sh0;
    const uint32_t* sdw = flag_word(sdirty, sbb, &sh0);
    sh0 /= 8;
    const int64_t nwords = (ns + sh0 + 3) / 4;
    // one superblock whose max holder shrank, by one wave: re-reduce its flagged blocks' 256
    // rowmax (the owning lane keeps the new block max in a register), then the superblock
    auto fix_superblock = [&](int64_t sb) {
        const int64_t b0 = sb * SBLK_BLOCKS, b1 = b0 + SBLK_BLOCKS < nblk ? b0 + SBLK_BLOCKS : nblk;
        float nv[SBLK_BLOCKS / WAVE];
        bool dq[SBLK_BLOCKS / WAVE];
        const float old_sb = ld_h<WT>(sblkmax + sbb + sb);  // with the flags and block maxima: one round trip
#pragma unroll
        for (int q = 0; q < SBLK_BLOCKS / WAVE; ++q) {
            const int64_t b = b0 + lane + q * WAVE;
            dq[q] = b < b1 && flag_get_h<WT>(bdirty, bb + b);
            nv[q] = b < b1 ? ld_h<WT>(blkmax + bb + b) : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < SBLK_BLOCKS / WAVE; ++q) {
            uint64_t dm = __ballot(dq[q]);
            while (dm) {  // up to DB dirty blocks per pass, all their loads in flight
                constexpr int DB = 8;
                int dl[DB];
                float x[DB];
#pragma unroll
                for (int i = 0; i < DB; ++i) {
                    dl[i] = dm ? __ffsll((long long)dm) - 1 : -1;  // wave-uniform
                    dm &= dm ? dm - 1 : 0;
                }
#pragma unroll
                for (int i = 0; i < DB; ++i) {
                    x[i] = 0.0f;
                    if (dl[i] < 0) continue;
                    const int64_t blk = b0 + q * WAVE + dl[i];
#pragma unroll
                    for (int k = 0; k < BLK / WAVE; ++k) {
                        const int64_t rr = blk * BLK + lane + k * WAVE;
                        if (rr < m.num_rows[t]) x[i] = fmaxf(x[i], ld_h<WT>(rowmax + m.row_base[t] + rr));
                    }
                }
#pragma unroll
                for (int i = 0; i < DB; ++i) {
                    if (dl[i] < 0) continue;
                    const float y = wave_max(x[i]);
                    if (lane == dl[i]) nv[q] = y;
                }
            }
            if (dq[q]) { blkmax[b0 + lane + q * WAVE + bb] = nv[q]; flag_clear(bdirty, b0 + lane + q * WAVE + bb); }
        }
        float v = 0.0f;
#pragma unroll
        for (int q = 0; q < SBLK_BLOCKS / WAVE; ++q) v = fmaxf(v, nv[q]);
        v = wave_max(v);
        if (lane == 0) {
            sblkmax[sbb + sb] = v;
            flag_clear(sdirty, sbb + sb);
            if (v < old_sb && old_sb >= tmax0) s_rescan = 1;  // the table max may have shrunk
        }
    };
    // up to FB listed superblocks whose max holder shrank (list entries i0, i0 + nw, ...), by one
    // wave, all their loads in flight together: their flags and block maxima (one round trip),
    // then their flagged blocks' 256 rowmax DB blocks at a time (the owning lane keeps the new
    // block max in a register), then the superblocks
    constexpr int Q = SBLK_BLOCKS / WAVE, DB = 8;
    __shared__ int s_fx[FB > 1 ? 16 : 1][2 * DB];  // per wave: the dirty blocks of a pass (combo f*Q+q, lane)
    __shared__ uint64_t s_dm[FB > 1 ? 16 : 1][FB * Q];  // per wave: each combo's dirty-lane ballot
    auto fix_batch = [&](const int* lst, int i0, int n) {
        int64_t b0[FB];
        float nv[FB][Q], old_sb[FB];
        bool dq[FB][Q];
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            const int i = i0 + f * nw;
            const bool act = i < n;
            const int64_t sb = act ? lst[i] : 0;
            b0[f] = sb * SBLK_BLOCKS;
            const int64_t b1 = act ? (b0[f] + SBLK_BLOCKS < nblk ? b0[f] + SBLK_BLOCKS : nblk) : b0[f];
            old_sb[f] = act ? ld_h<WT>(sblkmax + sbb + sb) : 0.0f;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int64_t b = b0[f] + lane + q * WAVE;
                dq[f][q] = b < b1 && flag_get_h<WT>(bdirty, bb + b);
                nv[f][q] = b < b1 ? ld_h<WT>(blkmax + bb + b) : 0.0f;
            }
        }
        int* fx = s_fx[w];
        auto flush = [&](int cnt) {  // cnt (wave-uniform) dirty blocks listed in fx
            float x[DB];
#pragma unroll
            for (int i = 0; i < DB; ++i) {
                x[i] = 0.0f;
                if (i >= cnt) continue;
                const int c = fx[2 * i], l = fx[2 * i + 1];
                int64_t base = 0;
#pragma unroll
                for (int f = 0; f < FB; ++f)
                    if (c / Q == f) base = b0[f];
                const int64_t blk = base + (c % Q) * WAVE + l;
#pragma unroll
                for (int k = 0; k < BLK / WAVE; ++k) {
                    const int64_t rr = blk * BLK + lane + k * WAVE;
                    if (rr < m.num_rows[t]) x[i] = fmaxf(x[i], ld_h<WT>(rowmax + m.row_base[t] + rr));
                }
            }
#pragma unroll
            for (int i = 0; i < DB; ++i) {
                if (i >= cnt) continue;
                const float y = wave_max(x[i]);
                const int c = fx[2 * i], l = fx[2 * i + 1];
#pragma unroll
                for (int f = 0; f < FB; ++f)
#pragma unroll
                    for (int q = 0; q < Q; ++q)
                        if (c == f * Q + q && lane == l) nv[f][q] = y;
            }
        };
        uint64_t* dms = s_dm[w];
#pragma unroll
        for (int f = 0; f < FB; ++f)
#pragma unroll
            for (int q = 0; q < Q; ++q) dms[f * Q + q] = __ballot(dq[f][q]);  // every lane: the same word
        int cnt = 0;
#pragma unroll 1
        for (int c = 0; c < FB * Q; ++c) {
            uint64_t dm = dms[c];
            while (dm) {  // wave-uniform
                fx[2 * cnt] = c;
                fx[2 * cnt + 1] = __ffsll((long long)dm) - 1;
                dm &= dm - 1;
                if (++cnt == DB) {
                    flush(DB);
                    cnt = 0;
                }
            }
        }
        if (cnt) flush(cnt);
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            if (i0 + f * nw >= n) break;  // uniform
            float v = 0.0f;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int64_t b = b0[f] + lane + q * WAVE;
                if (dq[f][q]) { blkmax[b + bb] = nv[f][q]; flag_clear(bdirty, b + bb); }
                v = fmaxf(v, nv[f][q]);
            }
            v = wave_max(v);
            if (lane == 0) {
                const int64_t sb = b0[f] / SBLK_BLOCKS;
                sblkmax[sbb + sb] = v;
                flag_clear(sdirty, sbb + sb);
                if (v < old_sb[f] && old_sb[f] >= tmax0) s_rescan = 1;  // the table max may have shrunk
            }
        }
    };
    // 1. list the flagged superblocks in LDS (one scan of the flag words); 2. one wave per
    // listed superblock. A list that overflows is finished by another scan (the fixed
    // superblocks' flags are clear by then).
    constexpr int FIN_LIST = 128;
    __shared__ int s_dl[FIN_LIST];
    __shared__ int s_dn;
    bool early = false;  // on_final() already called
    bool first = true;
    for (;;) {
        if (threadIdx.x == 0) s_dn = 0;
        __syncthreads();
        for (int64_t k0 = (int64_t)threadIdx.x; k0 < nwords; k0 += (int64_t)blockDim.x * U4) {
            uint32_t fw[U4];
#pragma unroll
            for (int j = 0; j < U4; ++j) {
                const int64_t k = k0 + (int64_t)j * blockDim.x;
                uint32_t x = k < nwords ? ld_h<WT>(sdw + k) : 0u;
                if (k == 0) x &= 0xFFFFFFFFu << (8 * sh0);            // bytes before superblock 0
                const int64_t nb = ns + sh0 - k * 4;                   // valid bytes in this word
                if (nb < 4) x &= nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u);
                fw[j] = x;
            }
#pragma unroll
            for (int j = 0; j < U4; ++j) {
                uint32_t x = fw[j];
                while (x) {  // rare: a superblock's max holder shrank
                    const int by = (__ffs((int)x) - 1) / 8;
                    x &= ~(0xFFu << (8 * by));
                    const int p = atomicAdd(&s_dn, 1);
                    if (p < FIN_LIST) s_dl[p] = (int)((k0 + (int64_t)j * blockDim.x) * 4 + by - sh0);
                }
            }
        }
        __syncthreads();
        const int nd = s_dn;
        if (!std::is_same<OnFinal, NoFinal>::value && tracked && first && nd <= FIN_LIST) {  // can the table max shrink?
            int hit = 0;
            for (int i = threadIdx.x; i < nd; i += blockDim.x) hit |= ld_h<WT>(sblkmax + sbb + s_dl[i]) >= tmax0;
            if (!__syncthreads_or(hit)) {
                on_final();
                early = true;
            }
        }
        first = false;
        const int nl = nd < FIN_LIST ? nd : FIN_LIST;
        if constexpr (FB > 1) {
            for (int i0 = w; i0 < nl; i0 += nw * FB) fix_batch(s_dl, i0, nl);
        } else {
            for (int i = w; i < nl; i += nw) fix_superblock(s_dl[i]);
        }
        if (nd <= FIN_LIST) break;  // uniform
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // cleared flags land before the next scan
        __syncthreads();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the new superblock maxima reach L2 first
    __syncthreads();
    if (!s_rescan) {  // uniform: tmax is exact already
        if (!early) on_final();
        return;
    }
    float v = 0.0f;
    for (int64_t k0 = threadIdx.x; k0 < ns; k0 += (int64_t)blockDim.x * U4) {
        float x[U4];
#pragma unroll
        for (int j = 0; j < U4; ++j) {
            const int64_t k = k0 + (int64_t)j * blockDim.x;
            x[j] = k < ns ? ld_h<WT>(sblkmax + sbb + k) : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < U4; ++j) v = fmaxf(v, x[j]);
    }
    v = wave_max(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = 0.0f;
        for (int k = 0; k < nw; ++k) r = fmaxf(r, red[k]);
        if constexpr (WTS) st_wt(tmax + t, r); else tmax[t] = r;  // WT: read by other workgroups (sc1)
    }
    if (!early) on_final();
}

// One rank's wire payload: [counts i32 T*SPLIT][rows i32 cap][values cap x D], 16-B aligned
// sections (dqrm_payload_bytes); values int8 (bits <= 8), int16 (<= 16) or f32 (32)
struct PayloadLayout {
    int64_t rows_off;   // bytes
    int64_t vals_off;   // bytes
    int64_t bytes;
    int elem;           // bytes per value
};

__host__ __device__ inline int64_t align16(int64_t x) { return (x + 15) & ~int64_t(15); }

__host__ __device__ inline PayloadLayout payload_layout(int T, int64_t cap, int D, int bits) {
    PayloadLayout p;
    p.elem = bits <= 8 ? 1 : (bits <= 16 ? 2 : 4);
    p.rows_off = align16(4 * (int64_t)T * DQRM_TABLE_SPLIT);  // header: entries per (table, slot)
    p.vals_off = p.rows_off + align16(4 * cap);
    p.bytes = p.vals_off + align16(cap * (int64_t)D * p.elem);
    return p;
}

// dequantize + SGD of one element: update.mul_(1/N), grad * s.item(), W.add_(-lr * .)
struct ApplyUpdate {
    int mode;
    float inv_n, sc, sim_f, nlr;
    DQRM_INLINE float operator()(float w, float acc) const {
        float v;
        if (mode == DQRM_UPD_DP) v = (acc * inv_n) * sc;                  // s_q_g_p_c.py:885,618-622
        else if (mode == DQRM_UPD_SIMULATED) v = acc * sim_f;            // sgd_quantized_gradients.py:366-371
        else v = acc * inv_n;                                            // FP32 sparse all_reduce (:319-327)
        return w + nlr * v;  // separately rounded product, then add
    }
};

}  // namespace
