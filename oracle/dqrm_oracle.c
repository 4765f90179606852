/*
 * dqrm_oracle.c — CPU restatement of the reference's DQRM embedding QAT path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product links or calls this file; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker
 * and as the timed CPU baseline ("kind": "port").
 *
 * Parity pin: the reference Python cannot be imported in this environment (denied; see
 * DESIGN.md) and ships no golden vectors. This restatement is pinned against fixtures
 * that tests/golden/make_golden.py generates by running the reference's call sequence
 * with the real third-party library the arithmetic lives in (PyTorch 2.10 CPU:
 * nn.EmbeddingBag(sparse=True), torch.round/clamp, Tensor.coalesce, torch.optim.SGD,
 * Gloo sparse all_reduce).
 *
 * Compile: gcc -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile). Every rounding
 * below is an explicit IEEE single operation; fmaf() appears only where torch's CPU
 * kernel performs a fused multiply-add (the sparse SGD axpy).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_ERR_INDEX 1u
#define ORACLE_ERR_OFFSET 2u

/* quant_utils.py:189-192: scale = clamp(max(|wmin|,|wmax|), min=1e-8) / (2^(b-1)-1) */
float oracle_sym_scale(float absmax, int bits) {
    const float n = (float)((1 << (bits - 1)) - 1);
    float a = absmax < 1e-8f ? 1e-8f : absmax;
    return a / n;
}

/* quant_utils.py:177-178: w_min = min(min(W,0)), w_max = max(max(W,0)); max(|.|,|.|) */
float oracle_table_absmax(const float* W, int64_t n, int D) {
    float wmin = INFINITY, wmax = -INFINITY;
    for (int64_t i = 0; i < n * (int64_t)D; ++i) {
        if (W[i] < wmin) wmin = W[i];
        if (W[i] > wmax) wmax = W[i];
    }
    if (n == 0) return 0.0f;
    float a = fabsf(wmin), b = fabsf(wmax);
    return b > a ? b : a;
}

/* quant_utils.py:101 + :343: q = clamp(round(1/s * x + 0), -n-1, n), round = half-even */
static inline float fake_quant(float x, float r, float lo, float hi) {
    float t = r * x;
    t = t + 0.0f;
    t = nearbyintf(t); /* default rounding mode: to nearest, ties to even */
    if (t < lo) t = lo;
    if (t > hi) t = hi;
    return t;
}

static void bag_range(const int64_t* off, int64_t B, int64_t L, int64_t b, int64_t* s0, int64_t* s1,
                      uint32_t* err) {
    int64_t a = off[b];
    int64_t e = (b + 1 < B) ? off[b + 1] : L;
    if (a < 0 || e > L || e < a) {
        if (err) *err |= ORACLE_ERR_OFFSET;
        a = a < 0 ? 0 : (a > L ? L : a);
        e = e < a ? a : (e > L ? L : e);
    }
    *s0 = a;
    *s1 = e;
}

/* QuantEmbeddingBagTwo.forward (quant_modules_not_quantize_grad.py:317-398), one table:
 * out = embedding_bag(idx, off, mode="sum") (:367, FP32, bag order from 0);
 * if !full_precision: y = fake_quant(out) * s (:378,:393). */
void oracle_emb_fwd(const float* W, int64_t n, int D, const int64_t* idx, int64_t L,
                    const int64_t* off, int64_t B, float s, int bits, int full_precision,
                    float* out, uint32_t* err) {
    const float r = 1.0f / s;
    const float lo = -(float)(1 << (bits - 1)), hi = (float)((1 << (bits - 1)) - 1);
    float* acc = (float*)malloc(sizeof(float) * (size_t)D);
    for (int64_t b = 0; b < B; ++b) {
        int64_t s0, s1;
        bag_range(off, B, L, b, &s0, &s1, err);
        for (int d = 0; d < D; ++d) acc[d] = 0.0f;
        for (int64_t p = s0; p < s1; ++p) {
            int64_t row = idx[p];
            if (row < 0 || row >= n) {
                if (err) *err |= ORACLE_ERR_INDEX;
                continue;
            }
            for (int d = 0; d < D; ++d) acc[d] = acc[d] + W[row * D + d];
        }
        for (int d = 0; d < D; ++d)
            out[b * D + d] = full_precision ? acc[d] : fake_quant(acc[d], r, lo, hi) * s;
    }
    free(acc);
}

/* SymmetricQuantFunction.backward (quant_utils.py:349-363) after autograd of q*s:
 * g' = (g * s) / s; EmbeddingBag sparse backward values[i] = g'[bag(i)] (uncoalesced, in
 * lookup order); torch.optim.SGD.step: dense.add_(sparse, alpha=-lr) = per entry, in
 * order, w = fma(v, -lr, w) (torch CPU axpy). */
void oracle_emb_bwd_sgd(float* W, int64_t n, int D, const int64_t* idx, int64_t L, const int64_t* off,
                        int64_t B, const float* dy, float s, int ste, float lr, uint32_t* err) {
    const float nlr = -lr;
    /* lookup order = position order p; bag(p) from the offsets */
    int64_t* bag_of = (int64_t*)malloc(sizeof(int64_t) * (size_t)(L > 0 ? L : 1));
    for (int64_t p = 0; p < L; ++p) bag_of[p] = -1;
    for (int64_t b = 0; b < B; ++b) {
        int64_t s0, s1;
        bag_range(off, B, L, b, &s0, &s1, err);
        for (int64_t p = s0; p < s1; ++p) bag_of[p] = b;
    }
    for (int64_t p = 0; p < L; ++p) {
        const int64_t row = idx[p], b = bag_of[p];
        if (b < 0) continue;
        if (row < 0 || row >= n) {
            if (err) *err |= ORACLE_ERR_INDEX;
            continue;
        }
        for (int d = 0; d < D; ++d) {
            float g = dy[b * D + d];
            if (ste) g = (g * s) / s;
            W[row * D + d] = fmaf(g, nlr, W[row * D + d]);
        }
    }
    free(bag_of);
}

static int cmp_pair(const void* a, const void* b) {
    const int64_t* x = (const int64_t*)a;
    const int64_t* y = (const int64_t*)b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    if (x[1] != y[1]) return x[1] < y[1] ? -1 : 1;
    return 0;
}

/* EmbeddingBag sparse backward + Tensor.coalesce() (s_q_g_p_c.py:859): rows ascending,
 * duplicates summed in ascending lookup position (first value copied, then +=).
 * Returns U; rows[U], vals[U*D]. */
int64_t oracle_emb_bwd_coalesce(int64_t n, int D, const int64_t* idx, int64_t L, const int64_t* off,
                                int64_t B, const float* dy, float s, int ste, int32_t* rows,
                                float* vals, uint32_t* err) {
    int64_t* bag_of = (int64_t*)malloc(sizeof(int64_t) * (size_t)(L > 0 ? L : 1));
    for (int64_t p = 0; p < L; ++p) bag_of[p] = -1;
    for (int64_t b = 0; b < B; ++b) {
        int64_t s0, s1;
        bag_range(off, B, L, b, &s0, &s1, err);
        for (int64_t p = s0; p < s1; ++p) bag_of[p] = b;
    }
    int64_t* pairs = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(L > 0 ? L : 1));
    int64_t m = 0;
    for (int64_t p = 0; p < L; ++p) {
        if (bag_of[p] < 0) continue;
        if (idx[p] < 0 || idx[p] >= n) {
            if (err) *err |= ORACLE_ERR_INDEX;
            continue;
        }
        pairs[2 * m] = idx[p];
        pairs[2 * m + 1] = p;
        ++m;
    }
    qsort(pairs, (size_t)m, 2 * sizeof(int64_t), cmp_pair);
    int64_t U = 0;
    for (int64_t i = 0; i < m; ++i) {
        const int64_t row = pairs[2 * i], b = bag_of[pairs[2 * i + 1]];
        const int head = (i == 0) || pairs[2 * (i - 1)] != row;
        if (head) {
            rows[U] = (int32_t)row;
            ++U;
        }
        float* v = vals + (U - 1) * D;
        for (int d = 0; d < D; ++d) {
            float g = dy[b * D + d];
            if (ste) g = (g * s) / s;
            v[d] = head ? g : v[d] + g;
        }
    }
    free(pairs);
    free(bag_of);
    return U;
}

/* linear_quantize + clamp on a flat array with one scale (quant_utils.py:75-101,343) */
void oracle_quantize(const float* x, int64_t n, float s, int bits, float* q) {
    const float r = 1.0f / s;
    const float lo = -(float)(1 << (bits - 1)), hi = (float)((1 << (bits - 1)) - 1);
    for (int64_t i = 0; i < n; ++i) q[i] = fake_quant(x[i], r, lo, hi);
}

/* INT4 rows as the packed fast path stores them: nibble = q + 8, element 2j low nibble */
void oracle_pack_int4(const float* W, int64_t n, int D, float s, uint8_t* out) {
    const float r = 1.0f / s;
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < D / 2; ++j) {
            int q0 = (int)fake_quant(W[i * D + 2 * j], r, -8.0f, 7.0f) + 8;
            int q1 = (int)fake_quant(W[i * D + 2 * j + 1], r, -8.0f, 7.0f) + 8;
            out[i * (D / 2) + j] = (uint8_t)(q0 | (q1 << 4));
        }
}
