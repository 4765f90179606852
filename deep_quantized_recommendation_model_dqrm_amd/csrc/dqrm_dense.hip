// dqrm_dense.hip — dense (MLP) layer gradient path of DQRM's data-parallel step, gfx950.
//
// Reference (YangZhou08/Deep_Quantized_Recommendation_Model_DQRM @ 2024-10-24,
// sgd_quantized_gradients_parallel_comm.py):
//   quantize_linear_grad  :892-929  per-channel (weight row) abs-max scale, all_reduce/N,
//                                   SymmetricQuantFunction, all_reduce/N
//   quantize_bias_grad    :931-961  the same with one scale per bias vector
//   grad_update_parallel_comm   MLP branch :337-409  grad.zero_(); grad.add_(buffer)
//   weight_update_parallel_comm MLP branch :630-668  W += (-lr * grad) * s
//
// Design: every weight row and every bias vector of all bot_l/top_l layers is one
// "channel"; the four phases are ONE launch each for all layers (multi-tensor style: the
// channel table holds the raw grad/param pointers, nothing is copied into a bucket except
// the wire). One wavefront per channel (rows are 13..512 floats in DLRM MLPs), lanes
// striding the row so every load/store instruction of a wave covers 256 contiguous bytes.
// Elementwise and tiny (Kaggle MLP: 0.47 M params): launch/latency-bound, HBM otherwise.
//
// The quantized all-reduce itself is RCCL's (torch.distributed, "nccl" on ROCm): the wire
// holds integer-valued fp16 (exact: |q| <= 128, N <= 16 ranks -> every partial sum is an
// integer of magnitude <= 2048, representable in fp16), so the sum is exact in any
// reduction order and the wire is half the FP32 gradient. int32 otherwise.
// Compiled with -ffp-contract=off: the reference's `1/s*g + 0`, `(-lr*g)*s`, `W + u` are
// separately rounded operations.

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <math.h>

#include "../../include/dqrm.h"

extern "C" int dqrm_internal_set_error(int code, const char* msg);  // dqrm_kernels.hip (hidden)

namespace {

constexpr int WAVE = 64;
constexpr int DWG = 256;                 // threads per workgroup
constexpr int CPW = DWG / WAVE;          // channels per workgroup (one per wave)

int dense_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return dqrm_internal_set_error(code, buf);
}

#define DHIP_TRY(expr)                                                                       \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return dense_error(DQRM_E_HIP, "HIP error: %s (%d)", hipGetErrorString(e_), (int)e_); \
    } while (0)

struct DenseArgs {
    int C;
    float* const* grad;
    float* const* param;
    const int32_t* len;
    const int64_t* wire_off;
};

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
    return v;
}

// torch.round (half to even) == rintf; clamp to [lo, hi]
__device__ __forceinline__ float quant1(float g, float rcp, float lo, float hi) {
    const float q = rintf(rcp * g + 0.0f);
    return fminf(fmaxf(q, lo), hi);
}

template <int WT> struct Wire;
template <> struct Wire<DQRM_WIRE_F16> {
    using T = __half;
    static __device__ __forceinline__ T enc(float q) { return __float2half_rn(q); }
    static __device__ __forceinline__ float dec(T v) { return __half2float(v); }
};
template <> struct Wire<DQRM_WIRE_I32> {
    using T = int32_t;
    static __device__ __forceinline__ T enc(float q) { return (int32_t)q; }
    static __device__ __forceinline__ float dec(T v) { return (float)v; }
};
template <> struct Wire<DQRM_WIRE_F32> {
    using T = float;
    static __device__ __forceinline__ T enc(float q) { return q; }
    static __device__ __forceinline__ float dec(T v) { return v; }
};

// s_loc[c] = clamp(max_j |g_j|, 1e-8) / qmax   (max(|min|, |max|) == max |g| for finite g)
__global__ void __launch_bounds__(DWG) k_dense_scale(DenseArgs a, float qmax, float* __restrict__ s_loc) {
    const int c = blockIdx.x * CPW + threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
    if (c >= a.C) return;
    const float* __restrict__ g = a.grad[c];
    const int n = a.len[c];
    float m0 = 0.0f, m1 = 0.0f;
    int j = lane;
    for (; j + WAVE < n; j += 2 * WAVE) {  // two loads in flight per lane
        m0 = fmaxf(m0, fabsf(g[j]));
        m1 = fmaxf(m1, fabsf(g[j + WAVE]));
    }
    if (j < n) m0 = fmaxf(m0, fabsf(g[j]));
    const float m = wave_max(fmaxf(m0, m1));
    if (lane == 0) s_loc[c] = fmaxf(m, 1e-8f) / qmax;
}

// scale average in descending rank order (Gloo's one-element all_reduce; every rank
// computes the same bits), then quantize the channel into the wire
template <int WT>
__global__ void __launch_bounds__(DWG) k_dense_quant(DenseArgs a, const float* __restrict__ s_all, int N,
                                                      float inv_n, float lo, float hi, float* __restrict__ s_avg,
                                                      typename Wire<WT>::T* __restrict__ wire) {
    const int c = blockIdx.x * CPW + threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
    if (c >= a.C) return;
    const float* __restrict__ g = a.grad[c];
    const int n = a.len[c];
    typename Wire<WT>::T* __restrict__ w = wire + a.wire_off[c];
    if (WT == DQRM_WIRE_F32) {
        for (int j = lane; j < n; j += WAVE) w[j] = Wire<WT>::enc(g[j]);
        return;
    }
    float s = s_all[(int64_t)(N - 1) * a.C + c];
    for (int r = N - 2; r >= 0; --r) s = s + s_all[(int64_t)r * a.C + c];
    s = s * inv_n;
    if (lane == 0) s_avg[c] = s;
    const float rcp = 1.0f / s;
    for (int j = lane; j < n; j += WAVE) w[j] = Wire<WT>::enc(quant1(g[j], rcp, lo, hi));
}

// grad = 0 + sum * (1/N)  (quantized) / sum * (1/N)  (FP32)
template <int WT>
__global__ void __launch_bounds__(DWG) k_dense_decode(DenseArgs a, const typename Wire<WT>::T* __restrict__ wire,
                                                       float inv_n) {
    const int c = blockIdx.x * CPW + threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
    if (c >= a.C) return;
    float* __restrict__ g = a.grad[c];
    const int n = a.len[c];
    const typename Wire<WT>::T* __restrict__ w = wire + a.wire_off[c];
    if (WT == DQRM_WIRE_F32)  // all_reduce(grad); grad.mul_(1/N)   (:366-369)
        for (int j = lane; j < n; j += WAVE) g[j] = Wire<WT>::dec(w[j]) * inv_n;
    else                      // grad.zero_(); grad.add_(q_sum * (1/N))
        for (int j = lane; j < n; j += WAVE) g[j] = 0.0f + Wire<WT>::dec(w[j]) * inv_n;
}

// param += (-lr * grad) * s   (s == nullptr: param += -lr * grad)
__global__ void __launch_bounds__(DWG) k_dense_update(DenseArgs a, const float* __restrict__ s, float nlr) {
    const int c = blockIdx.x * CPW + threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
    if (c >= a.C) return;
    const float* __restrict__ g = a.grad[c];
    float* __restrict__ p = a.param[c];
    const int n = a.len[c];
    if (s != nullptr) {
        const float sc = s[c];
        for (int j = lane; j < n; j += WAVE) p[j] = p[j] + (nlr * g[j]) * sc;
    } else {
        for (int j = lane; j < n; j += WAVE) p[j] = p[j] + nlr * g[j];
    }
}

int check_dense(const dqrm_dense_set* s) {
    if (!s) return dense_error(DQRM_E_INVALID, "dqrm_dense: null dense set");
    if (s->num_channels < 0 || s->total_elems < 0)
        return dense_error(DQRM_E_INVALID, "dqrm_dense: negative channel/element count");
    if (s->num_channels > 0 && (!s->grad || !s->param || !s->len || !s->wire_off))
        return dense_error(DQRM_E_INVALID, "dqrm_dense: null channel table");
    return DQRM_OK;
}

int check_bits(int bits) {
    if (bits != 32 && (bits < 2 || bits > 16))
        return dense_error(DQRM_E_INVALID, "dqrm_dense: bits must be 2..16 or 32 (got %d)", bits);
    return DQRM_OK;
}

DenseArgs args_of(const dqrm_dense_set* s) {
    return DenseArgs{s->num_channels, s->grad, s->param, s->len, s->wire_off};
}

dim3 grid_of(const dqrm_dense_set* s) { return dim3((unsigned)((s->num_channels + CPW - 1) / CPW)); }

}  // namespace

extern "C" {

int dqrm_dense_wire_type(int bits, int num_ranks) {
    if (num_ranks < 1) return DQRM_E_INVALID;
    if (bits == 32) return DQRM_WIRE_F32;
    if (bits < 2 || bits > 16) return DQRM_E_INVALID;
    // |q| <= 2^(bits-1): all partial sums over N ranks exact in fp16 iff N * 2^(bits-1) <= 2048
    if ((int64_t)num_ranks << (bits - 1) <= 2048) return DQRM_WIRE_F16;
    return DQRM_WIRE_I32;
}

int dqrm_dense_grad_scale(const dqrm_dense_set* set, int bits, float* s_loc, void* stream) {
    int rc = check_dense(set);
    if (rc) return rc;
    if ((rc = check_bits(bits))) return rc;
    if (bits == 32) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_scale: no scale for unquantized gradients");
    if (set->num_channels == 0) return DQRM_OK;
    if (!s_loc) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_scale: null s_loc");
    const float qmax = (float)((1 << (bits - 1)) - 1);
    hipLaunchKernelGGL(k_dense_scale, grid_of(set), dim3(DWG), 0, (hipStream_t)stream, args_of(set), qmax, s_loc);
    DHIP_TRY(hipGetLastError());
    return DQRM_OK;
}

int dqrm_dense_grad_quant(const dqrm_dense_set* set, int bits, const float* s_all, int num_ranks, float* s_avg,
                          int wire_type, void* wire, void* stream) {
    int rc = check_dense(set);
    if (rc) return rc;
    if ((rc = check_bits(bits))) return rc;
    if (num_ranks < 1) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: num_ranks < 1");
    if (set->num_channels == 0) return DQRM_OK;
    if (!wire) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: null wire");
    if ((bits == 32) != (wire_type == DQRM_WIRE_F32))
        return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: wire type %d does not match bits %d", wire_type, bits);
    if (bits != 32) {
        if (!s_all || !s_avg) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: null scale buffers");
        const int need = dqrm_dense_wire_type(bits, num_ranks);
        if (wire_type == DQRM_WIRE_F16 && need != DQRM_WIRE_F16)
            return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: fp16 wire inexact for bits %d, %d ranks",
                               bits, num_ranks);
    }
    const float inv_n = 1.0f / (float)num_ranks;
    const int n = bits == 32 ? 0 : (1 << (bits - 1)) - 1;
    const float lo = (float)(-n - 1), hi = (float)n;
    hipStream_t st = (hipStream_t)stream;
    switch (wire_type) {
        case DQRM_WIRE_F16:
            hipLaunchKernelGGL(k_dense_quant<DQRM_WIRE_F16>, grid_of(set), dim3(DWG), 0, st, args_of(set), s_all,
                               num_ranks, inv_n, lo, hi, s_avg, (__half*)wire);
            break;
        case DQRM_WIRE_I32:
            hipLaunchKernelGGL(k_dense_quant<DQRM_WIRE_I32>, grid_of(set), dim3(DWG), 0, st, args_of(set), s_all,
                               num_ranks, inv_n, lo, hi, s_avg, (int32_t*)wire);
            break;
        case DQRM_WIRE_F32:
            hipLaunchKernelGGL(k_dense_quant<DQRM_WIRE_F32>, grid_of(set), dim3(DWG), 0, st, args_of(set), s_all,
                               num_ranks, inv_n, lo, hi, s_avg, (float*)wire);
            break;
        default:
            return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_quant: unknown wire type %d", wire_type);
    }
    DHIP_TRY(hipGetLastError());
    return DQRM_OK;
}

int dqrm_dense_grad_decode(const dqrm_dense_set* set, const void* wire, int wire_type, int num_ranks, void* stream) {
    int rc = check_dense(set);
    if (rc) return rc;
    if (num_ranks < 1) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_decode: num_ranks < 1");
    if (set->num_channels == 0) return DQRM_OK;
    if (!wire) return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_decode: null wire");
    const float inv_n = 1.0f / (float)num_ranks;
    hipStream_t st = (hipStream_t)stream;
    switch (wire_type) {
        case DQRM_WIRE_F16:
            hipLaunchKernelGGL(k_dense_decode<DQRM_WIRE_F16>, grid_of(set), dim3(DWG), 0, st, args_of(set),
                               (const __half*)wire, inv_n);
            break;
        case DQRM_WIRE_I32:
            hipLaunchKernelGGL(k_dense_decode<DQRM_WIRE_I32>, grid_of(set), dim3(DWG), 0, st, args_of(set),
                               (const int32_t*)wire, inv_n);
            break;
        case DQRM_WIRE_F32:
            hipLaunchKernelGGL(k_dense_decode<DQRM_WIRE_F32>, grid_of(set), dim3(DWG), 0, st, args_of(set),
                               (const float*)wire, inv_n);
            break;
        default:
            return dense_error(DQRM_E_INVALID, "dqrm_dense_grad_decode: unknown wire type %d", wire_type);
    }
    DHIP_TRY(hipGetLastError());
    return DQRM_OK;
}

int dqrm_dense_update(const dqrm_dense_set* set, const float* s, float lr, void* stream) {
    int rc = check_dense(set);
    if (rc) return rc;
    if (set->num_channels == 0) return DQRM_OK;
    hipLaunchKernelGGL(k_dense_update, grid_of(set), dim3(DWG), 0, (hipStream_t)stream, args_of(set), s, -lr);
    DHIP_TRY(hipGetLastError());
    return DQRM_OK;
}

}  // extern "C"
