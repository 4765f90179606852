// Latency floors of the coalesce's dependency chain on MI355X (diagnostic, not product code).
//   P0  empty kernel, 208 x 256 threads: per-XCD start skew + launch duration
//   P1  empty kernel, 208 x 512 threads, 156 KiB dynamic LDS
//   P2  idx load -> slot compaction (ballots) -> dy row loads -> stores (no sort): the two
//       dependent HBM round trips every wide slot needs, 208 x 256
//   P3  as P2 with 4 sub-slots per slot, 832 x 64
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/floor_probe.hip -o tools/probe/floor_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ unsigned long long g_st[4096];

__global__ void p_empty(int dummy) {
    if (threadIdx.x == 0) g_st[blockIdx.x] = wall_clock64();
}

__global__ void __launch_bounds__(512) p_empty_lds(int dummy) {
    extern __shared__ unsigned char lds[];
    if (threadIdx.x == 0) { g_st[blockIdx.x] = wall_clock64(); lds[0] = (unsigned char)dummy; }
}

// rows [r0, r1) of slot s (8 slots, 256-row blocks)
__device__ void slot_rows(int64_t n, int s, int S, int64_t& r0, int64_t& r1) {
    const int64_t nb = (n + 255) / 256;
    r0 = nb * s / S * 256;
    int64_t e = nb * (s + 1) / S * 256;
    r1 = e < n ? e : n;
}

template <int TPB, int S>
__global__ void __launch_bounds__(TPB) p_floor(const int64_t* __restrict__ idx, const int64_t* __restrict__ nrows,
                                              const float* __restrict__ dy, float* __restrict__ out, int B) {
    __shared__ uint32_t keys[2048];
    __shared__ int wcnt[TPB / 64 + 1];
    const int t = blockIdx.x / S, s = blockIdx.x % S;
    if (threadIdx.x == 0) g_st[blockIdx.x] = wall_clock64();
    if (nrows[t] < 100000) return;  // wide tables only: the floor of a ~B/S-key slot
    constexpr int PER = 2048 / TPB;
    int64_t r[PER];
    const int64_t* ti = idx + (int64_t)t * B;
#pragma unroll
    for (int j = 0; j < PER; ++j) r[j] = ti[j * TPB + threadIdx.x];
    int64_t r0, r1;
    slot_rows(nrows[t], s, S, r0, r1);
    const int lane = threadIdx.x % 64, w = threadIdx.x / 64;
    const uint64_t lt = (1ull << lane) - 1;
    int n = 0;
    // wave-local compaction: wave w owns chunk columns; counts then a tiny scan
    int c = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) c += (r[j] >= r0 && r[j] < r1);
    // wave total
    int tot = c;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane == 0) wcnt[w] = tot;
    __syncthreads();
    int base = 0;
    for (int q = 0; q < TPB / 64; ++q) { base += q < w ? wcnt[q] : 0; n += wcnt[q]; }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const bool in = r[j] >= r0 && r[j] < r1;
        const uint64_t m = __ballot(in);
        if (in) keys[base + __popcll(m & lt)] = (uint32_t)(j * TPB + threadIdx.x);
        base += __popcll(m);
    }
    __syncthreads();
    // dy rows: 16 lanes per row (float4 each)
    const int g = threadIdx.x / 16, l = threadIdx.x % 16;
    constexpr int NG = TPB / 16;
    float4 v[8];
    const int64_t ob = (int64_t)t * B;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int e = g + k * NG;
        if (e < n) v[k] = reinterpret_cast<const float4*>(dy + ((int64_t)t * B + keys[e]) * 64)[l];
    }
    for (int e = g + 8 * NG; e < n; e += NG)
        reinterpret_cast<float4*>(out + (ob + e) * 64)[l] = reinterpret_cast<const float4*>(dy + ((int64_t)t * B + keys[e]) * 64)[l];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int e = g + k * NG;
        if (e < n) reinterpret_cast<float4*>(out + (ob + s * 0 + e) * 64)[l] = v[k];
    }
}

int main() {
    const int T = 26, B = 2048, D = 64;
    const int64_t rows_ref[T] = {9980200, 26095, 17224, 7383, 20152, 3, 7112, 1435, 62, 9756762, 1332128, 314263, 10,
                                 2208, 11168, 122, 4, 971, 14, 9994101, 7267918, 9946670, 415284, 12422, 102, 36};
    std::vector<int64_t> rows(T), hidx((size_t)T * B);
    for (int t = 0; t < T; ++t) rows[t] = rows_ref[t] >= 1000000 ? rows_ref[t] * 16 : rows_ref[t];
    srand(7);
    for (int t = 0; t < T; ++t)
        for (int b = 0; b < B; ++b) hidx[(size_t)t * B + b] = (int64_t)(((uint64_t)rand() << 31 ^ rand()) % rows[t]);
    int64_t *didx, *drows;
    float *ddy, *dout;
    CK(hipMalloc(&didx, hidx.size() * 8));
    CK(hipMalloc(&drows, T * 8));
    CK(hipMalloc(&ddy, (size_t)T * B * D * 4));
    CK(hipMalloc(&dout, (size_t)T * B * D * 4 * 2));
    CK(hipMemcpy(didx, hidx.data(), hidx.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(drows, rows.data(), T * 8, hipMemcpyHostToDevice));
    CK(hipMemset(ddy, 0, (size_t)T * B * D * 4));
    CK(hipFuncSetAttribute((const void*)p_empty_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto skew = [&](int nwg, const char* name) {
        std::vector<unsigned long long> st(nwg);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_st), nwg * 8));
        unsigned long long mn = *std::min_element(st.begin(), st.end());
        double per[8] = {0};
        for (int i = 0; i < nwg; ++i) per[i % 8] = std::max(per[i % 8], (st[i] - mn) / 100.0);
        printf("%-34s start skew per XCD (max us):", name);
        for (int x = 0; x < 8; ++x) printf(" %4.1f", per[x]);
        printf("\n");
    };
    auto timeit = [&](const char* name, int nwg, auto launch) {
        for (int i = 0; i < 20; ++i) launch();
        CK(hipDeviceSynchronize());
        const int N = 200;
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %7.2f us/launch (back-to-back, %d launches)\n", name, ms * 1000 / N, N);
        launch();
        CK(hipDeviceSynchronize());
        skew(nwg, name);
    };
    timeit("P0 empty 208x256", 208, [&] { hipLaunchKernelGGL(p_empty, dim3(208), dim3(256), 0, 0, 0); });
    timeit("P1 empty 208x512 156KiB LDS", 208,
           [&] { hipLaunchKernelGGL(p_empty_lds, dim3(208), dim3(512), 156 * 1024, 0, 0); });
    timeit("P0b empty 832x64", 832, [&] { hipLaunchKernelGGL(p_empty, dim3(832), dim3(64), 0, 0, 0); });
    timeit("P2 floor 208x256 (8 slots)", 208,
           [&] { hipLaunchKernelGGL((p_floor<256, 8>), dim3(T * 8), dim3(256), 0, 0, didx, drows, ddy, dout, B); });
    timeit("P2b floor 208x512 (8 slots)", 208,
           [&] { hipLaunchKernelGGL((p_floor<512, 8>), dim3(T * 8), dim3(512), 0, 0, didx, drows, ddy, dout, B); });
    timeit("P3 floor 832x256 (32 slots)", 832,
           [&] { hipLaunchKernelGGL((p_floor<256, 32>), dim3(T * 32), dim3(256), 0, 0, didx, drows, ddy, dout, B); });
    // single launches separated by sync (the diag scripts' regime)
    {
        float tot = 0;
        for (int i = 0; i < 50; ++i) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL((p_floor<256, 8>), dim3(T * 8), dim3(256), 0, 0, didx, drows, ddy, dout, B);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        printf("P2 isolated launches: %.2f us (event-bracketed)\n", tot * 1000 / 50);
    }
    return 0;
}
