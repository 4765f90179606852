// Random 256-B row access latency over a large slab: default hipMalloc vs
// hipExtMallocWithFlags(hipDeviceMallocContiguous). 208 workgroups x 512 threads, each
// lane-group of 16 loads one random row (float4 per lane) per round; R dependent rounds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__global__ void probe(float4* W, int64_t rows, int rounds, uint64_t seed, float* sink, unsigned long long* t,
                      int mode, float* rm) {
    const int lane = threadIdx.x % 16;
    uint64_t x = seed ^ (blockIdx.x * 1315423911ull + (threadIdx.x / 16) * 2654435761ull);
    float acc = 0.f;
    unsigned long long t0 = wall_clock64();
    for (int r = 0; r < rounds; ++r) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        int64_t row = (int64_t)((x >> 16) % (uint64_t)rows);
        row = (row + (int64_t)acc) % rows;  // dependent on the previous round
        float4 v[8];
        int64_t rr[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // mode >= 10: 8 independent rows per lane group per round
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            rr[k] = k == 0 ? row : (int64_t)((x >> 16) % (uint64_t)rows);
            if (k == 0 || mode >= 10) v[k] = W[rr[k] * 16 + lane];
        }
        float a2 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) if (k == 0 || mode >= 10) a2 += v[k].x + v[k].y + v[k].z + v[k].w;
        acc = a2 * 0.0f;
        if (mode % 10 >= 1)
#pragma unroll
            for (int k = 0; k < 8; ++k) if (k == 0 || mode >= 10) W[rr[k] * 16 + lane] = make_float4(v[k].x + 1.f, v[k].y, v[k].z, v[k].w);
        if (mode % 10 >= 2 && lane == 0)
#pragma unroll
            for (int k = 0; k < 8; ++k) if (k == 0 || mode >= 10) rm[rr[k]] = v[k].x;
    }
    if (mode % 10 >= 1) __syncthreads();  // drains the stores (vmcnt(0)) like the slot kernels' barriers
    unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
    if (acc == 123.f) sink[0] = acc;
}

static float* g_rm = nullptr;
static double run(const float4* W, int64_t rows, int rounds, int mode = 0, int nwg = 208, int nthr = 512) {
    float* sink; unsigned long long* t;
    hipMalloc(&sink, 4); hipMalloc(&t, 8192 * 8);
    for (int it = 0; it < 2; ++it)
        hipLaunchKernelGGL(probe, dim3(nwg), dim3(nthr), 0, 0, (float4*)W, rows, rounds, 1234 + it, sink, t, mode, g_rm);
    hipDeviceSynchronize();
    static unsigned long long h[8192]; hipMemcpy(h, t, nwg * 8, hipMemcpyDeviceToHost);
    double mx = 0; for (int i = 0; i < nwg; ++i) if (h[i] > mx) mx = h[i];
    hipFree(sink); hipFree(t);
    return mx / 100.0 / rounds;  // wall clock 100 MHz -> us per round
}

int main(int argc, char** argv) {
    const size_t gb = argc > 1 ? atoll(argv[1]) : 198;
    const size_t bytes = gb << 30;
    const int64_t rows = bytes / 256;
    for (int mode = 0; mode < 1; ++mode) {
        void* p = nullptr;
        hipError_t e = mode == 0 ? hipMalloc(&p, bytes) : hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous);
        if (e != hipSuccess) { printf("mode %d alloc failed: %s\n", mode, hipGetErrorString(e)); continue; }
        hipMemset(p, 0, bytes);
        hipDeviceSynchronize();
        if (!g_rm) hipMalloc(&g_rm, (size_t)rows * 4);
        printf("%s %zu GB, 1 row/group: load %.2f us/round | +row store %.2f | +4B store %.2f\n",
               mode ? "contiguous" : "default   ", gb, run((const float4*)p, rows, 8), run((const float4*)p, rows, 8, 1),
               run((const float4*)p, rows, 8, 2));
        printf("spread: 832 WGs x 8 rows/group (213k rows): load %.2f us/round; 1664 WGs x 256 thr x 1 row (26k rows): %.2f\n",
               run((const float4*)p, rows, 8, 10, 832), run((const float4*)p, rows, 8, 0, 1664, 256));
        printf("%s %zu GB, 8 rows/group (53k rows in flight): load %.2f us/round | +row store %.2f | +4B store %.2f\n",
               mode ? "contiguous" : "default   ", gb, run((const float4*)p, rows, 8, 10), run((const float4*)p, rows, 8, 11),
               run((const float4*)p, rows, 8, 12));
        hipFree(p);
    }
    // small slab for reference
    void* q; hipMalloc(&q, (size_t)2 << 30); hipMemset(q, 0, (size_t)2 << 30); hipDeviceSynchronize();
    printf("default 2 GB: %.2f us/round (8 rounds)\n", run((const float4*)q, ((size_t)2 << 30) / 256, 8));
    return 0;
}
