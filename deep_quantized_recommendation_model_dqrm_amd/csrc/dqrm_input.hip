// dqrm_input.hip — Criteo input path of the QAT step, gfx950.
//
// Reference (YangZhou08/Deep_Quantized_Recommendation_Model_DQRM @ 2024-10-24):
//   data_loader_terabyte.py  CriteoBinDataset.__getitem__ :227-237  one batch = B records of
//                            40 int32 (label, 13 dense, 26 categorical) from a flat binary file
//                            (written by numpy_to_binary :243-280)
//   data_loader_terabyte.py  _transform_features :68-87
//                              x_cat % max_ind_range (if > 0)          :71-72
//                              X    = log(float(x_int) + 1)             :75
//                              lS_i = x_cat.long().t()  [26][B]         :76,87
//                              y    = float(label).view(-1, 1)          :77
//                              lS_o = arange(B) per table               :85
//   dlrm_data_pytorch.py     collate_wrapper_criteo_offset :328-345 (same outputs, Kaggle)
//
// One launch turns the raw record block (already in HBM) into exactly what the embedding
// kernels and the MLP consume: the 160-B records are read coalesced into LDS (row pitch
// 41 words: conflict-free column reads), then dense features, labels and the TRANSPOSED
// categorical columns are written out — the [T][B] lS_i is the Criteo-form batch that the
// QAT kernels read with DQRM_BATCH_POOLING_ONE (offsets never read), so no host-side
// transpose / cast / modulo pass remains. Pure byte work: HBM-bound, 160 B read and
// 13*4 + 4 + 26*8 (+ 26*8 with lS_o) B written per sample.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <math.h>

#include "../../include/dqrm.h"

extern "C" int dqrm_internal_set_error(int code, const char* msg);  // dqrm_kernels.hip (hidden)

namespace {

constexpr int REC = DQRM_CRITEO_RECORD_INTS;  // 40
constexpr int NDEN = DQRM_CRITEO_DENSE;       // 13
constexpr int NCAT = DQRM_CRITEO_SPARSE;      // 26
constexpr int SPB = 64;                       // samples per workgroup pass
constexpr int PITCH = REC + 1;                // LDS row pitch (odd: column reads hit distinct banks)
constexpr int TPB = 256;

int input_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return dqrm_internal_set_error(code, buf);
}

// torch.remainder on int32 (Python semantics: the result takes the divisor's sign)
__device__ __forceinline__ int32_t py_mod(int32_t x, int32_t m) {
    int32_t r = x % m;
    return (r != 0 && ((r < 0) != (m < 0))) ? r + m : r;
}

__global__ void __launch_bounds__(TPB) k_criteo_unpack(const int32_t* __restrict__ rec, int64_t B, int32_t mod,
                                                        float* __restrict__ X, int64_t* __restrict__ lS_i,
                                                        float* __restrict__ y, int64_t* __restrict__ lS_o) {
    __shared__ int32_t s[SPB * PITCH];
    for (int64_t b0 = (int64_t)blockIdx.x * SPB; b0 < B; b0 += (int64_t)gridDim.x * SPB) {
        const int nb = (int)(B - b0 < SPB ? B - b0 : SPB);
        const int32_t* __restrict__ src = rec + b0 * REC;
        __syncthreads();  // the previous pass is done with s[]
        for (int i = threadIdx.x; i < nb * REC; i += TPB) {  // contiguous, coalesced
            const int b = i / REC, f = i - b * REC;
            s[b * PITCH + f] = src[i];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nb * NDEN; i += TPB) {  // X [B][13], contiguous writes
            const int b = i / NDEN, j = i - b * NDEN;
            X[b0 * NDEN + i] = logf((float)s[b * PITCH + 1 + j] + 1.0f);
        }
        for (int i = threadIdx.x; i < nb; i += TPB) y[b0 + i] = (float)s[i * PITCH];
        for (int i = threadIdx.x; i < nb * NCAT; i += TPB) {  // lS_i [26][B]: lanes along b
            const int t = i / nb, b = i - t * nb;
            int32_t v = s[b * PITCH + 1 + NDEN + t];
            if (mod > 0) v = py_mod(v, mod);
            lS_i[(int64_t)t * B + b0 + b] = (int64_t)v;
            if (lS_o) lS_o[(int64_t)t * B + b0 + b] = b0 + b;
        }
    }
}

}  // namespace

extern "C" {

int dqrm_criteo_unpack(const int32_t* records, int64_t num_samples, int32_t max_ind_range, float* dense,
                       int64_t* lS_i, float* labels, int64_t* lS_o, void* stream) {
    if (num_samples < 0) return input_error(DQRM_E_INVALID, "dqrm_criteo_unpack: negative sample count");
    if (num_samples == 0) return DQRM_OK;
    if (!records || !dense || !lS_i || !labels)
        return input_error(DQRM_E_INVALID, "dqrm_criteo_unpack: null pointer");
    int64_t blocks = (num_samples + SPB - 1) / SPB;
    if (blocks > 8192) blocks = 8192;  // grid-stride beyond (~32 workgroups per CU)
    hipLaunchKernelGGL(k_criteo_unpack, dim3((unsigned)blocks), dim3(TPB), 0, (hipStream_t)stream, records,
                       num_samples, max_ind_range, dense, lS_i, labels, lS_o);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return input_error(DQRM_E_HIP, "HIP error: %s (%d)", hipGetErrorString(e), (int)e);
    return DQRM_OK;
}

}  // extern "C"
