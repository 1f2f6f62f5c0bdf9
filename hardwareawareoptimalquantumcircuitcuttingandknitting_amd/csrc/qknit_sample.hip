// qknit_sample.hip — shot sampling of exact instance distributions (gfx950).
//
// The reference samples every instance circuit `shots` times on a simulator backend
// (third_party/qvm/qvm/run.py:42 `backend.run(instantiations, shots)`), turns the counts into
// frequencies keyed by (data bits, config bits) and drops those not above ACCURACY
// (quasi_distr.py:7-20 `from_counts`). Here the instance distributions are exact (qk_sweep);
// this file draws the samples from them on the GPU:
//   qk_sample_cdf     per instance, the inclusive prefix sums of P over all of its branch jobs
//                     (rows of pjob, |sign * P|) — one workgroup per instance;
//   qk_sample_counts  per reference label, `shots` draws (counter-based SplitMix64 stream keyed by
//                     seed, label, draw) located by binary search in its instance's CDF and counted
//                     per (branch job, outcome) with integer atomics (order-independent results);
//   qk_fold_counts    frequencies, the from_counts truncation at ACCURACY per (outcome, config
//                     bits), then the signed fold over the config bits (virtual_gates.py:105-124).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "internal.h"

namespace {

constexpr int ST = 256;  // threads per workgroup
constexpr int SPT = 8;   // consecutive values per thread per scan tile

int sfail(qk_ctx* ctx, const char* msg) {
    if (ctx) ctx->err = msg;
    return QK_EARG;
}

int slaunched(qk_ctx* ctx) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        ctx->err = hipGetErrorString(e);
        return QK_EHIP;
    }
    return QK_OK;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform double in [0, 1) for draw s of label l
__device__ __forceinline__ double draw(uint64_t seed, int64_t l, int64_t s) {
    const uint64_t z = splitmix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(l + 1) +
                                  0xD1B54A32D192ED03ull * (uint64_t)(s + 1));
    return (double)(z >> 11) * 0x1.0p-53;
}

__global__ __launch_bounds__(ST) void qk_cdf_kernel(const int64_t* __restrict__ seg_off, int64_t W,
                                                    const double* __restrict__ pjob, double* __restrict__ cdf) {
    __shared__ double part[ST];
    __shared__ double carry_s;
    const int tid = threadIdx.x;
    const int64_t begin = seg_off[blockIdx.x] * W, end = seg_off[blockIdx.x + 1] * W;
    if (tid == 0) carry_s = 0.0;
    __syncthreads();
    for (int64_t base = begin; base < end; base += (int64_t)ST * SPT) {
        double v[SPT];
        double run = 0.0;
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int64_t i = base + (int64_t)tid * SPT + k;
            run += i < end ? fabs(pjob[i]) : 0.0;
            v[k] = run;
        }
        part[tid] = run;
        __syncthreads();
        for (int off = 1; off < ST; off <<= 1) {  // inclusive scan of the thread totals
            const double add = tid >= off ? part[tid - off] : 0.0;
            __syncthreads();
            part[tid] += add;
            __syncthreads();
        }
        const double excl = carry_s + (tid ? part[tid - 1] : 0.0);
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int64_t i = base + (int64_t)tid * SPT + k;
            if (i < end) cdf[i] = excl + v[k];
        }
        __syncthreads();
        if (tid == ST - 1) carry_s += part[ST - 1];
        __syncthreads();
    }
}

__global__ __launch_bounds__(ST) void qk_sample_kernel(int64_t label_base, const int64_t* __restrict__ label_seg,
                                                       const int64_t* __restrict__ seg_off,
                                                       const int64_t* __restrict__ label_row_off, int64_t W,
                                                       const double* __restrict__ cdf, int64_t shots, uint64_t seed,
                                                       unsigned int* __restrict__ counts) {
    const int64_t l = blockIdx.x;
    const int64_t seg = label_seg[l];
    const int64_t begin = seg_off[seg] * W, n = (seg_off[seg + 1] - seg_off[seg]) * W;
    const double* c = cdf + begin;
    const double total = c[n - 1];
    unsigned int* out = counts + label_row_off[l] * W;
    for (int64_t s = threadIdx.x; s < shots; s += ST) {
        const double target = draw(seed, label_base + l, s) * total;
        int64_t lo = 0, hi = n - 1;  // first index with cdf > target
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (c[mid] > target) hi = mid;
            else lo = mid + 1;
        }
        atomicAdd(out + lo, 1u);
    }
}

__global__ void qk_fold_counts_kernel(int64_t n_labels, const int64_t* __restrict__ label_row_off, int64_t W,
                                      const double* __restrict__ row_sign, const unsigned int* __restrict__ counts,
                                      double inv_shots, double acc, double* __restrict__ q) {
    const int64_t total = n_labels * W;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t l = e / W, x = e - l * W;
        double s = 0.0;
        for (int64_t r = label_row_off[l]; r < label_row_off[l + 1]; ++r) {
            const double f = counts[r * W + x] * inv_shots;
            if (f > acc) s += row_sign[r] * f;
        }
        q[e] = s;
    }
}

}  // namespace

extern "C" {

int qk_sample_cdf(qk_ctx* ctx, int64_t n_seg, const int64_t* seg_off, int64_t width, const double* pjob,
                  double* cdf) {
    if (!ctx) return QK_EARG;
    if (n_seg < 0 || width <= 0) return sfail(ctx, "qk_sample_cdf: bad sizes");
    if (n_seg == 0) return QK_OK;
    if (!seg_off || !pjob || !cdf) return sfail(ctx, "qk_sample_cdf: null buffer");
    if (n_seg > 0x7fffffff) return sfail(ctx, "qk_sample_cdf: too many instances");
    if (hipSetDevice(ctx->device) != hipSuccess) return QK_EHIP;
    hipLaunchKernelGGL(qk_cdf_kernel, dim3((unsigned)n_seg), dim3(ST), 0, ctx->stream, seg_off, width, pjob, cdf);
    return slaunched(ctx);
}

int qk_sample_counts(qk_ctx* ctx, int64_t n_labels, int64_t label_base, const int64_t* label_seg,
                     const int64_t* seg_off, const int64_t* label_row_off, int64_t width, const double* cdf,
                     int64_t shots, uint64_t seed, unsigned int* counts) {
    if (!ctx) return QK_EARG;
    if (n_labels < 0 || label_base < 0 || width <= 0 || shots < 0) return sfail(ctx, "qk_sample_counts: bad sizes");
    if (n_labels == 0 || shots == 0) return QK_OK;
    if (!label_seg || !seg_off || !label_row_off || !cdf || !counts)
        return sfail(ctx, "qk_sample_counts: null buffer");
    if (n_labels > 0x7fffffff || shots > 0xffffffffll)
        return sfail(ctx, "qk_sample_counts: too many labels or shots");
    if (hipSetDevice(ctx->device) != hipSuccess) return QK_EHIP;
    hipLaunchKernelGGL(qk_sample_kernel, dim3((unsigned)n_labels), dim3(ST), 0, ctx->stream, label_base, label_seg,
                       seg_off,
                       label_row_off, width, cdf, shots, seed, counts);
    return slaunched(ctx);
}

int qk_fold_counts(qk_ctx* ctx, int64_t n_labels, const int64_t* label_row_off, int64_t width,
                   const double* row_sign, const unsigned int* counts, int64_t shots, double acc, double* q) {
    if (!ctx) return QK_EARG;
    if (n_labels < 0 || width <= 0 || shots <= 0) return sfail(ctx, "qk_fold_counts: bad sizes");
    if (n_labels == 0) return QK_OK;
    if (!label_row_off || !row_sign || !counts || !q) return sfail(ctx, "qk_fold_counts: null buffer");
    if (hipSetDevice(ctx->device) != hipSuccess) return QK_EHIP;
    int64_t blocks = (n_labels * width + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(qk_fold_counts_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, n_labels,
                       label_row_off, width, row_sign, counts, 1.0 / (double)shots, acc, q);
    return slaunched(ctx);
}

}  // extern "C"
