// qknit_post.hip — post-processing of the knitted distribution on the GPU (gfx950).
//
//   qk_threshold_count / qk_npd   reference-shaped result: the ACCURACY truncation of
//                                 QuasiDistr (third_party/qvm/qvm/quasi_distr.py:3,7-10) and
//                                 nearest_probability_distribution (quasi_distr.py:28-43,
//                                 applied at run.py:71), as select + radix sort + scan.
//   qk_hellinger                  sums for the Hellinger fidelity of the cut vs uncut result
//                                 (qiskit hellinger_fidelity, src/HwAwareCutter/Utilities.py:222-224).
//
// NPD closed form: with the kept entries sorted ascending v_0 <= ... <= v_{n-1} and exclusive
// prefix sums S_i, the reference loop drops exactly the prefix i < k where k is the first index
// with v_k + S_k / (n - k) >= 0 (once an entry is kept every later one is: v is ascending and
// beta/n stops changing); kept entries become v_i + S_k / (n - k).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdio>
#include <string>

#include "internal.h"

namespace {

int post_fail(qk_ctx* ctx, const char* msg) {
    if (ctx) ctx->err = msg;
    return QK_EARG;
}

#define QKP_HIP(ctx, call)                                       \
    do {                                                         \
        hipError_t e_ = (call);                                  \
        if (e_ != hipSuccess) {                                  \
            if (ctx) ctx->err = hipGetErrorString(e_);           \
            return QK_EHIP;                                      \
        }                                                        \
    } while (0)

struct AboveThreshold {
    const double* v;
    double acc;
    __host__ __device__ bool operator()(const int64_t& i) const { return fabs(v[i]) > acc; }
};

struct AbsGreater {
    const double* v;
    double acc;
    __host__ __device__ int64_t operator()(const int64_t& i) const { return fabs(v[i]) > acc ? 1 : 0; }
};

__global__ void gather_vals_kernel(int64_t n, const int64_t* __restrict__ keys, const double* __restrict__ src,
                                   double* __restrict__ dst) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[keys[i]];
}

// first[0] = min over i of (v_i + S_i/(n-i) >= 0 ? i : n)
__global__ void npd_first_kept_kernel(int64_t n, const double* __restrict__ v, const double* __restrict__ S,
                                      unsigned long long* __restrict__ first) {
    unsigned long long best = (unsigned long long)n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (v[i] + S[i] / (double)(n - i) >= 0.0 && (unsigned long long)i < best) best = (unsigned long long)i;
    }
    atomicMin(first, best);
}

__global__ void npd_emit_kernel(int64_t n, const double* __restrict__ v, const int64_t* __restrict__ keys,
                                const double* __restrict__ S, const unsigned long long* __restrict__ first,
                                int64_t* __restrict__ out_keys, double* __restrict__ out_vals) {
    const int64_t k = (int64_t)*first;
    if (k >= n) return;
    const double shift = S[k] / (double)(n - k);
    for (int64_t i = k + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        out_keys[i - k] = keys[i];
        out_vals[i - k] = v[i] + shift;
    }
}

__global__ void npd_count_kernel(int64_t count, const unsigned long long* __restrict__ first,
                                 int64_t* __restrict__ n_out) {
    *n_out = count - (int64_t)*first;
}

__global__ void hellinger_kernel(int64_t n, const double* __restrict__ p, const double* __restrict__ q,
                                 double* __restrict__ acc3) {
    double s = 0.0, sp = 0.0, sq = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double a = p[i] > 0.0 ? p[i] : 0.0, b = q[i] > 0.0 ? q[i] : 0.0;
        s += sqrt(a * b);
        sp += a;
        sq += b;
    }
    typedef hipcub::BlockReduce<double, 256> BR;
    __shared__ typename BR::TempStorage tmp;
    const double bs = BR(tmp).Sum(s);
    __syncthreads();
    const double bp = BR(tmp).Sum(sp);
    __syncthreads();
    const double bq = BR(tmp).Sum(sq);
    if (threadIdx.x == 0) {
        atomicAdd(acc3 + 0, bs);
        atomicAdd(acc3 + 1, bp);
        atomicAdd(acc3 + 2, bq);
    }
}

unsigned grid_for(int64_t total) {
    int64_t b = (total + 255) / 256;
    return (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int qk_threshold_count(qk_ctx* ctx, int64_t n, const double* vals, double acc, void* ws, int64_t ws_bytes,
                       int64_t* count_dev) {
    if (!ctx) return QK_EARG;
    if (n < 0 || !count_dev || (n > 0 && !vals)) return post_fail(ctx, "qk_threshold_count: bad argument");
    QKP_HIP(ctx, hipSetDevice(ctx->device));
    hipcub::CountingInputIterator<int64_t> it(0);
    hipcub::TransformInputIterator<int64_t, AbsGreater, hipcub::CountingInputIterator<int64_t>> flags(
        it, AbsGreater{vals, acc});
    size_t need = 0;
    QKP_HIP(ctx, hipcub::DeviceReduce::Sum(nullptr, need, flags, count_dev, n, ctx->stream));
    if (ws_bytes < (int64_t)need || (!ws && need)) {
        char buf[128];
        snprintf(buf, sizeof buf, "qk_threshold_count: workspace needs %zu bytes", need);
        ctx->err = buf;
        return QK_EARG;
    }
    QKP_HIP(ctx, hipcub::DeviceReduce::Sum(ws, need, flags, count_dev, n, ctx->stream));
    return QK_OK;
}

int qk_npd_workspace_bytes(int64_t n, int64_t count, int64_t* bytes) {
    if (!bytes || n < 0 || count < 0) return QK_EARG;
    hipcub::CountingInputIterator<int64_t> it(0);
    hipcub::TransformInputIterator<int64_t, AbsGreater, hipcub::CountingInputIterator<int64_t>> flags(
        it, AbsGreater{nullptr, 0.0});
    size_t s_cnt = 0, s_sel = 0, s_sort = 0, s_scan = 0;
    int64_t* dummy = nullptr;
    if (hipcub::DeviceReduce::Sum(nullptr, s_cnt, flags, dummy, n) != hipSuccess) return QK_EHIP;
    if (hipcub::DeviceSelect::If(nullptr, s_sel, it, dummy, dummy, n, AboveThreshold{nullptr, 0.0}) != hipSuccess)
        return QK_EHIP;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, s_sort, (double*)nullptr, (double*)nullptr, dummy, dummy,
                                           (int)(count > 0 ? count : 1)) != hipSuccess)
        return QK_EHIP;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, s_scan, (double*)nullptr, (double*)nullptr,
                                         (int)(count > 0 ? count : 1)) != hipSuccess)
        return QK_EHIP;
    size_t cub = s_cnt > s_sel ? s_cnt : s_sel;
    cub = cub > s_sort ? cub : s_sort;
    cub = cub > s_scan ? cub : s_scan;
    // + keys/vals (unsorted), keys/vals (sorted), prefix sums, selected count, first-kept index
    const size_t c = (size_t)(count > 0 ? count : 1);
    *bytes = (int64_t)(align256(cub) + 2 * align256(c * 8) + 2 * align256(c * 8) + align256(c * 8) + 256 + 256);
    return QK_OK;
}

// Truncate |v| <= acc, then project onto the simplex exactly as the reference's loop does.
// count must equal qk_threshold_count's result; out_keys/out_vals have room for count entries;
// *n_out_dev receives the number of entries written (device int64).
int qk_npd(qk_ctx* ctx, int64_t n, const double* vals, double acc, int64_t count, void* ws, int64_t ws_bytes,
           int64_t* out_keys, double* out_vals, int64_t* n_out_dev) {
    if (!ctx) return QK_EARG;
    if (n < 0 || count < 0 || count > n || !n_out_dev) return post_fail(ctx, "qk_npd: bad argument");
    if (count > 0x7fffffff) return post_fail(ctx, "qk_npd: more than 2^31 entries above threshold");
    int64_t need = 0;
    if (qk_npd_workspace_bytes(n, count, &need) != QK_OK) return post_fail(ctx, "qk_npd: workspace query failed");
    if (!ws || ws_bytes < need) return post_fail(ctx, "qk_npd: workspace too small");
    QKP_HIP(ctx, hipSetDevice(ctx->device));
    if (count == 0) {
        QKP_HIP(ctx, hipMemsetAsync(n_out_dev, 0, sizeof(int64_t), ctx->stream));
        return QK_OK;
    }
    char* base = (char*)ws;
    const size_t c = (size_t)count;
    hipcub::CountingInputIterator<int64_t> it(0);
    hipcub::TransformInputIterator<int64_t, AbsGreater, hipcub::CountingInputIterator<int64_t>> flags(
        it, AbsGreater{vals, acc});
    size_t s_cnt = 0, s_sel = 0, s_sort = 0, s_scan = 0;
    // size queries only (no launch): the same shapes qk_npd_workspace_bytes accounted for
    QKP_HIP(ctx, hipcub::DeviceReduce::Sum(nullptr, s_cnt, flags, n_out_dev, n));
    QKP_HIP(ctx, hipcub::DeviceSelect::If(nullptr, s_sel, it, out_keys, n_out_dev, n, AboveThreshold{vals, acc}));
    QKP_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, s_sort, (double*)nullptr, (double*)nullptr, out_keys,
                                                    out_keys, (int)c));
    QKP_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, s_scan, (double*)nullptr, (double*)nullptr, (int)c));
    size_t cub = s_cnt > s_sel ? s_cnt : s_sel;
    cub = cub > s_sort ? cub : s_sort;
    cub = cub > s_scan ? cub : s_scan;
    void* tmp = base;
    size_t off = align256(cub);
    int64_t* keys0 = (int64_t*)(base + off); off += align256(c * 8);
    double* vals0 = (double*)(base + off); off += align256(c * 8);
    int64_t* keys1 = (int64_t*)(base + off); off += align256(c * 8);
    double* vals1 = (double*)(base + off); off += align256(c * 8);
    double* S = (double*)(base + off); off += align256(c * 8);
    int64_t* nsel = (int64_t*)(base + off); off += 256;
    unsigned long long* first = (unsigned long long*)(base + off);

    size_t t = cub;
    QKP_HIP(ctx, hipcub::DeviceSelect::If(tmp, t, it, keys0, nsel, n, AboveThreshold{vals, acc}, ctx->stream));
    hipLaunchKernelGGL(gather_vals_kernel, dim3(grid_for(count)), dim3(256), 0, ctx->stream, count, keys0, vals,
                       vals0);
    t = cub;
    QKP_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, t, vals0, vals1, keys0, keys1, (int)c, 0, 64,
                                                    ctx->stream));
    t = cub;
    QKP_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, t, vals1, S, (int)c, ctx->stream));
    const unsigned long long init = (unsigned long long)count;
    QKP_HIP(ctx, hipMemcpyAsync(first, &init, sizeof init, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(npd_first_kept_kernel, dim3(grid_for(count)), dim3(256), 0, ctx->stream, count, vals1, S,
                       first);
    hipLaunchKernelGGL(npd_emit_kernel, dim3(grid_for(count)), dim3(256), 0, ctx->stream, count, vals1, keys1, S,
                       first, out_keys, out_vals);
    hipLaunchKernelGGL(npd_count_kernel, dim3(1), dim3(1), 0, ctx->stream, count, first, n_out_dev);
    QKP_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_hellinger(qk_ctx* ctx, int64_t n, const double* p, const double* q, double* acc3) {
    if (!ctx) return QK_EARG;
    if (n < 0 || !acc3 || (n > 0 && (!p || !q))) return post_fail(ctx, "qk_hellinger: bad argument");
    QKP_HIP(ctx, hipSetDevice(ctx->device));
    QKP_HIP(ctx, hipMemsetAsync(acc3, 0, 3 * sizeof(double), ctx->stream));
    if (n == 0) return QK_OK;
    hipLaunchKernelGGL(hellinger_kernel, dim3(grid_for(n)), dim3(256), 0, ctx->stream, n, p, q, acc3);
    QKP_HIP(ctx, hipGetLastError());
    return QK_OK;
}

}  // extern "C"
