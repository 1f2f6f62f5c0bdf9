// qknit_post.hip — post-processing of the knitted distribution on the GPU (gfx950).
//
//   qk_threshold_count / qk_npd   reference-shaped result: the ACCURACY truncation of
//                                 QuasiDistr (third_party/qvm/qvm/quasi_distr.py:3,7-10) and
//                                 nearest_probability_distribution (quasi_distr.py:28-43,
//                                 applied at run.py:71): count, select, radix sort and scan are
//                                 the hand-written primitives of qknit_prim.hip (prim.h).
//   qk_hellinger                  sums for the Hellinger fidelity of the cut vs uncut result
//                                 (qiskit hellinger_fidelity, src/HwAwareCutter/Utilities.py:222-224).
//
// NPD closed form: with the kept entries sorted ascending v_0 <= ... <= v_{n-1} and exclusive
// prefix sums S_i, the reference loop drops exactly the prefix i < k where k is the first index
// with v_k + S_k / (n - k) >= 0 (once an entry is kept every later one is: v is ascending and
// beta/n stops changing); kept entries become v_i + S_k / (n - k).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "internal.h"
#include "prim.h"

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

__global__ void hellinger_kernel(int64_t n, const double* __restrict__ p, const double* __restrict__ q,
                                 double* __restrict__ acc3) {
    double s = 0.0, sp = 0.0, sq = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double a = p[i] > 0.0 ? p[i] : 0.0, b = q[i] > 0.0 ? q[i] : 0.0;
        s += sqrt(a * b);
        sp += a;
        sq += b;
    }
    __shared__ double red[4];
    const double bs = qkp::block_sum256(s, red);
    const double bp = qkp::block_sum256(sp, red);
    const double bq = qkp::block_sum256(sq, red);
    if (threadIdx.x == 0) {
        atomicAdd(acc3 + 0, bs);
        atomicAdd(acc3 + 1, bp);
        atomicAdd(acc3 + 2, bq);
    }
}

// keys[i] += base for the min(count, capacity) selected entries
__global__ void add_base_kernel(const unsigned long long* __restrict__ count, int64_t capacity, int64_t base,
                                int64_t* __restrict__ keys) {
    const int64_t c = (int64_t)*count < capacity ? (int64_t)*count : capacity;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] += base;
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
    const size_t need = qkp::count_bytes();
    if (ws_bytes < (int64_t)need || !ws) {
        char buf[128];
        snprintf(buf, sizeof buf, "qk_threshold_count: workspace needs %zu bytes", need);
        ctx->err = buf;
        return QK_EARG;
    }
    QKP_HIP(ctx, hipSetDevice(ctx->device));
    QKP_HIP(ctx, qkp::count_abs_above(ctx->stream, ctx->cus, n, vals, acc, count_dev, ws, (size_t)ws_bytes));
    return QK_OK;
}

namespace {
int key_bits_below(int64_t n) {  // bits of the largest index < n
    int b = 0;
    while (b < 63 && (int64_t(1) << b) < n) ++b;
    return b;
}
}  // namespace

int qk_npd_workspace_bytes(int64_t n, int64_t count, int64_t* bytes) {
    if (!bytes || n < 0 || count < 0) return QK_EARG;
    const size_t c = (size_t)(count > 0 ? count : 1);
    // selected indices / values + the selected count, then the pair NPD's workspace
    const size_t npd = 2 * align256(8 * c) + 256 + npd_pairs_bytes((int64_t)c);
    const size_t cnt = qkp::count_bytes();
    *bytes = (int64_t)(npd > cnt ? npd : cnt);
    return QK_OK;
}

// Truncate |v| <= acc, then project onto the simplex exactly as the reference's loop does.
// count must equal qk_threshold_count's result; out_keys/out_vals have room for count entries;
// *n_out_dev receives the number of entries written (device int64). The kept (index, value) pairs are
// appended unordered, then sorted by index and stably by value (npd_pairs_bits): ties in value come
// out in index order, as the reference's sorted() over the dict does.
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
    size_t off = 0;
    int64_t* keys0 = (int64_t*)(base + off); off += align256(c * 8);
    double* vals0 = (double*)(base + off); off += align256(c * 8);
    unsigned long long* nsel = (unsigned long long*)(base + off); off += 256;
    QKP_HIP(ctx, hipMemsetAsync(nsel, 0, sizeof(unsigned long long), ctx->stream));
    QKP_HIP(ctx, qkp::select_abs_above(ctx->stream, ctx->cus, n, vals, acc, keys0, vals0, nsel, count));
    return npd_pairs_bits(ctx, count, keys0, vals0, key_bits_below(n), base + off, ws_bytes - (int64_t)off, out_keys,
                          out_vals, n_out_dev);
}

int qk_select_above(qk_ctx* ctx, int64_t n, const double* vals, double acc, int64_t key_base, int64_t capacity,
                    int64_t* keys, double* out_vals, int64_t* count_dev) {
    if (!ctx) return QK_EARG;
    if (n < 0 || capacity < 0 || !count_dev || (n > 0 && !vals) || (capacity > 0 && (!keys || !out_vals)))
        return post_fail(ctx, "qk_select_above: bad argument");
    QKP_HIP(ctx, hipSetDevice(ctx->device));
    QKP_HIP(ctx, hipMemsetAsync(count_dev, 0, sizeof(int64_t), ctx->stream));
    QKP_HIP(ctx, qkp::select_abs_above(ctx->stream, ctx->cus, n, vals, acc, keys, out_vals,
                                       (unsigned long long*)count_dev, capacity));
    if (key_base != 0 && capacity > 0)
        hipLaunchKernelGGL(add_base_kernel, dim3(grid_for(capacity)), dim3(256), 0, ctx->stream,
                           (const unsigned long long*)count_dev, capacity, key_base, keys);
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
