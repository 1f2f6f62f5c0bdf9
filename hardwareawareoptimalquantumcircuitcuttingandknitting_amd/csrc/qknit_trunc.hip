// qknit_trunc.hip — the reference's per-operation ACCURACY truncation on dense quasi-distributions
// (gfx950). The reference keeps a QuasiDistr as a dict and drops every entry with |v| <= ACCURACY
// each time one is built (quasi_distr.py:7-10): after from_counts (:12-20), after every merge
// (:55-60, virtual_circuit.py:216-228) and after every +, -, * of a per-gate knit
// (virtual_gates.py:105-124,179-194,262-286). run_virtual_circuit(truncation="reference") replays
// that sequence on dense device vectors (a dict key absent = a zero entry); these kernels are its
// arithmetic, one rounding per reference operation:
//
//   qk_qd_from_rows  out[dst[r] * width + x] = trunc(rows[r * width + x])      (instance distributions)
//   qk_qd_merge      out[ka(i) ^ kb(j)] = trunc(a[i] * b[j]) where nonzero, others 0 (QuasiDistr.merge)
//   qk_qd_axpby      out[i] = trunc(alpha * a[i] + beta * b[i])                  (+, -, scalar *)
//
// trunc(v) = |v| > acc ? v : 0. axpby is evaluated as fma(alpha, a, beta * b): with (1, +-1) that is
// round(a +- b), with (s, 0) round(s * a) — bit for bit the reference's one operation each.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "internal.h"

namespace {

int qd_fail(qk_ctx* ctx, const char* msg) {
    if (ctx) ctx->err = msg;
    return QK_EARG;
}

int qd_hip(qk_ctx* ctx, hipError_t e, const char* what) {
    if (e == hipSuccess) return QK_OK;
    if (ctx) ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    return QK_EHIP;
}

__device__ __forceinline__ double trunc_acc(double v, double acc) { return fabs(v) > acc ? v : 0.0; }

__global__ __launch_bounds__(256) void qd_from_rows_kernel(int64_t n_rows, int64_t width, const double* __restrict__ rows,
                                                           const int64_t* __restrict__ dst, double acc,
                                                           double* __restrict__ out) {
    const int64_t total = n_rows * width;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t r = i / width, x = i - r * width;
        out[dst[r] * width + x] = trunc_acc(rows[i], acc);
    }
}

// one thread per (i, j) pair: i = a's entry, j = b's entry; identity keys when the key array is null
__global__ __launch_bounds__(256) void qd_merge_kernel(int64_t na, const double* __restrict__ a,
                                                       const int64_t* __restrict__ ka, int64_t nb,
                                                       const double* __restrict__ b, const int64_t* __restrict__ kb,
                                                       double acc, double* __restrict__ out) {
    const int64_t total = na * nb;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
        const int64_t i = t / nb, j = t - i * nb;
        // the dict holds only kept products: a zero product (an entry one side cannot reach, e.g. a
        // config outcome the other side measures) must not overwrite the pair that owns the key
        const double v = trunc_acc(a[i] * b[j], acc);
        if (v != 0.0) out[(ka ? ka[i] : i) ^ (kb ? kb[j] : j)] = v;
    }
}

__global__ __launch_bounds__(256) void qd_axpby_kernel(int64_t n, double alpha, const double* __restrict__ a, double beta,
                                                       const double* __restrict__ b, double acc,
                                                       double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = trunc_acc(fma(alpha, a[i], beta * b[i]), acc);
}

unsigned qd_grid(int64_t n, int cus) {
    const int64_t g = (n + 255) / 256, cap = (int64_t)cus * 16;
    return (unsigned)(g < 1 ? 1 : (g < cap ? g : cap));
}

}  // namespace

extern "C" {

int qk_qd_from_rows(qk_ctx* ctx, int64_t n_rows, int64_t width, const double* rows, const int64_t* dst, double acc,
                    double* out) {
    if (!ctx) return QK_EARG;
    if (n_rows < 0 || width < 1 || acc < 0) return qd_fail(ctx, "qk_qd_from_rows: n_rows >= 0, width >= 1, acc >= 0");
    if (n_rows == 0) return QK_OK;
    if (!rows || !dst || !out) return qd_fail(ctx, "qk_qd_from_rows: null buffer");
    int rc = qd_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    hipLaunchKernelGGL(qd_from_rows_kernel, dim3(qd_grid(n_rows * width, ctx->cus)), dim3(256), 0, ctx->stream, n_rows,
                       width, rows, dst, acc, out);
    return qd_hip(ctx, hipGetLastError(), "qd_from_rows_kernel");
}

int qk_qd_merge(qk_ctx* ctx, int64_t na, const double* a, const int64_t* ka, int64_t nb, const double* b,
                const int64_t* kb, double acc, int64_t n_out, double* out) {
    if (!ctx) return QK_EARG;
    if (na < 1 || nb < 1 || n_out < 1 || acc < 0) return qd_fail(ctx, "qk_qd_merge: na, nb, n_out >= 1, acc >= 0");
    if (!a || !b || !out) return qd_fail(ctx, "qk_qd_merge: null buffer");
    if ((!ka && na > n_out) || (!kb && nb > n_out)) return qd_fail(ctx, "qk_qd_merge: identity keys beyond n_out");
    int rc = qd_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    rc = qd_hip(ctx, hipMemsetAsync(out, 0, (size_t)n_out * sizeof(double), ctx->stream), "hipMemsetAsync");
    if (rc) return rc;
    hipLaunchKernelGGL(qd_merge_kernel, dim3(qd_grid(na * nb, ctx->cus)), dim3(256), 0, ctx->stream, na, a, ka, nb, b,
                       kb, acc, out);
    return qd_hip(ctx, hipGetLastError(), "qd_merge_kernel");
}

int qk_qd_axpby(qk_ctx* ctx, int64_t n, double alpha, const double* a, double beta, const double* b, double acc,
                double* out) {
    if (!ctx) return QK_EARG;
    if (n < 0 || acc < 0) return qd_fail(ctx, "qk_qd_axpby: n >= 0, acc >= 0");
    if (n == 0) return QK_OK;
    if (!a || !b || !out) return qd_fail(ctx, "qk_qd_axpby: null buffer");
    int rc = qd_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    hipLaunchKernelGGL(qd_axpby_kernel, dim3(qd_grid(n, ctx->cus)), dim3(256), 0, ctx->stream, n, alpha, a, beta, b, acc,
                       out);
    return qd_hip(ctx, hipGetLastError(), "qd_axpby_kernel");
}

}  // extern "C"
