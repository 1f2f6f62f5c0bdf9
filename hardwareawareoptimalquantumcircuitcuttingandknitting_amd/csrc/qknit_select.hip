// qknit_select.hip — the reference-shaped (dict) result of a small-K two-fragment knit without the
// dense 2^N vector (gfx950).
//
//   qk_knit_select   out = {key: v} for every output v = sum_k A[k][i] B[k][j] with |v| > acc, key =
//                    pdep(i, maskA) | pdep(j, maskB): the knit of virtual_circuit.py:50-68 (merges
//                    qd:55-60, per-gate knits vg:105-124,179-194) followed by QuasiDistr's ACCURACY
//                    truncation (quasi_distr.py:7-10), fused. Each output is formed exactly as the
//                    dense write kernels do (v = fma(A[k][i], B[k][j], v) for k = 0..K-1 from 0), so
//                    the kept values are bit-identical to the dense path's.
//   qk_npd_pairs     nearest_probability_distribution (quasi_distr.py:28-43, run.py:71) on those
//                    pairs (qknit_post.hip holds the dense form).
//
// Tiles of 256 (i) x 256 (j) outputs. Before any arithmetic a tile is bounded on its per-k column
// maxima: |v| <= sum_k max_i |A[k][i]| max_j |B[k][j]| (per 256-column block, one pre-pass over the
// operands), and a tile whose bound (with a rounding margin) is <= acc holds no kept entry and is
// skipped whole: the 2^32 outputs of syc 32 5 (each ~2^-32) are never formed at ACCURACY = 1e-5.
// Kept entries are appended with one atomic per wave and kept-lane group (ballot + prefix popcount);
// qk_npd_pairs then sorts them by key and, stably, by value, so the result does not depend on the
// append order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "internal.h"
#include "prim.h"

namespace {

constexpr int SEL_K_MAX = 8;
constexpr int SEL_T = 256;  // tile edge (outputs along i and along j) = threads per workgroup
// A skipped tile's bound B satisfies B (1 + margin) <= acc: |computed v| <= (sum_k |a_k||b_k|)(1 + 2K u)
// and the bound itself is rounded by (1 + 2K u), u = 2^-53, K <= 8 -> margin 2^-47 would do.
constexpr double SEL_MARGIN = 1e-12;

int sel_fail(qk_ctx* ctx, const char* msg) {
    if (ctx) ctx->err = msg;
    return QK_EARG;
}

#define QKS_HIP(ctx, call)                             \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) {                        \
            if (ctx) ctx->err = hipGetErrorString(e_); \
            return QK_EHIP;                            \
        }                                              \
    } while (0)

__device__ __forceinline__ uint64_t pdep64(uint64_t x, uint64_t mask) {
    uint64_t r = 0;
    for (; mask; mask &= mask - 1, x >>= 1)
        if (x & 1) r |= mask & (~mask + 1);
    return r;
}

// colmax[blk][k] = max over the 256 columns of block blk of |X[k][col]| (0 past n); blocks of A first,
// then of B (one workgroup per block).
__global__ __launch_bounds__(SEL_T) void qk_select_colmax_kernel(int K, const double* __restrict__ A, int64_t lda,
                                                                 int64_t M, int64_t nblkA, const double* __restrict__ B,
                                                                 int64_t ldb, int64_t N, const int32_t* __restrict__ kdev,
                                                                 double* __restrict__ colmax) {
    if (kdev && *kdev <= 0) return;
    __shared__ double red[SEL_T / 64][SEL_K_MAX];
    const int64_t blk = blockIdx.x;
    const bool isA = blk < nblkA;
    const double* X = isA ? A : B;
    const int64_t ld = isA ? lda : ldb, n = isA ? M : N;
    const int64_t col = (isA ? blk : blk - nblkA) * SEL_T + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int k = 0; k < K; ++k) {
        double v = col < n ? fabs(X[k * ld + col]) : 0.0;
        for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
        if (lane == 0) red[wave][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < K) {
        double v = red[0][threadIdx.x];
        for (int w = 1; w < SEL_T / 64; ++w) v = fmax(v, red[w][threadIdx.x]);
        colmax[blk * SEL_K_MAX + threadIdx.x] = v;
    }
}

struct SelectArgs {
    int K;
    const double* __restrict__ A;
    int64_t lda, M, nblkA;
    const double* __restrict__ B;
    int64_t ldb, N, nblkB;
    uint64_t maskA, maskB;
    double acc;
    const double* __restrict__ colmax;  // [nblkA + nblkB][SEL_K_MAX]
    const int32_t* kdev;
    int64_t capacity;
    int64_t* __restrict__ keys;
    double* __restrict__ vals;
    unsigned long long* __restrict__ count;
};

__global__ __launch_bounds__(SEL_T) void qk_knit_select_kernel(SelectArgs a) {
    int K = a.K;
    if (a.kdev) {
        const int kd = *a.kdev;
        if (kd <= 0) return;
        K = kd < K ? kd : K;
    }
    __shared__ double sB[SEL_K_MAX][SEL_T];
    __shared__ uint64_t sKeyB[SEL_T];
    const int lane = threadIdx.x & 63;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    const int64_t tiles = a.nblkA * a.nblkB;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t bi = t % a.nblkA, bj = t / a.nblkA;
        double bound = 0.0;
        for (int k = 0; k < K; ++k)
            bound = fma(a.colmax[bi * SEL_K_MAX + k], a.colmax[(a.nblkA + bj) * SEL_K_MAX + k], bound);
        if (bound * (1.0 + SEL_MARGIN) <= a.acc) continue;  // uniform over the workgroup
        const int64_t i = bi * SEL_T + threadIdx.x;
        const int64_t j0 = bj * SEL_T;
        const int nj = (int)(a.N - j0 < SEL_T ? a.N - j0 : SEL_T);
        const bool live = i < a.M;
        double av[SEL_K_MAX];
#pragma unroll
        for (int k = 0; k < SEL_K_MAX; ++k) av[k] = (live && k < K) ? a.A[k * a.lda + i] : 0.0;
        const uint64_t keyA = live ? pdep64((uint64_t)i, a.maskA) : 0;
        __syncthreads();  // the previous tile's readers are done with the stage
        if (threadIdx.x < nj) {
            for (int k = 0; k < K; ++k) sB[k][threadIdx.x] = a.B[k * a.ldb + j0 + threadIdx.x];
            sKeyB[threadIdx.x] = pdep64((uint64_t)(j0 + threadIdx.x), a.maskB);
        }
        __syncthreads();
        for (int jj = 0; jj < nj; ++jj) {
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < SEL_K_MAX; ++k)
                if (k < K) v = fma(av[k], sB[k][jj], v);
            const bool keep = live && fabs(v) > a.acc;
            const uint64_t m = __ballot(keep);
            if (m) {  // wave-uniform
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(a.count, (unsigned long long)__popcll(m));
                base = __shfl(base, 0);
                if (keep) {
                    const int64_t idx = (int64_t)base + __popcll(m & below);
                    if (idx < a.capacity) {
                        a.keys[idx] = (int64_t)(keyA | sKeyB[jj]);
                        a.vals[idx] = v;
                    }
                }
            }
        }
    }
}

// ---- nearest_probability_distribution on (key, value) pairs (closed form: qknit_post.hip header)
__global__ void sel_first_kept_kernel(int64_t n, const double* __restrict__ v, const double* __restrict__ S,
                                      unsigned long long* __restrict__ first) {
    unsigned long long best = (unsigned long long)n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (v[i] + S[i] / (double)(n - i) >= 0.0 && (unsigned long long)i < best) best = (unsigned long long)i;
    atomicMin(first, best);
}

__global__ void sel_init_first_kernel(int64_t n, unsigned long long* __restrict__ first) {
    *first = (unsigned long long)n;
}

__global__ void sel_emit_kernel(int64_t n, const double* __restrict__ v, const int64_t* __restrict__ keys,
                                const double* __restrict__ S, const unsigned long long* __restrict__ first,
                                int64_t* __restrict__ out_keys, double* __restrict__ out_vals,
                                int64_t* __restrict__ n_out) {
    const int64_t k = (int64_t)*first;
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_out = n - k;
    if (k >= n) return;
    const double shift = S[k] / (double)(n - k);
    for (int64_t i = k + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        out_keys[i - k] = keys[i];
        out_vals[i - k] = v[i] + shift;
    }
}

unsigned sel_grid(int64_t total) {
    int64_t b = (total + 255) / 256;
    return (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

int64_t nblk(int64_t n) { return (n + SEL_T - 1) / SEL_T; }

}  // namespace

extern "C" {

int qk_knit_select_workspace_bytes(int nbits, uint64_t maskA, uint64_t maskB, int64_t* bytes) {
    if (!bytes || nbits < 1 || nbits > 62 || (maskA & maskB)) return QK_EARG;
    const int64_t M = int64_t(1) << __builtin_popcountll(maskA), N = int64_t(1) << __builtin_popcountll(maskB);
    *bytes = (nblk(M) + nblk(N)) * SEL_K_MAX * 8;
    return QK_OK;
}

int qk_knit_select(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B, int64_t ldb,
                   uint64_t maskA, uint64_t maskB, double acc, const int32_t* k_dev, void* work, int64_t work_bytes,
                   int64_t capacity, int64_t* keys, double* vals, int64_t* count_dev) {
    if (!ctx) return QK_EARG;
    if (nbits < 1 || nbits > 62 || K < 1 || K > SEL_K_MAX || !(acc >= 0.0))
        return sel_fail(ctx, "qk_knit_select: need 1 <= nbits <= 62, 1 <= K <= 8, acc >= 0");
    if ((maskA & maskB) || ((maskA | maskB) >> nbits))
        return sel_fail(ctx, "qk_knit_select: masks must be disjoint and inside the output bits");
    const int64_t M = int64_t(1) << __builtin_popcountll(maskA), N = int64_t(1) << __builtin_popcountll(maskB);
    if (!A || !B || !count_dev || (capacity > 0 && (!keys || !vals)) || capacity < 0)
        return sel_fail(ctx, "qk_knit_select: null buffer");
    if (lda < M || ldb < N) return sel_fail(ctx, "qk_knit_select: leading dimension too small");
    int64_t need = 0;
    qk_knit_select_workspace_bytes(nbits, maskA, maskB, &need);
    if (!work || work_bytes < need) return sel_fail(ctx, "qk_knit_select: workspace too small");
    QKS_HIP(ctx, hipSetDevice(ctx->device));
    QKS_HIP(ctx, hipMemsetAsync(count_dev, 0, sizeof(int64_t), ctx->stream));
    const int64_t na = nblk(M), nb = nblk(N);
    double* colmax = (double*)work;
    hipLaunchKernelGGL(qk_select_colmax_kernel, dim3((unsigned)(na + nb)), dim3(SEL_T), 0, ctx->stream, (int)K, A,
                       lda, M, na, B, ldb, N, k_dev, colmax);
    SelectArgs s{(int)K, A, lda, M, na, B, ldb, N, nb, maskA, maskB, acc, colmax, k_dev, capacity, keys, vals,
                 (unsigned long long*)count_dev};
    const int64_t tiles = na * nb, G0 = (int64_t)ctx->cus * 8;
    hipLaunchKernelGGL(qk_knit_select_kernel, dim3((unsigned)(tiles < G0 ? tiles : G0)), dim3(SEL_T), 0, ctx->stream,
                       s);
    QKS_HIP(ctx, hipGetLastError());
    return QK_OK;
}

}  // extern "C"

// nearest_probability_distribution of (key, value) pairs whose keys fit `key_bits` bits (internal.h:
// qk_npd_pairs and the dense qk_npd share it)
size_t npd_pairs_bytes(int64_t count) {
    const size_t c = (size_t)(count > 0 ? count : 1);
    const size_t prim = qkp::radix_sort_bytes((int64_t)c) > qkp::scan_bytes((int64_t)c) ? qkp::radix_sort_bytes((int64_t)c)
                                                                                      : qkp::scan_bytes((int64_t)c);
    // keys / vals sorted by key, then by value; prefix sums; first-kept index; the primitives' scratch
    return 5 * al256(8 * c) + 256 + al256(prim);
}

int npd_pairs_bits(qk_ctx* ctx, int64_t count, const int64_t* keys, const double* vals, int key_bits, void* ws,
                   int64_t ws_bytes, int64_t* out_keys, double* out_vals, int64_t* n_out_dev) {
    if (!ctx) return QK_EARG;
    if (count < 0 || count > 0x7fffffff || !n_out_dev || (count > 0 && (!keys || !vals || !out_keys || !out_vals)) ||
        key_bits < 0 || key_bits > 64)
        return sel_fail(ctx, "qk_npd_pairs: bad argument");
    if (!ws || ws_bytes < (int64_t)npd_pairs_bytes(count)) return sel_fail(ctx, "qk_npd_pairs: workspace too small");
    QKS_HIP(ctx, hipSetDevice(ctx->device));
    if (count == 0) {
        QKS_HIP(ctx, hipMemsetAsync(n_out_dev, 0, sizeof(int64_t), ctx->stream));
        return QK_OK;
    }
    const size_t c = (size_t)count;
    char* base = (char*)ws;
    size_t off = 0;
    int64_t* k1 = (int64_t*)(base + off); off += al256(8 * c);
    double* v1 = (double*)(base + off); off += al256(8 * c);
    int64_t* k2 = (int64_t*)(base + off); off += al256(8 * c);
    double* v2 = (double*)(base + off); off += al256(8 * c);
    double* S = (double*)(base + off); off += al256(8 * c);
    unsigned long long* first = (unsigned long long*)(base + off); off += 256;
    void* tmp = base + off;
    const size_t tmp_bytes = (size_t)ws_bytes - off;
    // by key, then stably by value: ties in value come out in key order whatever the append order was
    QKS_HIP(ctx, qkp::radix_sort_pairs(ctx->stream, count, (const uint64_t*)keys, (const uint64_t*)vals, (uint64_t*)k1,
                                       (uint64_t*)v1, 0, key_bits, qkp::KEY_U64, tmp, tmp_bytes));
    QKS_HIP(ctx, qkp::radix_sort_pairs(ctx->stream, count, (const uint64_t*)v1, (const uint64_t*)k1, (uint64_t*)v2,
                                       (uint64_t*)k2, 0, 64, qkp::KEY_F64, tmp, tmp_bytes));
    QKS_HIP(ctx, qkp::exclusive_sum(ctx->stream, count, v2, S, tmp, tmp_bytes));
    hipLaunchKernelGGL(sel_init_first_kernel, dim3(1), dim3(1), 0, ctx->stream, count, first);
    hipLaunchKernelGGL(sel_first_kept_kernel, dim3(sel_grid(count)), dim3(256), 0, ctx->stream, count, v2, S, first);
    hipLaunchKernelGGL(sel_emit_kernel, dim3(sel_grid(count)), dim3(256), 0, ctx->stream, count, v2, k2, S, first,
                       out_keys, out_vals, n_out_dev);
    QKS_HIP(ctx, hipGetLastError());
    return QK_OK;
}

extern "C" {

int qk_npd_pairs_workspace_bytes(int64_t count, int64_t* bytes) {
    if (!bytes || count < 0 || count > 0x7fffffff) return QK_EARG;
    *bytes = (int64_t)npd_pairs_bytes(count);
    return QK_OK;
}

int qk_npd_pairs(qk_ctx* ctx, int64_t count, const int64_t* keys, const double* vals, void* ws, int64_t ws_bytes,
                 int64_t* out_keys, double* out_vals, int64_t* n_out_dev) {
    // keys are any non-negative int64 (qk_knit_select: pdep of up to 62 output bits): all 64 bits sorted
    return npd_pairs_bits(ctx, count, keys, vals, 64, ws, ws_bytes, out_keys, out_vals, n_out_dev);
}

}  // extern "C"
