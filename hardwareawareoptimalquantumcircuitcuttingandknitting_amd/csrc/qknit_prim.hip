// qknit_prim.hip — device-wide primitives for the reference-shaped result (gfx950, hand-written;
// interface and rationale in prim.h): count / unordered select of |v| > acc, deterministic exclusive
// prefix sums, and a stable LSD radix sort of 64-bit (key, value) pairs.
//
// Radix sort layout. The input is cut into W contiguous chunks, one per single-wave workgroup (a
// multiple of 64 elements each). Per 8-bit digit pass:
//   rs_hist     each wave counts its chunk's digits in LDS: the lanes holding one digit are found
//               with one ballot per digit bit (peers = AND of matching ballots) and the lowest of them
//               adds the group's size — no LDS atomics, no workgroup barrier;
//   scan        exclusive prefix of the digit-major (digit, wave) counts: where wave w's elements of
//               digit d start in the output;
//   rs_scatter  each wave walks its chunk in order again; an element's position is its digit's running
//               offset (LDS) plus its rank among the peer lanes below it, and the group's lowest lane
//               advances the offset — stable, since chunks, waves and lanes are visited in input order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "prim.h"

namespace qkp {
namespace {

constexpr int RS_ELEMS_PER_WAVE = 8192;  // at least (fewer waves for small inputs)
constexpr int64_t RS_MAX_WAVES = 4096;
constexpr int SC_T = 256, SC_I = 8, SC_TILE = SC_T * SC_I;
constexpr int64_t SC_MAX_BLOCKS = 1024;

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

__device__ __forceinline__ uint64_t rs_image(uint64_t k, int order) {
    if (order == KEY_F64) return (k >> 63) ? ~k : (k | (uint64_t(1) << 63));
    return k;
}

// lanes of this wave whose digit equals mine, among the `active` ones
__device__ __forceinline__ uint64_t rs_peers(uint32_t d, int nb, uint64_t active) {
    uint64_t m = active;
    for (int b = 0; b < nb; ++b) {
        const bool bit = (d >> b) & 1;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(64) void rs_hist_kernel(int64_t n, int64_t chunk, int64_t W, const uint64_t* __restrict__ keys,
                                                     int shift, int nb, int order, uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[256];
    const int lane = threadIdx.x;
    const int64_t w = blockIdx.x;
    for (int d = lane; d < 256; d += 64) cnt[d] = 0;
    __syncthreads();
    const int64_t b0 = w * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
    const uint32_t dmask = (1u << nb) - 1;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    for (int64_t base = b0; base < b1; base += 64) {
        const int64_t i = base + lane;
        const bool act = i < b1;
        const uint32_t d = act ? (uint32_t)(rs_image(keys[i], order) >> shift) & dmask : 0u;
        const uint64_t m = rs_peers(d, nb, __ballot(act));
        if (act && (m & below) == 0) cnt[d] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    for (int d = lane; d < 256; d += 64) hist[(int64_t)d * W + w] = cnt[d];
}

__global__ __launch_bounds__(64) void rs_scatter_kernel(int64_t n, int64_t chunk, int64_t W,
                                                        const uint64_t* __restrict__ kin, const uint64_t* __restrict__ vin,
                                                        uint64_t* __restrict__ kout, uint64_t* __restrict__ vout, int shift,
                                                        int nb, int order, const uint32_t* __restrict__ offs) {
    __shared__ uint32_t run[256];
    const int lane = threadIdx.x;
    const int64_t w = blockIdx.x;
    for (int d = lane; d < 256; d += 64) run[d] = offs[(int64_t)d * W + w];
    __syncthreads();
    const int64_t b0 = w * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
    const uint32_t dmask = (1u << nb) - 1;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    for (int64_t base = b0; base < b1; base += 64) {
        const int64_t i = base + lane;
        const bool act = i < b1;
        const uint64_t key = act ? kin[i] : 0, val = act ? vin[i] : 0;
        const uint32_t d = act ? (uint32_t)(rs_image(key, order) >> shift) & dmask : 0u;
        const uint64_t m = rs_peers(d, nb, __ballot(act));
        const uint32_t rank = (uint32_t)__popcll(m & below);
        uint32_t pos = 0;
        if (act) pos = run[d] + rank;
        // the group's lowest lane (rank 0, pos = the running offset) advances it; every lane of the
        // wave has read run[] above (one wave: its LDS operations complete in program order)
        if (act && rank == 0) run[d] = pos + (uint32_t)__popcll(m);
        if (act) {
            kout[pos] = key;
            vout[pos] = val;
        }
    }
}

// ---------------------------------------------------------------- exclusive scan (T = uint32_t, double)
template <typename T>
__device__ __forceinline__ T block_excl_scan256(T v, T* wsum, T* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T inc = v;
    for (int off = 1; off < 64; off <<= 1) {
        const T y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    T ex = __shfl_up(inc, 1);
    if (lane == 0) ex = T(0);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    T pre = T(0);
    for (int k = 0; k < wave; ++k) pre += wsum[k];
    *total = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
    __syncthreads();
    return pre + ex;
}

template <typename T>
__global__ __launch_bounds__(SC_T) void sc_reduce_kernel(int64_t n, int64_t chunk, const T* __restrict__ in,
                                                         T* __restrict__ partial) {
    __shared__ T red[4];
    const int64_t b0 = blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
    T s = T(0);
    for (int64_t i = b0 + threadIdx.x; i < b1; i += SC_T) s += in[i];
    s = block_sum256(s, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// one workgroup: exclusive scan of the G <= SC_MAX_BLOCKS partials, in place
template <typename T>
__global__ __launch_bounds__(SC_T) void sc_partials_kernel(int64_t G, T* __restrict__ partial) {
    __shared__ T wsum[4];
    constexpr int PER = SC_MAX_BLOCKS / SC_T;
    T x[PER];
    T s = T(0);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = threadIdx.x * PER + j;
        x[j] = i < G ? partial[i] : T(0);
        s += x[j];
    }
    T total;
    T run = block_excl_scan256(s, wsum, &total);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int64_t i = threadIdx.x * PER + j;
        if (i < G) partial[i] = run;
        run += x[j];
    }
}

template <typename T>
__global__ __launch_bounds__(SC_T) void sc_scan_kernel(int64_t n, int64_t chunk, const T* in, T* out,
                                                       const T* __restrict__ partial) {
    __shared__ T tile[SC_TILE];
    __shared__ T wsum[4];
    const int64_t b0 = blockIdx.x * chunk, b1 = b0 + chunk < n ? b0 + chunk : n;
    T carry = partial[blockIdx.x];
    for (int64_t t0 = b0; t0 < b1; t0 += SC_TILE) {
#pragma unroll
        for (int j = 0; j < SC_I; ++j) {
            const int64_t i = t0 + j * SC_T + threadIdx.x;
            tile[j * SC_T + threadIdx.x] = i < b1 ? in[i] : T(0);
        }
        __syncthreads();
        T x[SC_I];
        T s = T(0);
#pragma unroll
        for (int j = 0; j < SC_I; ++j) {
            x[j] = tile[threadIdx.x * SC_I + j];
            s += x[j];
        }
        T total;
        T run = carry + block_excl_scan256(s, wsum, &total);  // (barriers inside: the tile is read)
#pragma unroll
        for (int j = 0; j < SC_I; ++j) {
            tile[threadIdx.x * SC_I + j] = run;
            run += x[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SC_I; ++j) {
            const int64_t i = t0 + j * SC_T + threadIdx.x;
            if (i < b1) out[i] = tile[j * SC_T + threadIdx.x];
        }
        carry += total;
        __syncthreads();
    }
}

struct ScanPlan {
    int64_t G, chunk;
};

ScanPlan scan_plan(int64_t n) {
    int64_t G = (n + SC_TILE - 1) / SC_TILE;
    G = G < 1 ? 1 : (G > SC_MAX_BLOCKS ? SC_MAX_BLOCKS : G);
    int64_t chunk = (n + G - 1) / G;
    chunk = (chunk + SC_TILE - 1) / SC_TILE * SC_TILE;
    if (chunk < SC_TILE) chunk = SC_TILE;
    G = (n + chunk - 1) / chunk;
    return {G < 1 ? 1 : G, chunk};
}

template <typename T>
hipError_t excl_scan(hipStream_t s, int64_t n, const T* in, T* out, T* partial) {
    if (n <= 0) return hipSuccess;
    const ScanPlan p = scan_plan(n);
    hipLaunchKernelGGL(sc_reduce_kernel<T>, dim3((unsigned)p.G), dim3(SC_T), 0, s, n, p.chunk, in, partial);
    hipLaunchKernelGGL(sc_partials_kernel<T>, dim3(1), dim3(SC_T), 0, s, p.G, partial);
    hipLaunchKernelGGL(sc_scan_kernel<T>, dim3((unsigned)p.G), dim3(SC_T), 0, s, n, p.chunk, in, out,
                       (const T*)partial);
    return hipGetLastError();
}

// ---------------------------------------------------------------- count / select
constexpr int CNT_U = 8;
constexpr int64_t CNT_WG_PER_CU = 64;
constexpr int64_t CNT_MAX_BLOCKS = 16384;
constexpr int64_t SEL_WG_PER_CU = 16;

template <bool VEC>
__global__ __launch_bounds__(256) void cnt_kernel(int64_t n, const double* __restrict__ v, double acc,
                                                  unsigned long long* __restrict__ partial) {
    __shared__ unsigned long long red[4];
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t c = 0;
    if (VEC) {
        typedef double vd2 __attribute__((ext_vector_type(2)));
        const vd2* __restrict__ v2 = reinterpret_cast<const vd2*>(v);
        const int64_t n2 = n >> 1;
        // nontemporal: the 2^32-entry vector is read once; 8 loads in flight per lane at 64 workgroups per CU
        // (tools/count_bench.hip, one box: 4.95 ms vs 5.17 at 4 loads / 16 per CU and 5.49 at 4 / 4 per CU)
        for (; i + (CNT_U - 1) * stride < n2; i += CNT_U * stride) {
            vd2 x[CNT_U];
#pragma unroll
            for (int u = 0; u < CNT_U; ++u) x[u] = __builtin_nontemporal_load(v2 + i + u * stride);
#pragma unroll
            for (int u = 0; u < CNT_U; ++u) c += (fabs(x[u].x) > acc) + (fabs(x[u].y) > acc);
        }
        for (; i < n2; i += stride) {
            const vd2 a = v2[i];
            c += (fabs(a.x) > acc) + (fabs(a.y) > acc);
        }
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) c += fabs(v[n - 1]) > acc;
    } else {
        for (; i < n; i += stride) c += fabs(v[i]) > acc;
    }
    const unsigned long long s = block_sum256<unsigned long long>(c, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void cnt_final_kernel(int64_t G, const unsigned long long* __restrict__ partial,
                                                        int64_t* __restrict__ out) {
    __shared__ unsigned long long red[4];
    unsigned long long s = 0;
    for (int64_t i = threadIdx.x; i < G; i += 256) s += partial[i];
    s = block_sum256(s, red);
    if (threadIdx.x == 0) *out = (int64_t)s;
}

__global__ __launch_bounds__(256) void sel_kernel(int64_t n, const double* __restrict__ v, double acc,
                                                  int64_t* __restrict__ idx, double* __restrict__ vals,
                                                  unsigned long long* __restrict__ count, int64_t cap) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    const int64_t stride = (int64_t)gridDim.x * 256;
    // wave-uniform loop: every lane of a wave shares `b`
    for (int64_t b = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); b < n; b += stride) {
        const int64_t i = b + lane;
        const double x = i < n ? v[i] : 0.0;
        const bool keep = i < n && fabs(x) > acc;
        const uint64_t m = __ballot(keep);
        if (m) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(count, (unsigned long long)__popcll(m));
            base = __shfl(base, 0);
            if (keep) {
                const int64_t p = (int64_t)base + __popcll(m & below);
                if (p < cap) {
                    idx[p] = i;
                    vals[p] = x;
                }
            }
        }
    }
}

struct RsPlan {
    int64_t W, chunk;
};

RsPlan rs_plan(int64_t n) {
    int64_t W = (n + RS_ELEMS_PER_WAVE - 1) / RS_ELEMS_PER_WAVE;
    W = W < 1 ? 1 : (W > RS_MAX_WAVES ? RS_MAX_WAVES : W);
    int64_t chunk = ((n + W - 1) / W + 63) & ~int64_t(63);
    if (chunk < 64) chunk = 64;
    W = (n + chunk - 1) / chunk;
    return {W < 1 ? 1 : W, chunk};
}

}  // namespace

size_t scan_bytes(int64_t n) { return al256(sizeof(double) * (size_t)scan_plan(n > 0 ? n : 1).G); }

hipError_t exclusive_sum(hipStream_t s, int64_t n, const double* in, double* out, void* tmp, size_t tmp_bytes) {
    if (tmp_bytes < scan_bytes(n)) return hipErrorInvalidValue;
    return excl_scan<double>(s, n, in, out, (double*)tmp);
}

size_t radix_sort_bytes(int64_t n) {
    const size_t c = (size_t)(n > 0 ? n : 1);
    const RsPlan p = rs_plan(n > 0 ? n : 1);
    const int64_t nh = 256 * p.W;
    return 2 * al256(8 * c) + al256(4 * (size_t)nh) + al256(4 * (size_t)scan_plan(nh).G);
}

hipError_t radix_sort_pairs(hipStream_t s, int64_t n, const uint64_t* keys_in, const uint64_t* vals_in,
                            uint64_t* keys_out, uint64_t* vals_out, int begin_bit, int end_bit, KeyOrder order,
                            void* tmp, size_t tmp_bytes) {
    if (n < 0 || n > 0x7fffffff || begin_bit < 0 || end_bit > 64 || begin_bit > end_bit) return hipErrorInvalidValue;
    if (tmp_bytes < radix_sort_bytes(n)) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const int npass = (end_bit - begin_bit + 7) / 8;
    if (npass == 0) {
        hipError_t e = hipMemcpyAsync(keys_out, keys_in, 8 * (size_t)n, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
        return hipMemcpyAsync(vals_out, vals_in, 8 * (size_t)n, hipMemcpyDeviceToDevice, s);
    }
    const RsPlan p = rs_plan(n);
    char* base = (char*)tmp;
    size_t off = 0;
    uint64_t* kt = (uint64_t*)(base + off); off += al256(8 * (size_t)n);
    uint64_t* vt = (uint64_t*)(base + off); off += al256(8 * (size_t)n);
    uint32_t* hist = (uint32_t*)(base + off); off += al256(4 * (size_t)(256 * p.W));
    uint32_t* part = (uint32_t*)(base + off);
    const uint64_t *ks = keys_in, *vs = vals_in;
    for (int pass = 0; pass < npass; ++pass) {
        const int shift = begin_bit + 8 * pass;
        const int nb = end_bit - shift < 8 ? end_bit - shift : 8;
        // the last pass lands in the caller's buffers: alternate backwards from there
        const bool to_out = ((npass - 1 - pass) & 1) == 0;
        uint64_t* kd = to_out ? keys_out : kt;
        uint64_t* vd = to_out ? vals_out : vt;
        hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)p.W), dim3(64), 0, s, n, p.chunk, p.W, ks, shift, nb, (int)order,
                           hist);
        hipError_t e = excl_scan<uint32_t>(s, 256 * p.W, hist, hist, part);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(rs_scatter_kernel, dim3((unsigned)p.W), dim3(64), 0, s, n, p.chunk, p.W, ks, vs, kd, vd, shift,
                           nb, (int)order, (const uint32_t*)hist);
        ks = kd;
        vs = vd;
    }
    return hipGetLastError();
}

size_t count_bytes() { return al256(sizeof(unsigned long long) * CNT_MAX_BLOCKS); }

hipError_t count_abs_above(hipStream_t s, int cus, int64_t n, const double* v, double acc, int64_t* count_dev,
                           void* tmp, size_t tmp_bytes) {
    if (tmp_bytes < count_bytes()) return hipErrorInvalidValue;
    unsigned long long* partial = (unsigned long long*)tmp;
    int64_t G = (int64_t)(cus > 0 ? cus : 256) * CNT_WG_PER_CU;
    const int64_t need = (n / 2 + 255) / 256;
    G = G > need ? need : G;
    G = G < 1 ? 1 : (G > CNT_MAX_BLOCKS ? CNT_MAX_BLOCKS : G);
    if ((reinterpret_cast<uintptr_t>(v) & 15) == 0)
        hipLaunchKernelGGL(cnt_kernel<true>, dim3((unsigned)G), dim3(256), 0, s, n, v, acc, partial);
    else
        hipLaunchKernelGGL(cnt_kernel<false>, dim3((unsigned)G), dim3(256), 0, s, n, v, acc, partial);
    hipLaunchKernelGGL(cnt_final_kernel, dim3(1), dim3(256), 0, s, G, (const unsigned long long*)partial, count_dev);
    return hipGetLastError();
}

hipError_t select_abs_above(hipStream_t s, int cus, int64_t n, const double* v, double acc, int64_t* idx,
                            double* vals, unsigned long long* count, int64_t capacity) {
    if (n <= 0) return hipSuccess;
    int64_t G = (int64_t)(cus > 0 ? cus : 256) * SEL_WG_PER_CU;
    const int64_t need = (n + 255) / 256;
    G = G > need ? need : G;
    hipLaunchKernelGGL(sel_kernel, dim3((unsigned)(G < 1 ? 1 : G)), dim3(256), 0, s, n, v, acc, idx, vals, count,
                       capacity);
    return hipGetLastError();
}

}  // namespace qkp
