// count_bench.hip — read-rate probe for the ACCURACY threshold count over 2^32 fp64 (qkp::count_abs_above,
// csrc/qknit_prim.hip): loads in flight per thread, nontemporal loads, grid width, contiguous chunks.
//   hipcc --offload-arch=gfx950 -O3 -o tools/count_bench tools/count_bench.hip && tools/count_bench [log2 n]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef double d2_t __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void count_stride(int64_t n2, const d2_t* __restrict__ v, double acc,
                                                    unsigned long long* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t c = 0;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        d2_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = NT ? __builtin_nontemporal_load(v + i + u * stride) : v[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) c += (fabs(x[u].x) > acc) + (fabs(x[u].y) > acc);
    }
    for (; i < n2; i += stride) {
        const d2_t x = v[i];
        c += (fabs(x.x) > acc) + (fabs(x.y) > acc);
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

// each workgroup one contiguous chunk, U 16-B loads per lane in flight per step
template <int U>
__global__ __launch_bounds__(256) void count_chunk(int64_t n2, int64_t chunk, const d2_t* __restrict__ v, double acc,
                                                   unsigned long long* __restrict__ out) {
    const int64_t b0 = (int64_t)blockIdx.x * chunk, b1 = b0 + chunk < n2 ? b0 + chunk : n2;
    uint32_t c = 0;
    int64_t i = b0 + threadIdx.x;
    for (; i + (U - 1) * 256 < b1; i += U * 256) {
        d2_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = v[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) c += (fabs(x[u].x) > acc) + (fabs(x[u].y) > acc);
    }
    for (; i < b1; i += 256) {
        const d2_t x = v[i];
        c += (fabs(x.x) > acc) + (fabs(x.y) > acc);
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;
    const int64_t n = int64_t(1) << lg, n2 = n / 2;
    int cus = 256;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    double* v;
    unsigned long long* cnt;
    CK(hipMalloc(&v, n * 8));
    CK(hipMalloc(&cnt, 8));
    CK(hipMemset(v, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        float best = 1e9, sum = 0;
        for (int r = 0; r < 6; ++r) {
            CK(hipMemset(cnt, 0, 8));
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) {
                best = ms < best ? ms : best;
                sum += ms;
            }
        }
        printf("{\"variant\": \"%s\", \"best_ms\": %.4f, \"avg_ms\": %.4f, \"TBs\": %.3f}\n", name, best, sum / 5,
               n * 8 / (best * 1e-3) / 1e12);
        fflush(stdout);
    };
    const d2_t* vv = reinterpret_cast<const d2_t*>(v);
    const bool nt_only = argc > 2 && atoi(argv[2]) == 1;  // round 2: nontemporal variants only, wider grids
    for (int wg : {4, 8, 16, 32, 64}) {
        const int G = cus * wg;
        char nm[64];
        if (!nt_only && wg <= 16) {
            snprintf(nm, sizeof nm, "stride U4 wg%d", wg);
            run(nm, [&] { hipLaunchKernelGGL((count_stride<4, false>), dim3(G), dim3(256), 0, 0, n2, vv, 1e-5, cnt); });
            snprintf(nm, sizeof nm, "stride U8 wg%d", wg);
            run(nm, [&] { hipLaunchKernelGGL((count_stride<8, false>), dim3(G), dim3(256), 0, 0, n2, vv, 1e-5, cnt); });
        }
        snprintf(nm, sizeof nm, "stride U4 nt wg%d", wg);
        run(nm, [&] { hipLaunchKernelGGL((count_stride<4, true>), dim3(G), dim3(256), 0, 0, n2, vv, 1e-5, cnt); });
        if (nt_only) {
            snprintf(nm, sizeof nm, "stride U2 nt wg%d", wg);
            run(nm, [&] { hipLaunchKernelGGL((count_stride<2, true>), dim3(G), dim3(256), 0, 0, n2, vv, 1e-5, cnt); });
            snprintf(nm, sizeof nm, "stride U8 nt wg%d", wg);
            run(nm, [&] { hipLaunchKernelGGL((count_stride<8, true>), dim3(G), dim3(256), 0, 0, n2, vv, 1e-5, cnt); });
        }
    }
    for (int64_t ck : {int64_t(1) << 12, int64_t(1) << 14, int64_t(1) << 16}) {  // d2 elements per workgroup
        char nm[64];
        snprintf(nm, sizeof nm, "chunk %lld U4", (long long)ck * 16);
        const int64_t G = (n2 + ck - 1) / ck;
        run(nm, [&] { hipLaunchKernelGGL((count_chunk<4>), dim3((unsigned)G), dim3(256), 0, 0, n2, ck, vv, 1e-5, cnt); });
    }
    CK(hipFree(v));
    return 0;
}
