// write_probe8.hip — do persistent writers lose to one-chunk-per-workgroup by having too many
// stores in flight? (round 4) Persistent store orders with an explicit wait after each store
// (W = stores a wave may have in flight: vmcnt(W - 1) before the next), into NB allocations.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe8 tools/write_probe8.hip && tools/write_probe8 [NB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef double d2_t __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void f_one16(double* __restrict__ out, int64_t n2) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n2) reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}
// comb tasks, store only: workgroup b = j R + r writes chunks j R I + it R + r

__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int bb, int64_t nblocks) {
    const int iters = 1 << (bb - 8);
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}
template <int W>
__device__ __forceinline__ void vm_wait() {
    if (W == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (W == 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    if (W == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    if (W == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
}
template <int W>
__global__ __launch_bounds__(256) void f_static_w(double* __restrict__ out, int bb, int64_t nblocks) {
    const int iters = 1 << (bb - 8);
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << bb);
        for (int it = 0; it < iters; ++it) {
            o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
            vm_wait<W>();
        }
    }
}
template <int W>
__global__ __launch_bounds__(256) void f_stride_w(double* __restrict__ out, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
        vm_wait<W>();
    }
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 5;
    const int64_t total = int64_t(1) << 32;
    const int64_t n2 = total / 2;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<double*> bufs;
    for (int b = 0; b < NB; ++b) {
        double* p = nullptr;
        CK(hipMalloc(&p, total * 8));
        bufs.push_back(p);
    }
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    struct Pat {
        std::string name;
        std::function<void(double*)> fn;
    };
    std::vector<Pat> pats;
    pats.push_back({"one16", [&](double* o) {
                        hipLaunchKernelGGL(f_one16, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, o, n2);
                    }});
    pats.push_back({"static 512K 64/CU", [=](double* o) {
                        hipLaunchKernelGGL(f_block_static, dim3((unsigned)(cus * 64)), dim3(256), 0, 0, o, 15, n2 >> 15);
                    }});
#define SW(W, WPC)                                                                                               \
    pats.push_back({"static 512K " #WPC "/CU w" #W, [=](double* o) {                                             \
                        hipLaunchKernelGGL(f_static_w<W>, dim3((unsigned)(cus * WPC)), dim3(256), 0, 0, o, 15, n2 >> 15); \
                    }});
#define GW(W, WPC)                                                                                              \
    pats.push_back({"grid-stride " #WPC "/CU w" #W, [=](double* o) {                                            \
                        hipLaunchKernelGGL(f_stride_w<W>, dim3((unsigned)(cus * WPC)), dim3(256), 0, 0, o, n2); \
                    }});
    SW(1, 8) SW(2, 8) SW(4, 8) SW(8, 8) SW(1, 64) SW(4, 64) GW(1, 8) GW(2, 8) GW(4, 8) GW(1, 64) GW(4, 64)
    std::vector<std::vector<float>> res(pats.size(), std::vector<float>(NB));
    for (int b = 0; b < NB; ++b)
        for (size_t p = 0; p < pats.size(); ++p) {
            pats[p].fn(bufs[b]);
            CK(hipDeviceSynchronize());
            std::vector<float> ms;
            for (int r = 0; r < 3; ++r) {
                CK(hipEventRecord(s, 0));
                pats[p].fn(bufs[b]);
                CK(hipEventRecord(e, 0));
                CK(hipEventSynchronize(e));
                float t = 0;
                CK(hipEventElapsedTime(&t, s, e));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            res[p][b] = ms[1];
        }
    printf("%-26s", "pattern (ms)");
    for (int b = 0; b < NB; ++b) printf("  buf%-4d", b);
    printf("\n");
    for (size_t p = 0; p < pats.size(); ++p) {
        printf("%-26s", pats[p].name.c_str());
        for (int b = 0; b < NB; ++b) printf("  %7.3f", res[p][b]);
        printf("\n");
    }
    return 0;
}
