// write_probe6.hip — is the placement lottery a translation-reach effect? (round 4)
// write_probe5: physically contiguous allocations are fast for the static 512-KiB-task order at some
// physical placements and slow at others, while one 4-KiB chunk per workgroup is fast everywhere.
// If the cause is the number of distinct pages each XCD's resident workgroups write at once (the
// static order: 256 tasks 4 MiB apart per XCD), XCD-contiguous task orders (each XCD's resident
// workgroups on consecutive tasks) should be fast into every allocation. Store-only variants:
//   static 512 KiB at 64 / 8 workgroups per CU (shipped order), XCD-contiguous 512 / 128 / 64 KiB,
//   static 64 KiB, non-persistent 64 KiB; into NB hipMalloc buffers.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe6 tools/write_probe6.hip && tools/write_probe6 [NB]
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
__global__ __launch_bounds__(256) void f_comb(double* __restrict__ out, int lgR, int lgI) {
    const int64_t b = blockIdx.x;
    const int64_t r = b & ((1 << lgR) - 1), j = b >> lgR;
    const int I = 1 << lgI;
    d2_t* o = reinterpret_cast<d2_t*>(out) + (((j << (lgR + lgI)) + r) << 8) + threadIdx.x;
#pragma unroll 4
    for (int it = 0; it < I; ++it) o[(int64_t)it << (lgR + 8)] = (d2_t){(double)it, 1.0};
}
__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int bb, int64_t nblocks) {
    const int iters = 1 << (bb - 8);
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}


// XCD-contiguous: workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x owns the x-th eighth
// of the output and its workgroups l = b / 8 take tasks l, l + G / 8, ... of that eighth
__global__ __launch_bounds__(256) void f_block_xcd(double* __restrict__ out, int bb, int64_t nblocks) {
    const int x = blockIdx.x & 7;
    const int64_t l = blockIdx.x >> 3, gx = gridDim.x >> 3;
    const int64_t per = nblocks >> 3;
    const int iters = 1 << (bb - 8);
    for (int64_t t = l; t < per; t += gx) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + ((x * per + t) << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}
// the same, XCD read from the hardware register instead of assumed from blockIdx
__global__ __launch_bounds__(256) void f_block_xcd_hw(double* __restrict__ out, int bb, int64_t nblocks,
                                                      unsigned* __restrict__ ctr) {
    __shared__ unsigned slot;
    const int x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;
    if (threadIdx.x == 0) slot = atomicAdd(ctr + 64 * x, 1u);
    __syncthreads();
    const int64_t l = slot, gx = gridDim.x >> 3;
    const int64_t per = nblocks >> 3;
    const int iters = 1 << (bb - 8);
    for (int64_t t = l; t < per; t += gx) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + ((x * per + t) << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
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
    unsigned* ctr = nullptr;
    CK(hipMalloc(&ctr, 8 * 64 * sizeof(unsigned)));
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
    for (int wpc : {64, 8})
        pats.push_back({"static 512K " + std::to_string(wpc) + "/CU", [=](double* o) {
                            hipLaunchKernelGGL(f_block_static, dim3((unsigned)(cus * wpc)), dim3(256), 0, 0, o, 15, n2 >> 15);
                        }});
    for (int bb : {15, 13, 12})
        for (int wpc : {8, 64})
            pats.push_back({"xcd-contig " + std::to_string((16 << bb) >> 10) + "K " + std::to_string(wpc) + "/CU",
                            [=](double* o) {
                                hipLaunchKernelGGL(f_block_xcd, dim3((unsigned)(cus * wpc)), dim3(256), 0, 0, o, bb,
                                                   n2 >> bb);
                            }});
    pats.push_back({"xcd-contig hw 512K 8/CU", [=](double* o) {
                        (void)hipMemsetAsync(ctr, 0, 8 * 64 * sizeof(unsigned), 0);
                        hipLaunchKernelGGL(f_block_xcd_hw, dim3((unsigned)(cus * 8)), dim3(256), 0, 0, o, 15, n2 >> 15, ctr);
                    }});
    pats.push_back({"xcd-contig hw 64K 8/CU", [=](double* o) {
                        (void)hipMemsetAsync(ctr, 0, 8 * 64 * sizeof(unsigned), 0);
                        hipLaunchKernelGGL(f_block_xcd_hw, dim3((unsigned)(cus * 8)), dim3(256), 0, 0, o, 12, n2 >> 12, ctr);
                    }});
    pats.push_back({"static 64K 8/CU", [=](double* o) {
                        hipLaunchKernelGGL(f_block_static, dim3((unsigned)(cus * 8)), dim3(256), 0, 0, o, 12, n2 >> 12);
                    }});
    pats.push_back({"non-persistent 64K", [=](double* o) {
                        hipLaunchKernelGGL(f_block_static, dim3((unsigned)(n2 >> 12)), dim3(256), 0, 0, o, 12, n2 >> 12);
                    }});
    std::vector<std::vector<float>> res(pats.size(), std::vector<float>(NB));
    for (int b = 0; b < NB; ++b) {
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
    }
    printf("%-30s", "pattern (ms per 34.36 GB)");
    for (int b = 0; b < NB; ++b) printf("  buf%-4d", b);
    printf("\n");
    for (size_t p = 0; p < pats.size(); ++p) {
        printf("%-30s", pats[p].name.c_str());
        for (int b = 0; b < NB; ++b) printf("  %7.3f", res[p][b]);
        printf("\n");
    }
    for (double* p : bufs) CK(hipFree(p));
    return 0;
}
