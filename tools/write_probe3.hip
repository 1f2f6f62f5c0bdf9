// write_probe3.hip — a knit written in the one-workgroup-per-4-KiB-chunk order (round 4).
// write_probe2 showed that of all store orders only the non-persistent one-chunk-per-workgroup
// order writes 2^32 fp64 at ~4.9 ms into every allocation (the shipped static 512-KiB-task order:
// 4.8 ms into some, 5.7-6.0 into others). Timed here into NB allocations: that store order alone,
// with two / four far-apart chunks per workgroup, and the knit in that order (operands gathered
// from L2 per lane, K from a device int, the first rows loaded before K is known) against the
// shipped kernel's static order, on syc 32 5's masks (A 0xF0F0F0F0, B 0x0F0F0F0F, K = 2) and
// syc 32 1's (A 0xFFFF0000, B 0xFFFF, K = 1).
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe3 tools/write_probe3.hip && tools/write_probe3 [NB]
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
// C chunks per workgroup: chunk b + j * (nchunks / C)
template <int C>
__global__ __launch_bounds__(256) void f_far(double* __restrict__ out, int64_t nchunks) {
    const int64_t step = nchunks / C;
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const int64_t c = blockIdx.x + j * step;
        reinterpret_cast<d2_t*>(out)[c * 256 + threadIdx.x] = (d2_t){(double)c, 1.0};
    }
}
// 512 threads: one 8-KiB chunk per workgroup (each wave 1 KiB)
__global__ __launch_bounds__(512) void f_one16_512(double* __restrict__ out, int64_t n2) {
    const int64_t i = (int64_t)blockIdx.x * 512 + threadIdx.x;
    if (i < n2) reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}

__device__ __forceinline__ uint32_t pext32(uint32_t x, uint32_t mask) {
    uint32_t r = 0, bit = 1;
    for (; mask; mask &= mask - 1, bit <<= 1)
        if (x & mask & (~mask + 1)) r |= bit;
    return r;
}

struct NPArgs {
    int K;  // host upper bound of the device K
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    const int* __restrict__ kdev;
    double* __restrict__ out;
    int64_t nchunks;
};

constexpr int KSPEC = 2;  // rows loaded before the device K arrives
constexpr int KMAX = 8;

// C chunks per workgroup (chunk b + j nchunks / C), operands gathered per lane
template <int C>
__global__ __launch_bounds__(256) void k_np(NPArgs a) {
    const int64_t step = a.nchunks / C;
    const int kd = *a.kdev;
    const uint32_t lane_o = 2u * threadIdx.x;
    const uint32_t rl = pext32(lane_o, a.maskA & 511u), cl = pext32(lane_o, a.maskB & 511u);
    const int ks = a.K < KSPEC ? a.K : KSPEC;
    double av[C][KSPEC];
    d2_t bv[C][KSPEC];
    uint32_t row[C], col[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const uint32_t base = (uint32_t)((blockIdx.x + j * step) << 9);
        row[j] = pext32(base, a.maskA) + rl;
        col[j] = pext32(base, a.maskB) + cl;
#pragma unroll
        for (int k = 0; k < KSPEC; ++k)
            if (k < ks) {
                av[j][k] = a.A[k * a.lda + row[j]];
                bv[j][k] = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col[j]);
            }
    }
    int K = kd < a.K ? kd : a.K;
    if (K <= 0) return;
#pragma unroll
    for (int j = 0; j < C; ++j) {
        d2_t acc = {0.0, 0.0};
#pragma unroll
        for (int k = 0; k < KSPEC; ++k)
            if (k < K) {
                acc.x = fma(av[j][k], bv[j][k].x, acc.x);
                acc.y = fma(av[j][k], bv[j][k].y, acc.y);
            }
        for (int k = KSPEC; k < K; ++k) {
            const double x = a.A[k * a.lda + row[j]];
            const d2_t y = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col[j]);
            acc.x = fma(x, y.x, acc.x);
            acc.y = fma(x, y.y, acc.y);
        }
        const int64_t c = blockIdx.x + j * step;
        *reinterpret_cast<d2_t*>(a.out + c * 512 + lane_o) = acc;
    }
}

// the shipped kernel's order: persistent, static 2^16-output tasks, operands staged in LDS (LDS
// stage of A only + B from global when BG)
struct OBArgs {
    int K, TB;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    int64_t ntasks;
    const int* kdev;
    double* __restrict__ out;
};
template <bool BG>
__global__ __launch_bounds__(256) void k_static(OBArgs a) {
    int K = a.K;
    {
        const int kd = *a.kdev;
        if (kd <= 0) return;
        K = kd < K ? kd : K;
    }
    __shared__ uint32_t tab[2][2][256];
    extern __shared__ double stage[];
    const uint32_t low = (1u << a.TB) - 1u;
    const uint32_t mAl = a.maskA & low, mBl = a.maskB & low;
    const int na = 1 << __builtin_popcount(mAl), nb = 1 << __builtin_popcount(mBl);
    double* sA = stage;
    double* sB = stage + (int64_t)a.K * na;
    for (int i = threadIdx.x; i < 512; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), mAl);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), mBl);
    }
    __syncthreads();
    const uint32_t r0 = tab[0][0][(2 * threadIdx.x) & 255], c0 = tab[1][0][(2 * threadIdx.x) & 255];
    const int iters = (1 << a.TB) / 512;
    for (int64_t t = blockIdx.x; t < a.ntasks; t += gridDim.x) {
        const uint32_t base = (uint32_t)(t << a.TB);
        const uint32_t ah = pext32(base, a.maskA), bh = pext32(base, a.maskB);
        __syncthreads();
        for (int i = threadIdx.x; i < K * na; i += 256) {
            const int k = i / na;
            sA[i] = a.A[k * a.lda + ah + (i - k * na)];
        }
        if (!BG)
            for (int i = threadIdx.x; i < K * nb; i += 256) {
                const int k = i / nb;
                sB[i] = a.B[k * a.ldb + bh + (i - k * nb)];
            }
        __syncthreads();
        const double* Bg = a.B + bh;
        double* o = a.out + (int64_t)base;
#pragma unroll 4
        for (int it = 0; it < iters; ++it) {
            const uint32_t hi = (uint32_t)(2 * it + (threadIdx.x >> 7));
            const uint32_t row = r0 + tab[0][1][hi], col = c0 + tab[1][1][hi];
            d2_t acc = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < KMAX; ++k)
                if (k < K) {
                    const double av = sA[k * na + row];
                    const d2_t bv = BG ? *reinterpret_cast<const d2_t*>(Bg + k * a.ldb + col)
                                       : *reinterpret_cast<const d2_t*>(sB + k * nb + col);
                    acc.x = fma(av, bv.x, acc.x);
                    acc.y = fma(av, bv.y, acc.y);
                }
            *reinterpret_cast<d2_t*>(o + 512 * it + 2 * threadIdx.x) = acc;
        }
    }
}

static uint32_t pext_h(uint32_t x, uint32_t m) {
    uint32_t r = 0, bit = 1;
    for (; m; m &= m - 1, bit <<= 1)
        if (x & m & (~m + 1)) r |= bit;
    return r;
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 4;
    const int64_t total = int64_t(1) << 32;
    const int64_t n2 = total / 2, nchunks = total / 512;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<double*> bufs;
    for (int b = 0; b < NB; ++b) {
        double* p = nullptr;
        CK(hipMalloc(&p, total * 8));
        bufs.push_back(p);
    }
    // operands: K rows of 2^16 per side, seeded values
    const int64_t L = 65536;
    std::vector<double> hA(2 * L), hB(2 * L);
    for (int64_t i = 0; i < 2 * L; ++i) {
        hA[i] = std::sin(0.37 * (double)i + 0.1) * 1e-3;
        hB[i] = std::cos(0.53 * (double)i + 0.2) * 1e-3;
    }
    double *A = nullptr, *B = nullptr;
    int *kd = nullptr, *kd1 = nullptr;
    CK(hipMalloc(&A, 2 * L * 8));
    CK(hipMalloc(&B, 2 * L * 8));
    CK(hipMemcpy(A, hA.data(), 2 * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), 2 * L * 8, hipMemcpyHostToDevice));
    int two = 2, one = 1;
    CK(hipMalloc(&kd, 4));
    CK(hipMalloc(&kd1, 4));
    CK(hipMemcpy(kd, &two, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(kd1, &one, 4, hipMemcpyHostToDevice));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));

    struct Pat {
        std::string name;
        std::function<void(double*)> fn;
    };
    std::vector<Pat> pats;
    pats.push_back({"fill one16", [&](double* o) {
                        hipLaunchKernelGGL(f_one16, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, o, n2);
                    }});
    pats.push_back({"fill one16, 512 threads", [&](double* o) {
                        hipLaunchKernelGGL(f_one16_512, dim3((unsigned)(n2 / 512)), dim3(512), 0, 0, o, n2);
                    }});
    pats.push_back({"fill 2 far chunks", [&](double* o) {
                        hipLaunchKernelGGL(f_far<2>, dim3((unsigned)(nchunks / 2)), dim3(256), 0, 0, o, nchunks);
                    }});
    pats.push_back({"fill 4 far chunks", [&](double* o) {
                        hipLaunchKernelGGL(f_far<4>, dim3((unsigned)(nchunks / 4)), dim3(256), 0, 0, o, nchunks);
                    }});
    struct Cfg {
        const char* name;
        uint32_t mA, mB;
        int K;
        int* kd;
    } cfgs[2] = {{"syc32_5", 0xF0F0F0F0u, 0x0F0F0F0Fu, 2, kd}, {"syc32_1", 0xFFFF0000u, 0x0000FFFFu, 1, kd1}};
    for (const Cfg& c : cfgs) {
        NPArgs na{c.K, A, L, B, L, c.mA, c.mB, c.kd, nullptr, nchunks};
        pats.push_back({std::string("knit np 1 chunk ") + c.name, [=](double* o) {
                            NPArgs a = na;
                            a.out = o;
                            hipLaunchKernelGGL(k_np<1>, dim3((unsigned)nchunks), dim3(256), 0, 0, a);
                        }});
        pats.push_back({std::string("knit np 2 far ") + c.name, [=](double* o) {
                            NPArgs a = na;
                            a.out = o;
                            hipLaunchKernelGGL(k_np<2>, dim3((unsigned)(nchunks / 2)), dim3(256), 0, 0, a);
                        }});
        pats.push_back({std::string("knit np 4 far ") + c.name, [=](double* o) {
                            NPArgs a = na;
                            a.out = o;
                            hipLaunchKernelGGL(k_np<4>, dim3((unsigned)(nchunks / 4)), dim3(256), 0, 0, a);
                        }});
        const bool bg = c.mB == 0xFFFFu;
        const int tb = 16;
        const size_t st = 8 * (size_t)c.K * ((size_t(1) << __builtin_popcount(c.mA & 0xFFFF)) +
                                             (bg ? 0 : (size_t(1) << __builtin_popcount(c.mB & 0xFFFF))));
        OBArgs ob{c.K, tb, A, L, B, L, c.mA, c.mB, total >> tb, c.kd, nullptr};
        pats.push_back({std::string("knit static (shipped) ") + c.name, [=](double* o) {
                            OBArgs a = ob;
                            a.out = o;
                            if (bg)
                                hipLaunchKernelGGL(k_static<true>, dim3((unsigned)(cus * 64)), dim3(256), st, 0, a);
                            else
                                hipLaunchKernelGGL(k_static<false>, dim3((unsigned)(cus * 64)), dim3(256), st, 0, a);
                        }});
    }

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
        printf("buffer %d done\n", b);
        fflush(stdout);
    }
    // spot-check the knit values of the last pattern run per config against the host
    {
        std::vector<double> h(1 << 20);
        for (const Cfg& c : cfgs) {
            NPArgs a{c.K, A, L, B, L, c.mA, c.mB, c.kd, bufs[0], nchunks};
            hipLaunchKernelGGL(k_np<2>, dim3((unsigned)(nchunks / 2)), dim3(256), 0, 0, a);
            CK(hipDeviceSynchronize());
            double maxd = 0;
            for (int64_t off : {int64_t(0), (int64_t(1) << 31) + 12345 * 512, total - (1 << 20)}) {
                CK(hipMemcpy(h.data(), bufs[0] + off, h.size() * 8, hipMemcpyDeviceToHost));
                for (int64_t i = 0; i < (int64_t)h.size(); i += 97) {
                    const uint32_t o = (uint32_t)(off + i);
                    double v = 0;
                    for (int k = 0; k < c.K; ++k) v = std::fma(hA[k * L + pext_h(o, c.mA)], hB[k * L + pext_h(o, c.mB)], v);
                    maxd = std::max(maxd, std::fabs(v - h[i]));
                }
            }
            printf("check %s: max |np - host| = %.3g\n", c.name, maxd);
        }
    }
    printf("%-36s", "pattern (ms per 34.36 GB)");
    for (int b = 0; b < NB; ++b) printf("  buf%-4d", b);
    printf("\n");
    for (size_t p = 0; p < pats.size(); ++p) {
        printf("%-36s", pats[p].name.c_str());
        for (int b = 0; b < NB; ++b) printf("  %7.3f", res[p][b]);
        printf("\n");
    }
    for (double* p : bufs) CK(hipFree(p));
    return 0;
}
