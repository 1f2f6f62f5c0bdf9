// write_probe7.hip — why is a knit workgroup per 4-KiB chunk slow? (round 4)
// write_probe3: one knit workgroup per chunk (operands gathered from L2 per lane) takes 20 ms for
// 2^32 outputs where a store-only workgroup per chunk takes 4.9 ms. Variants here separate the
// index arithmetic (pext over 32-bit masks), the operand loads and the device-K load:
//   np-full: per-lane pext loops + loads (write_probe3's kernel)
//   np-hd: pext by precomputed compress constants (Hacker's Delight 7-4, 5 steps, masks fixed per launch)
//   np-noload: the pext arithmetic, no operand loads (values from the indices)
//   np-fixed: loads from fixed rows (no pext)
//   np-hd-nok: np-hd without the device-K load
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe7 tools/write_probe7.hip && tools/write_probe7 [NB]
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


__device__ __forceinline__ uint32_t pext32(uint32_t x, uint32_t mask) {
    uint32_t r = 0, bit = 1;
    for (; mask; mask &= mask - 1, bit <<= 1)
        if (x & mask & (~mask + 1)) r |= bit;
    return r;
}
// compress (pext) with the five move masks of Hacker's Delight 7-4, computed on the host
struct Cmp {
    uint32_t m, mv[5];
};
static Cmp cmp_consts(uint32_t m) {
    Cmp c;
    c.m = m;
    uint32_t mk = ~m << 1;
    for (int i = 0; i < 5; ++i) {
        uint32_t mp = mk ^ (mk << 1);
        mp ^= mp << 2;
        mp ^= mp << 4;
        mp ^= mp << 8;
        mp ^= mp << 16;
        const uint32_t mv = mp & m;
        c.mv[i] = mv;
        m = (m ^ mv) | (mv >> (1 << i));
        mk &= ~mp;
    }
    return c;
}
__device__ __forceinline__ uint32_t pext_hd(uint32_t x, const Cmp& c) {
    x &= c.m;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t t = x & c.mv[i];
        x = (x ^ t) | (t >> (1 << i));
    }
    return x;
}
static uint32_t pext_h(uint32_t x, uint32_t m) {
    uint32_t r = 0, bit = 1;
    for (; m; m &= m - 1, bit <<= 1)
        if (x & m & (~m + 1)) r |= bit;
    return r;
}

struct NPArgs {
    int K;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    Cmp cA, cB;
    const int* __restrict__ kdev;
    double* __restrict__ out;
};
constexpr int KS = 2;
// mode 0 full (loop pext), 1 hd pext, 2 no loads, 3 fixed rows, 4 hd without the device K
template <int MODE>
__global__ __launch_bounds__(256) void k_np(NPArgs a) {
    const uint32_t o = (blockIdx.x << 9) | (threadIdx.x << 1);
    uint32_t row, col;
    if (MODE == 0) {
        row = pext32(blockIdx.x << 9, a.maskA) + pext32(threadIdx.x << 1, a.maskA & 511u);
        col = pext32(blockIdx.x << 9, a.maskB) + pext32(threadIdx.x << 1, a.maskB & 511u);
    } else if (MODE == 3) {
        row = threadIdx.x & 15;
        col = (threadIdx.x & 7) * 2;
    } else {
        row = pext_hd(o, a.cA);
        col = pext_hd(o, a.cB);
    }
    int K = a.K;
    if (MODE != 4) {
        const int kd = *a.kdev;
        K = kd < K ? kd : K;
    }
    d2_t acc = {0.0, 0.0};
    if (MODE == 2) {
        acc.x = (double)row;
        acc.y = (double)col;
    } else {
        double av[KS];
        d2_t bv[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k)
            if (k < a.K) {
                av[k] = a.A[k * a.lda + row];
                bv[k] = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col);
            }
#pragma unroll
        for (int k = 0; k < KS; ++k)
            if (k < K) {
                acc.x = fma(av[k], bv[k].x, acc.x);
                acc.y = fma(av[k], bv[k].y, acc.y);
            }
    }
    if (K <= 0) return;
    *reinterpret_cast<d2_t*>(a.out + o) = acc;
}

// C chunks per workgroup: FAR: chunk b + j (nchunks / C); else C consecutive chunks b C + j
template <int C, bool FAR>
__global__ __launch_bounds__(256) void k_np_multi(NPArgs a, int64_t nchunks) {
    const int kd = *a.kdev;
    const int K = kd < a.K ? kd : a.K;
    double av[C][KS];
    d2_t bv[C][KS];
    uint32_t o[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const uint32_t c = FAR ? (uint32_t)(blockIdx.x + j * (nchunks / C)) : (uint32_t)(blockIdx.x * C + j);
        o[j] = (c << 9) | (threadIdx.x << 1);
        const uint32_t row = pext_hd(o[j], a.cA), col = pext_hd(o[j], a.cB);
#pragma unroll
        for (int k = 0; k < KS; ++k)
            if (k < a.K) {
                av[j][k] = a.A[k * a.lda + row];
                bv[j][k] = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col);
            }
    }
    if (K <= 0) return;
#pragma unroll
    for (int j = 0; j < C; ++j) {
        d2_t acc = {0.0, 0.0};
#pragma unroll
        for (int k = 0; k < KS; ++k)
            if (k < K) {
                acc.x = fma(av[j][k], bv[j][k].x, acc.x);
                acc.y = fma(av[j][k], bv[j][k].y, acc.y);
            }
        *reinterpret_cast<d2_t*>(a.out + o[j]) = acc;
    }
}
// 512 threads, one 8-KiB (2-chunk) block per workgroup, one store per lane
__global__ __launch_bounds__(512) void k_np512(NPArgs a) {
    const uint32_t o = (blockIdx.x << 10) | (threadIdx.x << 1);
    const uint32_t row = pext_hd(o, a.cA), col = pext_hd(o, a.cB);
    const int kd = *a.kdev;
    const int K = kd < a.K ? kd : a.K;
    double av[KS];
    d2_t bv[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k)
        if (k < a.K) {
            av[k] = a.A[k * a.lda + row];
            bv[k] = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col);
        }
    if (K <= 0) return;
    d2_t acc = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < KS; ++k)
        if (k < K) {
            acc.x = fma(av[k], bv[k].x, acc.x);
            acc.y = fma(av[k], bv[k].y, acc.y);
        }
    *reinterpret_cast<d2_t*>(a.out + o) = acc;
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 2;
    const int64_t total = int64_t(1) << 32;
    const int64_t n2 = total / 2, nchunks = total / 512;
    std::vector<double*> bufs;
    for (int b = 0; b < NB; ++b) {
        double* p = nullptr;
        CK(hipMalloc(&p, total * 8));
        bufs.push_back(p);
    }
    const int64_t L = 65536;
    std::vector<double> hA(2 * L), hB(2 * L);
    for (int64_t i = 0; i < 2 * L; ++i) {
        hA[i] = std::sin(0.37 * (double)i + 0.1) * 1e-3;
        hB[i] = std::cos(0.53 * (double)i + 0.2) * 1e-3;
    }
    double *A = nullptr, *B = nullptr;
    int* kd = nullptr;
    CK(hipMalloc(&A, 2 * L * 8));
    CK(hipMalloc(&B, 2 * L * 8));
    CK(hipMemcpy(A, hA.data(), 2 * L * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), 2 * L * 8, hipMemcpyHostToDevice));
    int two = 2;
    CK(hipMalloc(&kd, 4));
    CK(hipMemcpy(kd, &two, 4, hipMemcpyHostToDevice));
    for (uint32_t m : {0xF0F0F0F0u, 0x0F0F0F0Fu, 0xFFFF0000u, 0x12345678u})
        for (uint32_t x : {0u, 0xFFFFFFFFu, 0xDEADBEEFu, 0x13579BDFu})
            if (pext_h(x, m) != [&] { Cmp c = cmp_consts(m); uint32_t y = x & c.m; for (int i = 0; i < 5; ++i) { uint32_t t = y & c.mv[i]; y = (y ^ t) | (t >> (1 << i)); } return y; }())
                printf("pext_hd mismatch m %08x x %08x\n", m, x);
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
    NPArgs na{2, A, L, B, L, 0xF0F0F0F0u, 0x0F0F0F0Fu, cmp_consts(0xF0F0F0F0u), cmp_consts(0x0F0F0F0Fu), kd, nullptr};
    auto add = [&](const char* nm, auto kern) {
        pats.push_back({nm, [=](double* o) {
                            NPArgs a = na;
                            a.out = o;
                            hipLaunchKernelGGL(kern, dim3((unsigned)nchunks), dim3(256), 0, 0, a);
                        }});
    };
    add("np-full", k_np<0>);
    add("np-hd", k_np<1>);
    add("np-noload", k_np<2>);
    add("np-fixed", k_np<3>);
    add("np-hd-nok", k_np<4>);
    auto addm = [&](const char* nm, auto kern, int C) {
        pats.push_back({nm, [=](double* o) {
                            NPArgs a = na;
                            a.out = o;
                            hipLaunchKernelGGL(kern, dim3((unsigned)(nchunks / C)), dim3(256), 0, 0, a, nchunks);
                        }});
    };
    addm("np-hd 2 far", k_np_multi<2, true>, 2);
    addm("np-hd 4 far", k_np_multi<4, true>, 4);
    addm("np-hd 2 adjacent", k_np_multi<2, false>, 2);
    addm("np-hd 4 adjacent", k_np_multi<4, false>, 4);
    pats.push_back({"np-hd 512 threads", [=](double* o) {
                        NPArgs a = na;
                        a.out = o;
                        hipLaunchKernelGGL(k_np512, dim3((unsigned)(nchunks / 2)), dim3(512), 0, 0, a);
                    }});
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
    {  // np-hd values against the host
        std::vector<double> h(1 << 20);
        NPArgs a = na;
        a.out = bufs[0];
        hipLaunchKernelGGL(k_np<1>, dim3((unsigned)nchunks), dim3(256), 0, 0, a);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), bufs[0] + (int64_t(3) << 30), h.size() * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t i = 0; i < (int64_t)h.size(); ++i) {
            const uint32_t o = (uint32_t)((int64_t(3) << 30) + i);
            double v = 0;
            for (int k = 0; k < 2; ++k) v = std::fma(hA[k * L + pext_h(o, 0xF0F0F0F0u)], hB[k * L + pext_h(o, 0x0F0F0F0Fu)], v);
            bad += v != h[i];
        }
        printf("np-hd: %lld of %zu differ from the host\n", (long long)bad, h.size());
    }
    printf("%-20s", "pattern (ms)");
    for (int b = 0; b < NB; ++b) printf("  buf%-4d", b);
    printf("\n");
    for (size_t p = 0; p < pats.size(); ++p) {
        printf("%-20s", pats[p].name.c_str());
        for (int b = 0; b < NB; ++b) printf("  %7.3f", res[p][b]);
        printf("\n");
    }
    return 0;
}
