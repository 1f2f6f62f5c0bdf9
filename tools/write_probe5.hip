// write_probe5.hip — allocation methods (kernels from write_probe4): one workgroup per task, non-persistent (round 4).
// write_probe2/3: only the non-persistent one-4-KiB-chunk-per-workgroup store order is fast into
// every allocation; every order in which each resident workgroup streams its own region (the
// shipped static 512-KiB tasks, grid-stride) is fast into some allocations and slow into others,
// and a knit workgroup per chunk is latency bound (20 ms). Here a task is a COMB: task (j, r)
// writes the 4-KiB chunks j R I + it R + r, it < I, so the R tasks dispatched together write one
// contiguous R x 4 KiB window per iteration (like one-chunk-per-workgroup), while each workgroup
// still writes I chunks from one operand stage. The dispatcher's in-order launch keeps the running
// tasks consecutive (no drift as in a persistent grid).
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe4 tools/write_probe4.hip && tools/write_probe4 [NB]
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
__device__ __forceinline__ uint32_t pdep32(uint32_t x, uint32_t mask) {
    uint32_t r = 0, bit = 1;
    for (; mask; mask &= mask - 1, bit <<= 1)
        if (x & bit) r |= mask & (~mask + 1);
    return r;
}

constexpr int KMAX = 8;

// comb-task knit: out[o] = sum_k A[k][pext(o, mA)] B[k][pext(o, mB)]. Local coordinate lam (< 2^(9 +
// lgI)): bits 0..8 = output bits 0..8, bits 9.. = output bits 9 + lgR ..; o = base(j, r) + map(lam)
struct CombArgs {
    int K, lgR, lgI;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    const int* __restrict__ kdev;
    double* __restrict__ out;
};
__device__ __forceinline__ uint32_t lam_to_o(uint32_t lam, int lgR) {
    return (lam & 511u) | ((lam >> 9) << (9 + lgR));
}
__device__ __forceinline__ uint32_t o_to_lam_mask(uint32_t m, int lgR, int lgI) {  // lam bits whose o bit is in m
    const uint32_t lo = m & 511u;
    const uint32_t hi = (m >> (9 + lgR)) & ((1u << lgI) - 1u);
    return lo | (hi << 9);
}
__global__ __launch_bounds__(256) void k_comb(CombArgs a) {
    int K = a.K;
    {
        const int kd = *a.kdev;
        if (kd <= 0) return;
        K = kd < K ? kd : K;
    }
    __shared__ uint32_t tab[2][2][256];
    extern __shared__ double stage[];
    const uint32_t lA = o_to_lam_mask(a.maskA, a.lgR, a.lgI), lB = o_to_lam_mask(a.maskB, a.lgR, a.lgI);
    const int na = 1 << __builtin_popcount(lA), nb = 1 << __builtin_popcount(lB);
    double* sA = stage;
    double* sB = stage + (int64_t)a.K * na;
    const uint32_t b = blockIdx.x;
    const uint32_t r = b & ((1u << a.lgR) - 1u), j = b >> a.lgR;
    const uint32_t base = ((j << (a.lgR + a.lgI)) + r) << 9;  // output offset of lam = 0
    const uint32_t ah = pext32(base, a.maskA), bh = pext32(base, a.maskB);
    for (int i = threadIdx.x; i < K * na; i += 256) {
        const int k = i / na, s = i - k * na;
        sA[i] = a.A[k * a.lda + ah + pext32(lam_to_o(pdep32(s, lA), a.lgR), a.maskA)];
    }
    for (int i = threadIdx.x; i < K * nb; i += 256) {
        const int k = i / nb, s = i - k * nb;
        sB[i] = a.B[k * a.ldb + bh + pext32(lam_to_o(pdep32(s, lB), a.lgR), a.maskB)];
    }
    for (int i = threadIdx.x; i < 512; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), lA);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), lB);
    }
    __syncthreads();
    const uint32_t r0 = tab[0][0][(2 * threadIdx.x) & 255], c0 = tab[1][0][(2 * threadIdx.x) & 255];
    const int I = 1 << a.lgI;
    double* o = a.out + base + 2 * threadIdx.x;
#pragma unroll 4
    for (int it = 0; it < I; ++it) {
        const uint32_t hi = (uint32_t)(2 * it + (threadIdx.x >> 7));  // lam bits 8..15
        const uint32_t row = r0 + tab[0][1][hi], col = c0 + tab[1][1][hi];
        d2_t acc = {0.0, 0.0};
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (k < K) {
                const double av = sA[k * na + row];
                const d2_t bv = *reinterpret_cast<const d2_t*>(sB + k * nb + col);
                acc.x = fma(av, bv.x, acc.x);
                acc.y = fma(av, bv.y, acc.y);
            }
        *reinterpret_cast<d2_t*>(o + ((int64_t)it << (9 + a.lgR))) = acc;
    }
}

// the shipped kernel (persistent, static contiguous 2^16-output tasks)
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


struct Buf {
    std::string how;
    double* p;
    std::function<void()> release;
};

int main(int argc, char** argv) {
    const int64_t total = int64_t(1) << 32;
    const size_t bytes = (size_t)total * 8;
    const int64_t n2 = total / 2;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
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
    pats.push_back({"fill static 512K 64/CU", [&](double* o) {
                        hipLaunchKernelGGL(f_block_static, dim3((unsigned)(cus * 64)), dim3(256), 0, 0, o, 15, n2 >> 15);
                    }});
    struct Cfg {
        const char* name;
        uint32_t mA, mB;
        int K;
        int* kd;
    } cfgs[2] = {{"syc32_5", 0xF0F0F0F0u, 0x0F0F0F0Fu, 2, kd}, {"syc32_1", 0xFFFF0000u, 0x0000FFFFu, 1, kd1}};
    for (const Cfg& c : cfgs) {
        const bool bg = c.mB == 0xFFFFu;
        const size_t st = 8 * (size_t)c.K * ((size_t(1) << __builtin_popcount(c.mA & 0xFFFF)) +
                                             (bg ? 0 : (size_t(1) << __builtin_popcount(c.mB & 0xFFFF))));
        OBArgs ob{c.K, 16, A, L, B, L, c.mA, c.mB, total >> 16, c.kd, nullptr};
        pats.push_back({std::string("knit static ") + c.name, [=](double* o) {
                            OBArgs a = ob;
                            a.out = o;
                            if (bg)
                                hipLaunchKernelGGL(k_static<true>, dim3((unsigned)(cus * 64)), dim3(256), st, 0, a);
                            else
                                hipLaunchKernelGGL(k_static<false>, dim3((unsigned)(cus * 64)), dim3(256), st, 0, a);
                        }});
    }
    auto measure = [&](const Buf& b) {
        printf("%-34s %p", b.how.c_str(), (void*)b.p);
        for (auto& pt : pats) {
            pt.fn(b.p);
            CK(hipDeviceSynchronize());
            std::vector<float> ms;
            for (int r = 0; r < 3; ++r) {
                CK(hipEventRecord(s, 0));
                pt.fn(b.p);
                CK(hipEventRecord(e, 0));
                CK(hipEventSynchronize(e));
                float t = 0;
                CK(hipEventElapsedTime(&t, s, e));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            printf("  %7.3f", ms[1]);
        }
        printf("\n");
        fflush(stdout);
    };
    printf("%-34s %-14s", "allocation", "address");
    for (auto& pt : pats) printf("  %s |", pt.name.c_str());
    printf("\n");

    auto plain = [&]() -> Buf {
        double* p = nullptr;
        CK(hipMalloc(&p, bytes));
        return {"hipMalloc", p, [p] { (void)hipFree(p); }};
    };
    auto contig = [&]() -> Buf {
        double* p = nullptr;
        hipError_t err = hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocContiguous);
        if (err != hipSuccess) {
            printf("hipExtMallocWithFlags(contiguous): %s\n", hipGetErrorString(err));
            return {"", nullptr, [] {}};
        }
        return {"hipExtMallocWithFlags contiguous", p, [p] { (void)hipFree(p); }};
    };
    auto vmm = [&](size_t chunk, size_t align) -> Buf {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t gran = 0;
        CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
        void* va = nullptr;
        hipError_t err = hipMemAddressReserve(&va, bytes, align, nullptr, 0);
        if (err != hipSuccess) {
            printf("hipMemAddressReserve: %s\n", hipGetErrorString(err));
            return {"", nullptr, [] {}};
        }
        std::vector<hipMemGenericAllocationHandle_t> hs;
        for (size_t off = 0; off < bytes; off += chunk) {
            const size_t sz = std::min(chunk, bytes - off);
            hipMemGenericAllocationHandle_t h;
            err = hipMemCreate(&h, sz, &prop, 0);
            if (err != hipSuccess) {
                printf("hipMemCreate(%zu): %s\n", sz, hipGetErrorString(err));
                return {"", nullptr, [] {}};
            }
            CK(hipMemMap((char*)va + off, sz, 0, h, 0));
            hs.push_back(h);
        }
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        char nm[96];
        snprintf(nm, sizeof nm, "VMM chunk %zu MiB align %zu MiB (gran %zu KiB)", chunk >> 20, align >> 20, gran >> 10);
        return {nm, (double*)va, [va, hs, bytes] {
                    (void)hipMemUnmap(va, bytes);
                    for (auto h : hs) (void)hipMemRelease(h);
                    (void)hipMemAddressFree(va, bytes);
                }};
    };
    std::vector<Buf> held;
    auto run = [&](Buf b) {
        if (!b.p) return;
        measure(b);
        held.push_back(b);
    };
    run(plain());
    run(plain());
    run(plain());
    run(contig());
    run(contig());
    for (auto& b : held) b.release();
    held.clear();
    CK(hipDeviceSynchronize());
    printf("-- all freed\n");
    run(vmm(bytes, size_t(1) << 30));
    run(vmm(size_t(1) << 30, size_t(1) << 30));
    run(vmm(size_t(2) << 20, size_t(2) << 20));
    run(contig());
    run(plain());
    for (auto& b : held) b.release();
    return 0;
}
