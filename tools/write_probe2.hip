// write_probe2.hip — which write orders are fast into EVERY 34 GB allocation? (round 4)
// The blocked knit writes 4.8 ms into some allocations and 5.8 ms into others. Here
// NB buffers of 2^32 fp64 are allocated at once and every pattern is timed into each of them:
//   store-only: one workgroup per 4-KiB chunk (non-persistent), contiguous blocks per workgroup,
//   grid-stride at two grid sizes, the knit's static persistent 512-KiB-task order, and ticketed
//   persistent orders (each workgroup takes the next unit from a device counter, so the units in
//   flight stay a contiguous window however the workgroups drift);
//   knit: the shipped static blocked knit and a ticketed blocked knit on synthetic K = 2 operands.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe2 tools/write_probe2.hip && tools/write_probe2 [NB]
#include <hip/hip_runtime.h>

#include <algorithm>
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
// one 4-KiB chunk per workgroup, chunks permuted inside each 2-MiB page (bit-reversed 9-bit index)
__global__ __launch_bounds__(256) void f_one16_perm(double* __restrict__ out, int64_t n2) {
    const uint32_t b = blockIdx.x;
    const uint32_t c = (b & ~511u) | (__builtin_bitreverse32(b & 511u) >> 23);
    const int64_t i = (int64_t)c * 256 + threadIdx.x;
    if (i < n2) reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}
__global__ __launch_bounds__(256) void f_stride(double* __restrict__ out, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}
// non-persistent: workgroup b writes the contiguous block b of 2^bb 16-B vectors
__global__ __launch_bounds__(256) void f_block(double* __restrict__ out, int bb) {
    d2_t* o = reinterpret_cast<d2_t*>(out) + ((int64_t)blockIdx.x << bb);
    const int iters = 1 << (bb - 8);
#pragma unroll 4
    for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
}
// persistent static: workgroup b writes blocks b, b + G, b + 2G, ... (the shipped knit's task order)
__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int bb, int64_t nblocks) {
    const int iters = 1 << (bb - 8);
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}
// persistent ticketed: each workgroup takes the next block of 2^bb vectors from *ctr (the next
// ticket is fetched while the current block is written); xcd != 0: one counter per XCD, XCD x
// writes blocks 8 t + x
__global__ __launch_bounds__(256) void f_block_ticket(double* __restrict__ out, int bb, int64_t nblocks,
                                                      unsigned* __restrict__ ctr, int xcd) {
    __shared__ unsigned tk[2];
    const int iters = 1 << (bb - 8);
    const int x = xcd ? (__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7) : 0;
    unsigned* c = ctr + x;
    const int64_t nb = xcd ? nblocks / 8 : nblocks;
    if (threadIdx.x == 0) tk[0] = atomicAdd(c, 1u);
    __syncthreads();
    int s = 0;
    unsigned u = tk[0];
    while ((int64_t)u < nb) {
        unsigned nxt = 0;
        if (threadIdx.x == 0) nxt = atomicAdd(c, 1u);
        const int64_t blk = xcd ? 8 * (int64_t)u + x : (int64_t)u;
        d2_t* o = reinterpret_cast<d2_t*>(out) + (blk << bb);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
        if (threadIdx.x == 0) tk[s ^ 1] = nxt;
        __syncthreads();
        s ^= 1;
        u = tk[s];
    }
}

__device__ __forceinline__ uint32_t pext32(uint32_t x, uint32_t mask) {
    uint32_t r = 0, bit = 1;
    for (; mask; mask &= mask - 1, bit <<= 1)
        if (x & mask & (~mask + 1)) r |= bit;
    return r;
}

// synthetic knit out[o] = sum_k A[k][pext(o, mA)] B[k][pext(o, mB)] (K = 2), tasks of 2^TB outputs with
// A / B staged in LDS; ticket = nullptr: static order (task b + j G, the shipped kernel), else ticketed
struct KArgs {
    int K, TB;
    const double* A;
    int64_t lda;
    const double* B;
    int64_t ldb;
    uint32_t maskA, maskB;
    int64_t ntasks;
    double* out;
    unsigned* ticket;
};
__global__ __launch_bounds__(256) void k_blocked(KArgs a) {
    __shared__ uint32_t tab[2][2][256];
    __shared__ unsigned tk[2];
    extern __shared__ double stage[];
    const int K = a.K;
    const uint32_t low = (1u << a.TB) - 1u;
    const uint32_t mAl = a.maskA & low, mBl = a.maskB & low;
    const int na = 1 << __builtin_popcount(mAl), nb = 1 << __builtin_popcount(mBl);
    double* sA = stage;
    double* sB = stage + (int64_t)K * na;
    for (int i = threadIdx.x; i < 512; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), mAl);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), mBl);
    }
    if (a.ticket && threadIdx.x == 0) tk[0] = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const uint32_t r0 = tab[0][0][(2 * threadIdx.x) & 255], c0 = tab[1][0][(2 * threadIdx.x) & 255];
    const int iters = (1 << a.TB) / 512;
    int s = 0;
    int64_t t = a.ticket ? (int64_t)tk[0] : (int64_t)blockIdx.x;
    while (t < a.ntasks) {
        unsigned nxt = 0;
        if (a.ticket && threadIdx.x == 0) nxt = atomicAdd(a.ticket, 1u);
        const uint32_t base = (uint32_t)(t << a.TB);
        const uint32_t ah = pext32(base, a.maskA), bh = pext32(base, a.maskB);
        for (int i = threadIdx.x; i < K * na; i += 256) {
            const int k = i / na;
            sA[i] = a.A[k * a.lda + ah + (i - k * na)];
        }
        for (int i = threadIdx.x; i < K * nb; i += 256) {
            const int k = i / nb;
            sB[i] = a.B[k * a.ldb + bh + (i - k * nb)];
        }
        __syncthreads();
        double* o = a.out + (int64_t)base;
#pragma unroll 4
        for (int it = 0; it < iters; ++it) {
            const uint32_t hi = (uint32_t)(2 * it + (threadIdx.x >> 7));
            const uint32_t row = r0 + tab[0][1][hi & 255], col = c0 + tab[1][1][hi & 255];
            d2_t acc = {0.0, 0.0};
            for (int k = 0; k < 2; ++k) {
                const double av = sA[k * na + row];
                const d2_t bv = *reinterpret_cast<const d2_t*>(sB + k * nb + col);
                acc.x = fma(av, bv.x, acc.x);
                acc.y = fma(av, bv.y, acc.y);
            }
            *reinterpret_cast<d2_t*>(o + 512 * it + 2 * threadIdx.x) = acc;
        }
        if (a.ticket && threadIdx.x == 0) tk[s ^ 1] = nxt;
        __syncthreads();  // stage readers done; ticket visible
        if (a.ticket) {
            s ^= 1;
            t = tk[s];
        } else {
            t += gridDim.x;
        }
    }
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 4;
    const int64_t total = int64_t(1) << 32;  // doubles per buffer
    const int64_t n2 = total / 2;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<double*> bufs;
    for (int b = 0; b < NB; ++b) {
        double* p = nullptr;
        CK(hipMalloc(&p, total * 8));
        bufs.push_back(p);
        printf("buffer %d at %p\n", b, (void*)p);
    }
    unsigned* ctr = nullptr;
    CK(hipMalloc(&ctr, 64 * sizeof(unsigned)));
    // synthetic operands: K = 2 rows of 2^16 per side
    double *A = nullptr, *B = nullptr;
    CK(hipMalloc(&A, 2 * 65536 * 8));
    CK(hipMalloc(&B, 2 * 65536 * 8));
    CK(hipMemset(A, 0, 2 * 65536 * 8));
    CK(hipMemset(B, 0, 2 * 65536 * 8));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    int occ_block = 0, occ_knit = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_block, f_block_ticket, 256, 0));
    const size_t kst = 8 * 2 * (256 + 256);
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_knit, k_blocked, 256, kst));
    printf("cus %d, resident workgroups per CU: ticket fill %d, knit %d\n", cus, occ_block, occ_knit);
    fflush(stdout);

    struct Pat {
        std::string name;
        std::function<void(double*)> fn;
    };
    std::vector<Pat> pats;
    pats.push_back({"memset", [&](double* o) { (void)hipMemsetAsync(o, 0, total * 8, 0); }});
    pats.push_back({"one16 (4 KiB/wg, non-persistent)",
                    [&](double* o) { hipLaunchKernelGGL(f_one16, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, o, n2); }});
    pats.push_back({"one16 permuted in 2 MiB",
                    [&](double* o) { hipLaunchKernelGGL(f_one16_perm, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, o, n2); }});
    for (int wpc : {8, 64}) {
        pats.push_back({"grid-stride " + std::to_string(wpc) + " wg/CU", [&, wpc](double* o) {
                            hipLaunchKernelGGL(f_stride, dim3((unsigned)(cus * wpc)), dim3(256), 0, 0, o, n2);
                        }});
    }
    for (int bb : {9, 11, 15}) {
        pats.push_back({"block " + std::to_string((16 << bb) / 1024) + " KiB non-persistent", [&, bb](double* o) {
                            hipLaunchKernelGGL(f_block, dim3((unsigned)(n2 >> bb)), dim3(256), 0, 0, o, bb);
                        }});
    }
    for (int wpc : {8, 64}) {
        pats.push_back({"block 512 KiB static " + std::to_string(wpc) + " wg/CU", [&, wpc](double* o) {
                            hipLaunchKernelGGL(f_block_static, dim3((unsigned)(cus * wpc)), dim3(256), 0, 0, o, 15,
                                               n2 >> 15);
                        }});
    }
    for (int xcd : {0, 1})
        for (int bb : {8, 10, 12, 15}) {
            pats.push_back({"ticket " + std::string(xcd ? "per-XCD " : "") + std::to_string((16 << bb) / 1024) + " KiB",
                            [&, bb, xcd](double* o) {
                                (void)hipMemsetAsync(ctr, 0, 64 * sizeof(unsigned), 0);
                                hipLaunchKernelGGL(f_block_ticket, dim3((unsigned)(cus * occ_block)), dim3(256), 0, 0,
                                                   o, bb, n2 >> bb, ctr, xcd);
                            }});
        }
    const uint32_t mA = 0xF0F0F0F0u, mB = 0x0F0F0F0Fu;
    for (int tb : {16, 14, 13}) {
        for (int tick : {0, 1}) {
            if (!tick && tb != 16) continue;
            const uint32_t low = (1u << tb) - 1;
            const size_t st = 8 * 2 * ((size_t(1) << __builtin_popcount(mA & low)) + (size_t(1) << __builtin_popcount(mB & low)));
            pats.push_back({std::string("knit ") + (tick ? "ticket" : "static 64 wg/CU") + " TB " + std::to_string(tb),
                            [&, tb, tick, st](double* o) {
                                KArgs a{2, tb, A, 65536, B, 65536, mA, mB, total >> tb, o, tick ? ctr : nullptr};
                                if (tick) (void)hipMemsetAsync(ctr, 0, 64 * sizeof(unsigned), 0);
                                const unsigned g = tick ? (unsigned)(cus * occ_knit) : (unsigned)(cus * 64);
                                hipLaunchKernelGGL(k_blocked, dim3(g), dim3(256), st, 0, a);
                            }});
        }
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
