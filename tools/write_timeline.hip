// write_timeline.hip — where a write's time goes: the blocked knit's store pattern (K = 2, 2^16-output
// tasks of 512 KiB, operands staged in LDS, 256 threads, one 16-B store per lane per 4-KiB iteration)
// writing n = 2^32 or a 2^29 slice, every workgroup recording the wall clock (100 MHz) at the start
// and end of each task. Prints per-launch duration and the write rate in 20-us bins of the launch, so
// a fixed start-up stall (translation misses of a cold front) or a drain tail shows where it sits.
//   hipcc --offload-arch=gfx950 -O3 tools/write_timeline.hip -o tools/write_timeline
//   ./write_timeline [log2_n ...]   (default: 32 29)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));        \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int TB = 16, K = 2, NA = 256, NB = 256;

__device__ __forceinline__ uint32_t pext32(uint32_t x, uint32_t m) {
    uint32_t r = 0;
    for (uint32_t bb = 1; m; bb <<= 1, m &= m - 1)
        if (x & m & -m) r |= bb;
    return r;
}

// maskA = odd bits, maskB = even bits (the syc 32 5 layout interleaves the two fragments' clbits)
__global__ __launch_bounds__(256) void write_kernel(const double* __restrict__ A, const double* __restrict__ B,
                                                    double* __restrict__ out, int64_t n_tasks, int64_t spread,
                                                    unsigned long long* __restrict__ stamps, int per_wg) {
    __shared__ double sA[K * NA], sB[K * NB];
    __shared__ uint32_t tab[2][2][256];  // pext of bytes 0 / 1 of a task offset, per side (as the knit)
    const uint32_t mA = 0xAAAAAAAAu, mB = 0x55555555u, low = (1u << TB) - 1;
    for (int i = threadIdx.x; i < 512; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), mA & low);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), mB & low);
    }
    __syncthreads();
    const uint32_t r0 = tab[0][0][(2 * threadIdx.x) & 255], c0 = tab[1][0][(2 * threadIdx.x) & 255];
    const int64_t per_part = n_tasks / spread;
    int slot = 0;
    for (int64_t i = blockIdx.x; i < n_tasks; i += gridDim.x, ++slot) {
        const unsigned long long t0 = wall_clock64();
        const int64_t t = (i % spread) * per_part + i / spread;
        const uint32_t base = (uint32_t)(t << TB);
        const uint32_t ah = pext32(base, mA), bh = pext32(base, mB);
        __syncthreads();
        for (int j = threadIdx.x; j < K * NA; j += 256) sA[j] = A[(j / NA) * 65536 + ah + j % NA];
        for (int j = threadIdx.x; j < K * NB; j += 256) sB[j] = B[(j / NB) * 65536 + bh + j % NB];
        __syncthreads();
        double* o = out + (int64_t)t * (1 << TB);
#pragma unroll 4
        for (int it = 0; it < (1 << TB) / 512; ++it) {
            const uint32_t hi = (uint32_t)(2 * it + (threadIdx.x >> 7));
            const uint32_t row = r0 + tab[0][1][hi], col = c0 + tab[1][1][hi];
            double2 acc = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double av = sA[k * NA + row];
                const double2 bv = *reinterpret_cast<const double2*>(sB + k * NB + col);
                acc.x = fma(av, bv.x, acc.x);
                acc.y = fma(av, bv.y, acc.y);
            }
            *reinterpret_cast<double2*>(o + 512 * it + 2 * threadIdx.x) = acc;
        }
        if (threadIdx.x == 0 && slot < per_wg) {
            stamps[2 * ((int64_t)blockIdx.x * per_wg + slot)] = t0;
            stamps[2 * ((int64_t)blockIdx.x * per_wg + slot) + 1] = wall_clock64();
        }
    }
}

int main(int argc, char** argv) {
    std::vector<int> sizes;
    for (int i = 1; i < argc; ++i) sizes.push_back(atoi(argv[i]));
    if (sizes.empty()) sizes = {32, 29};
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double *A, *B, *out;
    CK(hipMalloc(&A, K * 65536 * 8));
    CK(hipMalloc(&B, K * 65536 * 8));
    CK(hipMemset(A, 0, K * 65536 * 8));
    CK(hipMemset(B, 0, K * 65536 * 8));
    CK(hipMalloc(&out, (size_t(1) << 32) * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int lg : sizes) {
        const int64_t n_tasks = (int64_t(1) << lg) >> TB;
        for (int wgpc : {64, 0}) {
            const int64_t G0 = wgpc ? (int64_t)cus * wgpc : n_tasks;
            const int64_t G = n_tasks < G0 ? n_tasks : G0;
            const int per_wg = (int)((n_tasks + G - 1) / G);
            const int64_t spread = (n_tasks >= 4 * G && n_tasks % 8 == 0) ? 8 : 1;
            unsigned long long* st;
            CK(hipMalloc(&st, (size_t)G * per_wg * 16));
            CK(hipMemset(st, 0, (size_t)G * per_wg * 16));
            float ms = 0;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(e0));
                write_kernel<<<dim3((unsigned)G), dim3(256)>>>(A, B, out, n_tasks, spread, st, per_wg);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
            }
            std::vector<unsigned long long> h((size_t)G * per_wg * 2);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long lo = ~0ull, hi = 0;
            for (size_t i = 0; i < h.size(); i += 2)
                if (h[i]) {
                    lo = h[i] < lo ? h[i] : lo;
                    hi = h[i + 1] > hi ? h[i + 1] : hi;
                }
            // 100 MHz clock: 10 ns ticks; 20-us bins, each task's 512 KiB spread evenly over its span
            const double bin = 2000.0;
            const int nb = (int)((hi - lo) / bin) + 1;
            std::vector<double> bytes(nb, 0.0);
            std::vector<int> starts(nb, 0), ends(nb, 0);
            for (size_t i = 0; i < h.size(); i += 2) {
                if (!h[i]) continue;
                const double s = (double)(h[i] - lo), e = (double)(h[i + 1] - lo), span = e - s > 1 ? e - s : 1;
                starts[(int)(s / bin)]++;
                ends[(int)(e / bin)]++;
                for (int b = (int)(s / bin); b <= (int)(e / bin) && b < nb; ++b) {
                    const double a0 = b * bin > s ? b * bin : s, a1 = (b + 1) * bin < e ? (b + 1) * bin : e;
                    if (a1 > a0) bytes[b] += 524288.0 * (a1 - a0) / span;
                }
            }
            printf("{\"log2_n\": %d, \"grid\": %lld, \"tasks_per_wg\": %d, \"spread\": %lld, \"event_ms\": %.4f, "
                   "\"stamp_span_ms\": %.4f, \"TBps_event\": %.3f, \"bins_us\": 20, \"TBps_per_bin\": [",
                   lg, (long long)G, per_wg, (long long)spread, ms, (hi - lo) * 1e-5,
                   (double)(int64_t(1) << lg) * 8 / (ms * 1e-3) / 1e12);
            for (int b = 0; b < nb; ++b) printf("%s%.2f", b ? ", " : "", bytes[b] / (bin * 1e-8) / 1e12);
            printf("], \"task_starts_per_bin\": [");
            for (int b = 0; b < nb; ++b) printf("%s%d", b ? ", " : "", starts[b]);
            printf("], \"task_ends_per_bin\": [");
            for (int b = 0; b < nb; ++b) printf("%s%d", b ? ", " : "", ends[b]);
            printf("]}\n");
            fflush(stdout);
            CK(hipFree(st));
        }
    }
    return 0;
}
