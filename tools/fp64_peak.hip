// FP64 issue-rate probe for gfx950: v_mfma_f64_16x16x4_f64 alone, v_fma_f64 alone, and both at
// once (MFMA waves and VALU waves sharing a CU; and one wave interleaving both). Decides whether
// the knit contraction can split work between the matrix core and the vector FP64 pipe.
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_peak.hip -o tools/fp64_peak && ./tools/fp64_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4_t __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

// inline asm keeps the accumulators in place (the builtin in a loop made the compiler copy
// them between AGPRs and VGPRs every iteration)
__device__ __forceinline__ void mfma(d4_t& acc, double a, double b) {
    asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma_loop(double* out, int iters) {
    d4_t acc[8];
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (d4_t){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) mfma(acc[i], a, b);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ void fma_loop(double* out, int iters) {
    double x[16];
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1e-9;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = i * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = __builtin_fma(x[i], a, b);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) { mfma_loop(out, iters); }
__global__ __launch_bounds__(256) void k_fma(double* out, int iters) { fma_loop(out, iters); }
// waves 0..3 MFMA, waves 4..7 VALU
__global__ __launch_bounds__(512) void k_split(double* out, int mi, int fi) {
    if ((threadIdx.x >> 6) < 4) mfma_loop(out, mi);
    else fma_loop(out, fi);
}
// one wave interleaves: 8 MFMA then 8x16 FMA per iteration
__global__ __launch_bounds__(256) void k_mix(double* out, int iters) {
    d4_t acc[8];
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    double x[16];
    const double fa = 1.0 + threadIdx.x * 1e-9, fb = 1e-9;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = i * 1e-3;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (d4_t){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            mfma(acc[i], a, b);
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = __builtin_fma(x[j], fa, fb);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    printf("device %s, %d CUs, clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
    double* out;
    hipMalloc(&out, (size_t)cus * 8 * 512 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch, double flops) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.3f ms  %7.2f TF/s\n", name, ms, flops / (ms * 1e-3) / 1e12);
    };
    const double mfma_flop_wave = 2.0 * 16 * 16 * 4 * 8 * ITERS;  // per wave
    const double fma_flop_wave = 2.0 * 64 * 16 * 8 * ITERS;
    for (int wpc : {1, 2}) {  // 256-thread workgroups per CU
        const int grid = cus * wpc;
        char nm[64];
        snprintf(nm, sizeof nm, "mfma f64 only (%d WG/CU x 4 waves)", wpc);
        run(nm, [&] { k_mfma<<<grid, 256>>>(out, ITERS); }, mfma_flop_wave * grid * 4);
        snprintf(nm, sizeof nm, "fma f64 only (%d WG/CU x 4 waves)", wpc);
        run(nm, [&] { k_fma<<<grid, 256>>>(out, ITERS); }, fma_flop_wave * grid * 4);
        snprintf(nm, sizeof nm, "one wave interleaved (%d WG/CU)", wpc);
        run(nm, [&] { k_mix<<<grid, 256>>>(out, ITERS); },
            (mfma_flop_wave + fma_flop_wave) * grid * 4);
    }
    for (int fi : {ITERS / 4, ITERS / 2, ITERS}) {
        const int grid = cus;
        char nm[64];
        snprintf(nm, sizeof nm, "split waves mfma|fma (fma iters %d)", fi);
        run(nm, [&] { k_split<<<grid, 512>>>(out, ITERS, fi); },
            (mfma_flop_wave + fma_flop_wave * fi / ITERS) * grid * 4);
    }
    hipFree(out);
    return 0;
}
