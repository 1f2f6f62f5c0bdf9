// fill_probe.hip — which store structure reaches the HBM write rate on this box? 2^32 fp64 (34.36 GB)
// written by: hipMemsetAsync; one thread per 16 B (non-persistent grid, one launch / 2^28-entry chunks);
// one thread per 32 B (two 16-B stores); a grid-stride fill at 8 / 64 workgroups per CU. Median of 5.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fill_probe tools/fill_probe.hip && tools/fill_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <functional>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

typedef double d2_t __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void f_one16(double* __restrict__ out, int64_t n2) {  // n2: 16-B vectors
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n2) reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}
__global__ __launch_bounds__(256) void f_one32(double* __restrict__ out, int64_t n4) {  // n4: 32-B vectors
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) {
        reinterpret_cast<d2_t*>(out)[2 * i] = (d2_t){(double)i, 1.0};
        reinterpret_cast<d2_t*>(out)[2 * i + 1] = (d2_t){(double)i, 2.0};
    }
}
__global__ __launch_bounds__(256) void f_stride(double* __restrict__ out, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256)
        reinterpret_cast<d2_t*>(out)[i] = (d2_t){(double)i, 1.0};
}
// a workgroup writes one contiguous block of 2^bb 16-B vectors (bb >= 8), 256 vectors per iteration
__global__ __launch_bounds__(256) void f_block(double* __restrict__ out, int bb) {
    d2_t* o = reinterpret_cast<d2_t*>(out) + ((int64_t)blockIdx.x << bb);
    const int iters = 1 << (bb - 8);
#pragma unroll 4
    for (int it = 0; it < iters; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
}

// XCD-aware blocks: workgroup b runs on XCD b % 8 (round-robin dispatch) and writes only the chunks c
// (2^cb 16-B vectors each) with c % 8 == b % 8: m = 2^(bb - cb) of them, 8 chunks apart
__global__ __launch_bounds__(256) void f_block_xcd(double* __restrict__ out, int bb, int cb) {
    const int x = blockIdx.x & 7;
    const int64_t i = blockIdx.x >> 3;
    const int m = 1 << (bb - cb), per = 1 << (cb - 8);
    d2_t* o = reinterpret_cast<d2_t*>(out);
    for (int j = 0; j < m; ++j) {
        const int64_t c = 8 * (i * m + j) + x;
#pragma unroll 4
        for (int it = 0; it < per; ++it) o[(c << cb) + 256 * it + threadIdx.x] = (d2_t){(double)j, 1.0};
    }
}

// the XCD (XCC_ID hardware register, bits 3:0) each workgroup of a one16-shaped launch ran on
__global__ __launch_bounds__(256) void f_xcc_map(int* __restrict__ xcc_of) {
    if (threadIdx.x == 0) xcc_of[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15;
}
// one16 order, but a workgroup writes the chunks of its own XCD: the k-th workgroup to start on XCD x
// (per-XCD counter) writes chunk 8 k + x
__global__ __launch_bounds__(256) void f_one16_xcc(double* __restrict__ out, int* __restrict__ ctr) {
    __shared__ int slot;
    const int x = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7;
    if (threadIdx.x == 0) slot = atomicAdd(&ctr[x], 1);
    __syncthreads();
    const int64_t c = 8 * (int64_t)slot + x;
    reinterpret_cast<d2_t*>(out)[c * 256 + threadIdx.x] = (d2_t){(double)c, 1.0};
}

int main() {
    const int64_t total = int64_t(1) << 32;  // doubles
    double* out = nullptr;
    CK(hipMalloc(&out, total * 8));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    auto run = [&](const char* name, std::function<void()> fn) -> int {
        fn();
        CK(hipDeviceSynchronize());
        std::vector<float> ms;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(s, 0));
            fn();
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            float t = 0;
            CK(hipEventElapsedTime(&t, s, e));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-34s median %.3f ms  min %.3f ms  = %.2f TB/s\n", name, ms[2], ms[0], total * 8.0 / ms[2] / 1e9);
        fflush(stdout);
        return 0;
    };
    const int64_t n2 = total / 2, n4 = total / 4;
    run("hipMemsetAsync", [&] { (void)hipMemsetAsync(out, 0, total * 8, 0); });
    run("one thread / 16 B, one launch", [&] { hipLaunchKernelGGL(f_one16, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, out, n2); });
    run("one thread / 32 B, one launch", [&] { hipLaunchKernelGGL(f_one32, dim3((unsigned)(n4 / 256)), dim3(256), 0, 0, out, n4); });
    run("one thread / 32 B, 16 x 2^28 chunks", [&] {
        const int64_t c4 = n4 / 16;
        for (int c = 0; c < 16; ++c)
            hipLaunchKernelGGL(f_one32, dim3((unsigned)(c4 / 256)), dim3(256), 0, 0, out + (int64_t)c * 4 * c4, c4);
    });
    for (int wpc : {8, 64})
        for (int dummy = 0; dummy < 1; ++dummy) {
            char nm[64];
            snprintf(nm, sizeof nm, "grid-stride 16 B, %d wg/CU", wpc);
            run(nm, [&] { hipLaunchKernelGGL(f_stride, dim3((unsigned)(cus * wpc)), dim3(256), 0, 0, out, n2); });
        }
    for (int bb : {9, 11, 13, 15}) {  // 8 KiB .. 512 KiB per workgroup
        char nm[64];
        snprintf(nm, sizeof nm, "block of %lld KiB per workgroup", (long long)(16ll << bb) / 1024);
        run(nm, [&] { hipLaunchKernelGGL(f_block, dim3((unsigned)(n2 >> bb)), dim3(256), 0, 0, out, bb); });
    }
    for (int cb : {7, 8, 9, 10})
        for (int bb : {11, 15}) {
            if (cb < 8 && bb < 11) continue;
            char nm[64];
            snprintf(nm, sizeof nm, "xcd blocks %lld KiB, chunk %lld B", (long long)(16ll << bb) / 1024, 16ll << cb);
            if (cb < 8) continue;  // chunk below one 256-thread iteration: not expressible here
            run(nm, [&] { hipLaunchKernelGGL(f_block_xcd, dim3((unsigned)(n2 >> bb)), dim3(256), 0, 0, out, bb, cb); });
        }
    {
        const int nb = 4096;
        int* d = nullptr;
        CK(hipMalloc(&d, nb * sizeof(int)));
        hipLaunchKernelGGL(f_xcc_map, dim3(nb), dim3(256), 0, 0, d);
        std::vector<int> h(nb);
        CK(hipMemcpy(h.data(), d, nb * sizeof(int), hipMemcpyDeviceToHost));
        int rr = 0;
        for (int b = 0; b < nb; ++b) rr += (h[b] == b % 8);
        printf("xcc map: %d of %d workgroups on XCD blockIdx %% 8; first 16:", rr, nb);
        for (int b = 0; b < 16; ++b) printf(" %d", h[b]);
        printf("\n");
        CK(hipFree(d));
        int* ctr = nullptr;
        CK(hipMalloc(&ctr, 8 * sizeof(int)));
        run("one16, chunk = 8 k + own XCD", [&] {
            (void)hipMemsetAsync(ctr, 0, 8 * sizeof(int), 0);
            hipLaunchKernelGGL(f_one16_xcc, dim3((unsigned)(n2 / 256)), dim3(256), 0, 0, out, ctr);
        });
        CK(hipFree(ctr));
    }
    CK(hipFree(out));
    return 0;
}
