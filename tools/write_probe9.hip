// write_probe9.hip — which physical memory is "slow"? (round 4)
// write_probe8 with 8 x 34 GB allocations on a fresh box: the first six take the static 512-KiB-task
// write at 4.9-5.0 ms, the last two at 5.9-6.0, while one 4-KiB chunk per workgroup writes 4.8-5.0
// into all eight. Here the device is filled with NB x 1 GiB allocations (allocation order ~ physical
// order on a fresh device) and each is written by both orders: a map of the slow regions.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe9 tools/write_probe9.hip && tools/write_probe9 [NB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef double d2_t __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void f_one16(double* __restrict__ out) {
    reinterpret_cast<d2_t*>(out)[(int64_t)blockIdx.x * 256 + threadIdx.x] = (d2_t){1.0, 1.0};
}
// one 512-KiB block per workgroup, 2048 workgroups: every resident workgroup streams its own block
__global__ __launch_bounds__(256) void f_block(double* __restrict__ out) {
    d2_t* o = reinterpret_cast<d2_t*>(out) + ((int64_t)blockIdx.x << 15);
#pragma unroll 4
    for (int it = 0; it < 128; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
}

int main(int argc, char** argv) {
    const int NB = argc > 1 ? atoi(argv[1]) : 260;
    const size_t bytes = size_t(1) << 30;
    std::vector<double*> bufs;
    for (int b = 0; b < NB; ++b) {
        double* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) break;
        bufs.push_back(p);
    }
    printf("allocated %zu x 1 GiB\n", bufs.size());
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    auto timed = [&](auto launch) {
        launch();
        std::vector<float> ms;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(s, 0));
            launch();
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            float t = 0;
            CK(hipEventElapsedTime(&t, s, e));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        return ms[2];
    };
    printf("buf  address          one16_us  block_us  GB/s_one16 GB/s_block\n");
    for (size_t b = 0; b < bufs.size(); ++b) {
        double* p = bufs[b];
        const float t1 = timed([&] { hipLaunchKernelGGL(f_one16, dim3(bytes / 4096), dim3(256), 0, 0, p); });
        const float t2 = timed([&] { hipLaunchKernelGGL(f_block, dim3(bytes >> 19), dim3(256), 0, 0, p); });
        printf("%3zu  %p  %8.1f  %8.1f  %8.0f  %8.0f\n", b, (void*)p, t1 * 1e3, t2 * 1e3, bytes / t1 / 1e6,
               bytes / t2 / 1e6);
    }
    for (double* p : bufs) CK(hipFree(p));
    return 0;
}
