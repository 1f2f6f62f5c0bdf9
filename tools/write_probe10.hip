// write_probe10.hip — does the slow write follow the physical memory or the mapping? (round 4)
// The device is filled with 1-GiB physical allocations (hipMemCreate); 34-GiB buffers are mapped from
// them in creation order (buffer k = handles 34 k .. 34 k + 33) and interleaved (buffer k = handles
// 8 j + k), and the static 512-KiB-task order and the one-chunk-per-workgroup order are timed into each.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe10 tools/write_probe10.hip && tools/write_probe10
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
__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int64_t nblocks) {
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << 15);
#pragma unroll 4
        for (int it = 0; it < 128; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t G = size_t(1) << 30, NPER = 32;  // 32 GiB buffers (2^32 doubles)
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    std::vector<hipMemGenericAllocationHandle_t> hs;
    for (int i = 0; i < 280; ++i) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, G, &prop, 0) != hipSuccess) break;
        hs.push_back(h);
    }
    printf("created %zu x 1 GiB physical allocations\n", hs.size());
    const size_t nbuf = hs.size() / NPER;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    auto timed = [&](auto launch) {
        launch();
        std::vector<float> ms;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(s, 0));
            launch();
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            float t = 0;
            CK(hipEventElapsedTime(&t, s, e));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        return ms[1];
    };
    const size_t bytes = NPER * G;
    const int64_t n2 = bytes / 16;
    for (int layout = 0; layout < 3; ++layout) {
        for (size_t k = 0; k < nbuf; ++k) {
            void* va = nullptr;
            CK(hipMemAddressReserve(&va, bytes, G, nullptr, 0));
            for (size_t j = 0; j < NPER; ++j) {
                size_t idx = layout == 0 ? k * NPER + j : layout == 1 ? j * nbuf + k : (k * NPER + (j * 7) % NPER);
                CK(hipMemMap((char*)va + j * G, G, 0, hs[idx], 0));
            }
            CK(hipMemSetAccess(va, bytes, &acc, 1));
            double* p = (double*)va;
            const float t1 = timed([&] { hipLaunchKernelGGL(f_one16, dim3(n2 / 256), dim3(256), 0, 0, p); });
            const float t2 = timed([&] {
                hipLaunchKernelGGL(f_block_static, dim3(cus * 64), dim3(256), 0, 0, p, (int64_t)(n2 >> 15));
            });
            printf("%s buffer %zu: one16 %.3f ms  static %.3f ms\n",
                   layout == 0 ? "in-order   " : layout == 1 ? "interleaved" : "permuted   ", k, t1, t2);
            fflush(stdout);
            CK(hipDeviceSynchronize());
            CK(hipMemUnmap(va, bytes));
            CK(hipMemAddressFree(va, bytes));
        }
    }
    for (auto h : hs) CK(hipMemRelease(h));
    return 0;
}
