// write_probe12.hip — is the slow write a property of single 1-GiB physical chunks? (round 4)
// Creates M 1-GiB chunks (hipMemCreate), times a store-only fill of each chunk mapped alone, then maps
// 32-GiB buffers from the 32 fastest and from the 32 slowest chunks and times the static 512-KiB-task
// fill of each (the knit's store pattern).
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe12 tools/write_probe12.hip && tools/write_probe12 [M]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <numeric>
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

__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int64_t nblocks) {
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << 15);
#pragma unroll 4
        for (int it = 0; it < 128; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 96;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t G = size_t(1) << 30;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    std::vector<hipMemGenericAllocationHandle_t> hs(M);
    for (int i = 0; i < M; ++i) CK(hipMemCreate(&hs[i], G, &prop, 0));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    auto time_fill = [&](double* p, size_t bytes, int reps) {
        const int64_t nb = (int64_t)(bytes >> 19);
        std::vector<float> ms;
        for (int r = 0; r <= reps; ++r) {
            CK(hipEventRecord(s, 0));
            hipLaunchKernelGGL(f_block_static, dim3(cus * 64), dim3(256), 0, 0, p, nb);
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            float t = 0;
            CK(hipEventElapsedTime(&t, s, e));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        return ms[ms.size() / 2];
    };
    // every chunk alone
    std::vector<float> t1(M);
    for (int i = 0; i < M; ++i) {
        void* va = nullptr;
        CK(hipMemAddressReserve(&va, G, G, nullptr, 0));
        CK(hipMemMap(va, G, 0, hs[i], 0));
        CK(hipMemSetAccess(va, G, &acc, 1));
        t1[i] = time_fill((double*)va, G, 5);
        CK(hipDeviceSynchronize());
        CK(hipMemUnmap(va, G));
        CK(hipMemAddressFree(va, G));
    }
    std::vector<int> order(M);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return t1[a] < t1[b]; });
    printf("per-chunk 1-GiB fill (ms), sorted:");
    for (int i = 0; i < M; ++i) printf(" %.4f", t1[order[i]]);
    printf("\n");
    // 32-GiB buffers from the fastest / slowest / creation-order chunks
    const char* names[3] = {"fastest 32", "slowest 32", "first 32"};
    for (int which = 0; which < 3; ++which) {
        void* va = nullptr;
        const size_t bytes = 32 * G;
        CK(hipMemAddressReserve(&va, bytes, G, nullptr, 0));
        for (int j = 0; j < 32; ++j) {
            const int idx = which == 0 ? order[j] : which == 1 ? order[M - 1 - j] : j;
            CK(hipMemMap((char*)va + j * G, G, 0, hs[idx], 0));
        }
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        printf("%s chunks: 32-GiB static fill %.3f ms\n", names[which], time_fill((double*)va, bytes, 3));
        fflush(stdout);
        CK(hipDeviceSynchronize());
        CK(hipMemUnmap(va, bytes));
        CK(hipMemAddressFree(va, bytes));
    }
    for (auto h : hs) CK(hipMemRelease(h));
    return 0;
}
