// write_probe13.hip — a recipe for 32-GiB mappings that write fast every time? (round 4)
// write_probe11: 32-GiB buffers mapped straight from fresh 1-GiB chunks write at 4.8-5.9 ms, by buffer;
// write_probe12: buffers composed from chunks that had each been mapped alone (1-GiB range) and written
// first were all fast (4.93-4.94). Per buffer here: 32 fresh chunks, then
//   mode 0: mapped straight into the 32-GiB range (qk_out_alloc),
//   mode 1: each chunk first mapped alone in its own 1-GiB range, filled, unmapped; then composed,
//   mode 2: as 1 without the fill (map / unmap only),
//   mode 3: mapped straight into the 32-GiB range, then every chunk filled once before timing.
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe13 tools/write_probe13.hip && tools/write_probe13 MODE [NBUF]
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

__global__ __launch_bounds__(256) void f_block_static(double* __restrict__ out, int64_t nblocks) {
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << 15);
#pragma unroll 4
        for (int it = 0; it < 128; ++it) o[256 * it + threadIdx.x] = (d2_t){(double)it, 1.0};
    }
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int nbuf = argc > 2 ? atoi(argv[2]) : 6;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t G = size_t(1) << 30, NPER = 32, bytes = NPER * G;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    auto fill = [&](double* p, size_t n) {
        hipLaunchKernelGGL(f_block_static, dim3(cus * 64), dim3(256), 0, 0, p, (int64_t)(n >> 19));
    };
    for (int k = 0; k < nbuf; ++k) {
        std::vector<hipMemGenericAllocationHandle_t> hs(NPER);
        for (auto& h : hs) CK(hipMemCreate(&h, G, &prop, 0));
        if (mode == 1 || mode == 2) {
            for (auto h : hs) {
                void* cva = nullptr;
                CK(hipMemAddressReserve(&cva, G, G, nullptr, 0));
                CK(hipMemMap(cva, G, 0, h, 0));
                CK(hipMemSetAccess(cva, G, &acc, 1));
                if (mode == 1) fill((double*)cva, G);
                CK(hipDeviceSynchronize());
                CK(hipMemUnmap(cva, G));
                CK(hipMemAddressFree(cva, G));
            }
        }
        void* va = nullptr;
        CK(hipMemAddressReserve(&va, bytes, G, nullptr, 0));
        for (size_t j = 0; j < NPER; ++j) CK(hipMemMap((char*)va + j * G, G, 0, hs[j], 0));
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        if (mode == 3)
            for (size_t j = 0; j < NPER; ++j) fill((double*)((char*)va + j * G), G);
        std::vector<float> ms;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(s, 0));
            fill((double*)va, bytes);
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            float t = 0;
            CK(hipEventElapsedTime(&t, s, e));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("mode %d buffer %d: static %.3f ms (min %.3f)\n", mode, k, ms[1], ms[0]);
        fflush(stdout);
        // kept mapped (as held drop-in results would be)
    }
    return 0;
}
