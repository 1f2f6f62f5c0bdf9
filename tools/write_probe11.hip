// write_probe11.hip — which 34-GiB qk_out_alloc-style mappings write fast? (round 4)
// tools/out_mapping_probe.py found the bench knit fast (4.84-4.92 ms) into the first two 32-GiB
// mappings of a process and slow (5.6-5.9 ms) into every later one, held or not, while
// write_probe10 (all physical chunks created first, one buffer mapped at a time) found all fast.
// Modes: 0 = chunks created per buffer, buffers kept mapped (qk_out_alloc); 1 = all chunks first,
// buffers kept mapped; 2 = chunks per buffer, each buffer unmapped (and released) after its timing;
// +10: the range is reserved 1 GiB larger and the buffer mapped at its first 1-GiB-aligned address
// (hipMemAddressReserve returns 2-MiB-aligned ranges whatever alignment is asked).
// Every buffer is timed right after mapping and again after 0.5 s and 2 s of an idle GPU (does the
// slow mode follow work the driver does on freshly allocated memory in the background?).
//   hipcc --offload-arch=gfx950 -O3 -o tools/write_probe11 tools/write_probe11.hip && tools/write_probe11 MODE
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <unistd.h>

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
    const int arg = argc > 1 ? atoi(argv[1]) : 0;
    const int mode = arg % 10;
    const bool align = arg >= 10;
    const int nbuf = argc > 2 ? atoi(argv[2]) : 6;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t G = size_t(1) << 30, NPER = 32;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    std::vector<hipMemGenericAllocationHandle_t> all;
    if (mode == 1) {
        for (int i = 0; i < nbuf * (int)NPER; ++i) {
            hipMemGenericAllocationHandle_t h;
            CK(hipMemCreate(&h, G, &prop, 0));
            all.push_back(h);
        }
    }
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    const size_t bytes = NPER * G;
    const int64_t n2 = bytes / 16;
    for (int k = 0; k < nbuf; ++k) {
        void* base = nullptr;
        CK(hipMemAddressReserve(&base, bytes + (align ? G : 0), G, nullptr, 0));
        void* va = align ? (void*)(((uintptr_t)base + G - 1) & ~(uintptr_t)(G - 1)) : base;
        std::vector<hipMemGenericAllocationHandle_t> hs;
        for (size_t j = 0; j < NPER; ++j) {
            hipMemGenericAllocationHandle_t h;
            if (mode == 1) h = all[k * NPER + j];
            else CK(hipMemCreate(&h, G, &prop, 0));
            hs.push_back(h);
            CK(hipMemMap((char*)va + j * G, G, 0, h, 0));
        }
        CK(hipMemSetAccess(va, bytes, &acc, 1));
        double* p = (double*)va;
        float med[3];
        const int waits_ms[3] = {0, 500, 2000};
        for (int w = 0; w < 3; ++w) {
            usleep(1000 * waits_ms[w]);
            std::vector<float> ms;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(s, 0));
                hipLaunchKernelGGL(f_block_static, dim3(cus * 64), dim3(256), 0, 0, p, (int64_t)(n2 >> 15));
                CK(hipEventRecord(e, 0));
                CK(hipEventSynchronize(e));
                float t = 0;
                CK(hipEventElapsedTime(&t, s, e));
                if (r) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            med[w] = ms[1];
        }
        printf("mode %d%s buffer %d va %p (mod 1 GiB %#zx): static %.3f ms at once, %.3f after 0.5 s, %.3f after 2 s\n",
               mode, align ? " aligned" : "", k, va, (size_t)((uintptr_t)va % G), med[0], med[1], med[2]);
        fflush(stdout);
        if (mode == 2) {
            CK(hipDeviceSynchronize());
            CK(hipMemUnmap(va, bytes));
            for (auto h : hs) CK(hipMemRelease(h));
        }
    }
    return 0;
}
