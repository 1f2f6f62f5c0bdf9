// Fiber exchange cost on gfx950: the sweep kernels' LDS round trip against wavefront shuffles.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fiber_exchange_probe.hip -o tools/fiber_exchange_probe
//   ./tools/fiber_exchange_probe            (one JSON line per variant)
//
// Each thread holds a 16-amplitude fiber (4 tile bits) in registers, as the per-program sweep kernels
// do (sweep_codegen.py: PER = 16, v[16] double2). Between two gate groups the fiber moves to other
// tile bits. The kernels here do R rounds of (one FMA per amplitude component, then a fiber change):
//   ops     no fiber change (the arithmetic alone: subtracted from the others)
//   lds     the production form: 16 double2 stores at the old fiber, barrier, 16 loads at the new
//           fiber, barrier (the XOR swizzle of sweep_codegen._swz); cost independent of the bits moved
//   shfl k  k fiber bits swapped with k lane bits inside the wavefront: per bit, 8 selects of the
//           double2 to send, 8 double2 __shfl_xor (4 dwords each), 8 selects back
//   dpp k   as shfl k, lane bits 0 / 1 through DPP quad permutes (k <= 2)
// The tile is 2^12 amplitudes (64 KiB LDS, 256 threads), 8192 workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int TB = 12, NT = 1 << (TB - 4), PER = 16;

__device__ __forceinline__ unsigned swz(unsigned t) { return t ^ (((t >> 4) ^ (t >> 8)) & 15u); }

__device__ __forceinline__ double shfl_x(double x, int m) { return __shfl_xor(x, m, 64); }

template <int MASK>
__device__ __forceinline__ double dpp_x(double x) {
    // quad_perm selector for lane ^ MASK within a quad (MASK 1: [1,0,3,2]; MASK 2: [2,3,0,1])
    constexpr int sel = MASK == 1 ? (1 | (0 << 2) | (3 << 4) | (2 << 6)) : (2 | (3 << 2) | (0 << 4) | (1 << 6));
    int lo = __double2loint(x), hi = __double2hiint(x);
    lo = __builtin_amdgcn_update_dpp(0, lo, sel, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, sel, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

template <int MODE, int K>  // MODE 0 ops, 1 lds, 2 shfl, 3 dpp
__global__ __launch_bounds__(NT) void fiber_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                   int rounds, double c) {
    __shared__ double2 lds[1 << TB];
    const unsigned tid = threadIdx.x;
    const long long base = (long long)blockIdx.x << TB;
    double2 v[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) v[r] = in[base + tid + NT * r];
    for (int it = 0; it < rounds; ++it) {
#pragma unroll
        for (int r = 0; r < PER; ++r) {
            if (c != 0.0) {  // c = 0: data movement only (the check below)
                v[r].x = fma(v[r].x, c, v[r].y);
                v[r].y = fma(v[r].y, c, -v[r].x);
            }
        }
        if constexpr (MODE == 1) {
            // old fiber: tile bits 8..11 (thread bits 0..7 below them); new fiber: tile bits 0..3
            // (alternating rounds go back, so every round moves all 4 bits)
            const bool fwd = !(it & 1);
#pragma unroll
            for (int r = 0; r < PER; ++r) {
                const unsigned a = fwd ? (tid | (unsigned)r << 8) : ((tid << 4) | (unsigned)r);
                lds[swz(a)] = v[r];
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < PER; ++r) {
                const unsigned a = fwd ? ((tid << 4) | (unsigned)r) : (tid | (unsigned)r << 8);
                v[r] = lds[swz(a)];
            }
            __syncthreads();
        } else if constexpr (MODE >= 2) {
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const int t = j;  // fiber bit j <-> lane bit j
                const bool b = (tid >> t) & 1u;
#pragma unroll
                for (int r = 0; r < PER; ++r) {
                    if (r & (1 << j)) continue;
                    const int r1 = r | (1 << j);
                    double2 s = b ? v[r] : v[r1];
                    double2 g;
                    if constexpr (MODE == 2) {
                        g.x = shfl_x(s.x, 1 << t);
                        g.y = shfl_x(s.y, 1 << t);
                    } else {
                        if (t == 0) { g.x = dpp_x<1>(s.x); g.y = dpp_x<1>(s.y); }
                        else { g.x = dpp_x<2>(s.x); g.y = dpp_x<2>(s.y); }
                    }
                    if (b) v[r] = g; else v[r1] = g;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < PER; ++r) out[base + tid + NT * r] = v[r];
}

template <int MODE, int K>
static void run(const char* name, const double2* in, double2* out, int blocks, int rounds) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto launch = [&] { fiber_kernel<MODE, K><<<blocks, NT>>>(in, out, rounds, 0.999999); };
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    // per round, per wavefront-instruction-slot: ns per round over the whole grid
    printf("{\"variant\": \"%s\", \"k_bits\": %d, \"ms\": %.4f, \"rounds\": %d, \"workgroups\": %d, "
           "\"ns_per_round\": %.3f}\n", name, K, best, rounds, blocks, best * 1e6 / rounds);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 8192;
    const int rounds = argc > 2 ? atoi(argv[2]) : 64;
    const size_t n = (size_t)blocks << TB;
    double2 *in, *out;
    CHECK(hipMalloc(&in, n * sizeof(double2)));
    CHECK(hipMalloc(&out, n * sizeof(double2)));
    std::vector<double2> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = make_double2(1e-3 * (double)(i % 977), 1e-3 * (double)(i % 613));
    CHECK(hipMemcpy(in, h.data(), n * sizeof(double2), hipMemcpyHostToDevice));
    run<0, 0>("ops", in, out, blocks, rounds);
    run<1, 4>("lds", in, out, blocks, rounds);
    run<2, 1>("shfl", in, out, blocks, rounds);
    run<2, 2>("shfl", in, out, blocks, rounds);
    run<2, 3>("shfl", in, out, blocks, rounds);
    run<2, 4>("shfl", in, out, blocks, rounds);
    run<3, 1>("dpp", in, out, blocks, rounds);
    run<3, 2>("dpp", in, out, blocks, rounds);
    // the shuffle forms move data as an exchange of fiber bits 0..k-1 with lane bits 0..k-1: thread t,
    // register r then holds the amplitude first held by thread t', register r' (bits j < k swapped)
    auto check = [&](auto kern, int K, const char* name) {
        kern<<<blocks, NT>>>(in, out, 1, 0.0);
        CHECK(hipDeviceSynchronize());
        std::vector<double2> o(n);
        CHECK(hipMemcpy(o.data(), out, n * sizeof(double2), hipMemcpyDeviceToHost));
        long long bad = 0;
        const unsigned m = (1u << K) - 1;
        for (size_t b = 0; b < (size_t)blocks; b += 97)
            for (unsigned t = 0; t < (unsigned)NT; ++t)
                for (unsigned r = 0; r < (unsigned)PER; ++r) {
                    const unsigned t0 = (t & ~m) | (r & m), r0 = (r & ~m) | (t & m);
                    const double2 want = h[(b << TB) + t0 + NT * r0], got = o[(b << TB) + t + NT * r];
                    bad += want.x != got.x || want.y != got.y;
                }
        printf("{\"check\": \"%s\", \"k_bits\": %d, \"mismatches\": %lld}\n", name, K, bad);
        if (bad) exit(2);
    };
    check(fiber_kernel<2, 4>, 4, "shfl");
    check(fiber_kernel<3, 2>, 2, "dpp");
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
}
