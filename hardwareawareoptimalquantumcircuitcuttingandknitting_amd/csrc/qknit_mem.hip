// qknit_mem.hip — output buffers mapped from 1-GiB physical allocations (gfx950).
//
// The knit's dominant kernel streams the 2^N output (syc 32: 2^32 fp64 = 34.4 GB per step) from
// persistent workgroups, each writing its own 512-KiB task. Into a plain hipMalloc buffer that write
// is bimodal: 4.83-4.87 ms into some allocations, 5.8-6.0 ms into others on the same box
// (tools/write_probe2..8). Composing the output from 1-GiB physical allocations (hipMemCreate) mapped
// into a reserved range made every buffer fast in one probe (tools/write_probe10), but later probes
// found the slow mode in such mappings too once several are made in a process, so
// engine.out_buffer times every new mapping of 4 GiB or more (a full 2^32 output or a multi-GPU
// rank's slice) with qk_out_write_rate and keeps the fastest of at most three.
//
//   qk_out_alloc(ctx, bytes, &ptr)  device memory of at least `bytes`, 1-GiB physical chunks (the
//                                   last holds only the rest, a multiple of the granularity) mapped
//                                   read-write for ctx's device; below 1 GiB one chunk at an
//                                   alignment of its power-of-two size
//   qk_out_write_rate(ctx, p, n, &gbs)  GB/s of the knit's static store order over [p, p + n) (one
//                                   timed launch after a warm one; the contents are overwritten).
//                                   It first drains the device: an error left by earlier work is
//                                   reported as "pre-existing", not as the probe's own
//   qk_out_free(ctx, ptr)           synchronizes the device, unmaps, releases the physical chunks;
//                                   the virtual range stays reserved (retired, never mapped again)
//   qk_out_stats(out, n)            process counters: reservations made / failed, live and retired
//                                   ranges and bytes, the largest reservation
//
// Retired ranges: a freed range whose addresses were reserved again for the next mapping read back
// wrong — 32-KiB runs of a live small mapping came back as zeros after other mappings had been freed
// and re-reserved (tools/diag/mapped_loop.py: 44 of 60 drop-in calls on cx_8x8 with 512-KiB outputs;
// none while no mapping was ever freed, tools/diag/mapped_read.py), i.e. translations of the old
// mapping outlived it. So a freed range's addresses are never handed out again: the physical memory
// goes back at once, the address range never. A reservation that fails is an error, and the caller
// (engine.out_buffer) falls back to an ordinary allocation with a warning. The device's reservable
// address space was measured with tools/va_probe.py (profiles/r06*_va_probe.json): see DESIGN.md §4.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

#include "internal.h"

namespace {

struct OutMapping {
    size_t bytes;  // reserved and mapped
    int device;
    std::vector<hipMemGenericAllocationHandle_t> chunks;
};

std::mutex g_mu;
std::map<uintptr_t, OutMapping> g_maps;
std::vector<std::pair<void*, size_t>> g_retired;  // unmapped ranges kept reserved (see above)

// process counters (qk_out_stats), under g_mu
struct OutStats {
    int64_t reserved = 0, reserve_failed = 0, map_failed = 0;  // hipMemAddressReserve calls ok / failed; chunk map failures
    int64_t live = 0, live_bytes = 0, retired = 0, retired_bytes = 0, max_bytes = 0;
    int64_t probe_pre_errors = 0;  // qk_out_write_rate calls that found an error left by earlier work
};
OutStats g_stats;

constexpr size_t OUT_CHUNK = size_t(1) << 30;

int mem_fail(qk_ctx* ctx, int code, const char* what, hipError_t e) {
    if (ctx) {
        char buf[256];
        snprintf(buf, sizeof buf, "%s: %s", what, e == hipSuccess ? "invalid argument" : hipGetErrorString(e));
        ctx->err = buf;
    }
    return code;
}

void unmap_release(void* va, OutMapping& m) {
    (void)hipMemUnmap(va, m.bytes);
    for (auto h : m.chunks) (void)hipMemRelease(h);
    (void)hipMemAddressFree(va, m.bytes);
}

// unmap and release the physical chunks; the range stays reserved, retired
void unmap_retire(void* va, OutMapping& m) {
    (void)hipMemUnmap(va, m.bytes);
    for (auto h : m.chunks) (void)hipMemRelease(h);
    std::lock_guard<std::mutex> lk(g_mu);
    g_retired.emplace_back(va, m.bytes);
    g_stats.live -= 1;
    g_stats.live_bytes -= (int64_t)m.bytes;
    g_stats.retired += 1;
    g_stats.retired_bytes += (int64_t)m.bytes;
}

}  // namespace

extern "C" {

int qk_out_alloc(qk_ctx* ctx, int64_t bytes, void** ptr) {
    if (!ctx || !ptr || bytes <= 0) return mem_fail(ctx, QK_EARG, "qk_out_alloc: need a context, bytes > 0", hipSuccess);
    *ptr = nullptr;
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_alloc: hipSetDevice", e);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = ctx->device;
    size_t gran = 0;
    e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    if (e != hipSuccess || gran == 0) return mem_fail(ctx, QK_EHIP, "qk_out_alloc: allocation granularity", e);
    size_t want = ((size_t)bytes + gran - 1) / gran * gran;
    // QKNIT_OUT_CHUNK_MB (A/B experiments, read per call): physical chunk size, a multiple of the granularity
    const char* chunk_env = getenv("QKNIT_OUT_CHUNK_MB");
    const size_t big = chunk_env ? ((size_t)atoll(chunk_env) << 20) / gran * gran : OUT_CHUNK;
    size_t chunk = big > 0 ? big : OUT_CHUNK, align = chunk;
    if (want < chunk) {  // one chunk, aligned to its power-of-two size
        chunk = want;
        align = gran;
        while (align < want) align <<= 1;
    }
    const size_t n_chunks = (want + chunk - 1) / chunk;
    // the last chunk holds only the rest (a multiple of the granularity): 1.1 GiB maps 1.1, not 2 GiB
    OutMapping m{want, ctx->device, {}};
    void* va = nullptr;
    // A failed reservation is an error (the caller falls back to an ordinary allocation): retired ranges
    // are never handed back, since translations of an unmapped range outlive it — round 4 kept them
    // and released them all when a reservation failed, and a new mapping that landed on one could
    // fault on its first write (a 2 -> 4-rank process, profiles/r05bb_*)
    e = hipMemAddressReserve(&va, m.bytes, align, nullptr, 0);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (e != hipSuccess) g_stats.reserve_failed += 1;
        else g_stats.reserved += 1;
    }
    if (e != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_alloc: hipMemAddressReserve", e);
    size_t mapped = 0;
    for (size_t i = 0; i < n_chunks; ++i) {
        hipMemGenericAllocationHandle_t h;
        const size_t sz = i + 1 < n_chunks ? chunk : want - i * chunk;
        e = hipMemCreate(&h, sz, &prop, 0);
        if (e == hipSuccess) {
            e = hipMemMap((char*)va + i * chunk, sz, 0, h, 0);
            if (e != hipSuccess) (void)hipMemRelease(h);
        }
        if (e != hipSuccess) {
            (void)hipMemUnmap(va, mapped);
            for (auto hh : m.chunks) (void)hipMemRelease(hh);
            (void)hipMemAddressFree(va, m.bytes);  // never mapped whole: nothing to outlive
            {
                std::lock_guard<std::mutex> lk(g_mu);
                g_stats.map_failed += 1;
            }
            return mem_fail(ctx, QK_EHIP, "qk_out_alloc: hipMemCreate / hipMemMap", e);
        }
        m.chunks.push_back(h);
        mapped += sz;
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(va, m.bytes, &acc, 1);
    if (e != hipSuccess) {
        unmap_release(va, m);
        return mem_fail(ctx, QK_EHIP, "qk_out_alloc: hipMemSetAccess", e);
    }
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_stats.live += 1;
        g_stats.live_bytes += (int64_t)m.bytes;
        if ((int64_t)m.bytes > g_stats.max_bytes) g_stats.max_bytes = (int64_t)m.bytes;
        g_maps[(uintptr_t)va] = std::move(m);
    }
    *ptr = va;
    return QK_OK;
}

int qk_out_free(qk_ctx* ctx, void* ptr) {
    if (!ptr) return QK_OK;
    OutMapping m;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_maps.find((uintptr_t)ptr);
        if (it == g_maps.end()) return mem_fail(ctx, QK_EARG, "qk_out_free: not a qk_out_alloc pointer", hipSuccess);
        m = std::move(it->second);
        g_maps.erase(it);
    }
    (void)hipSetDevice(m.device);
    // kernels on any stream may still write the buffer: the mapping goes only when they are done
    hipError_t e = hipDeviceSynchronize();
    unmap_retire(ptr, m);
    if (e != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_free: hipDeviceSynchronize", e);
    return QK_OK;
}

// The static store order of the knit's write (512-KiB blocks, a grid-stride over them): the rate
// qk_out_write_rate reports for a mapping.
__global__ __launch_bounds__(256) void qk_out_probe_kernel(double* __restrict__ out, int64_t nblocks) {
    typedef double d2_t __attribute__((ext_vector_type(2)));
    for (int64_t t = blockIdx.x; t < nblocks; t += gridDim.x) {
        d2_t* o = reinterpret_cast<d2_t*>(out) + (t << 15);
#pragma unroll 4
        for (int it = 0; it < 128; ++it) o[256 * it + threadIdx.x] = (d2_t){0.0, 0.0};
    }
}

int qk_out_write_rate(qk_ctx* ctx, void* ptr, int64_t bytes, double* gbs) {
    if (!ctx || !ptr || !gbs || bytes < (int64_t(1) << 19))
        return mem_fail(ctx, QK_EARG, "qk_out_write_rate: need a context, a buffer of >= 512 KiB, an out pointer", hipSuccess);
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_write_rate: hipSetDevice", e);
    // Drain the device first: an error that earlier asynchronous work left (a fault in another stream's
    // kernel) would otherwise surface at this call's event wait and read as the probe's own
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
        {
            std::lock_guard<std::mutex> lk(g_mu);
            g_stats.probe_pre_errors += 1;
        }
        return mem_fail(ctx, QK_EHIP, "qk_out_write_rate: pre-existing error (earlier work, before the probe)", e);
    }
    {  // the probe's grid covers exactly [ptr, ptr + 512 KiB * nblocks): the range must be one live mapping
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_maps.upper_bound((uintptr_t)ptr);
        bool inside = false;
        if (it != g_maps.begin()) {
            --it;
            inside = (uintptr_t)ptr + (uintptr_t)bytes <= it->first + it->second.bytes;
        }
        if (!inside) return mem_fail(ctx, QK_EARG, "qk_out_write_rate: range is not inside a live qk_out_alloc mapping", hipSuccess);
    }
    const int64_t nblocks = bytes >> 19;
    hipEvent_t t0, t1;
    if ((e = hipEventCreate(&t0)) != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_write_rate: event", e);
    if ((e = hipEventCreate(&t1)) != hipSuccess) {
        (void)hipEventDestroy(t0);
        return mem_fail(ctx, QK_EHIP, "qk_out_write_rate: event", e);
    }
    const dim3 grid((unsigned)(ctx->cus > 0 ? ctx->cus : 256) * 64);
    hipLaunchKernelGGL(qk_out_probe_kernel, grid, dim3(256), 0, ctx->stream, (double*)ptr, nblocks);  // warm
    (void)hipEventRecord(t0, ctx->stream);
    hipLaunchKernelGGL(qk_out_probe_kernel, grid, dim3(256), 0, ctx->stream, (double*)ptr, nblocks);
    (void)hipEventRecord(t1, ctx->stream);
    e = hipGetLastError();  // launch errors
    if (e == hipSuccess) e = hipEventSynchronize(t1);
    float ms = 0.0f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t0, t1);
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (e != hipSuccess) return mem_fail(ctx, QK_EHIP, "qk_out_write_rate", e);
    *gbs = ms > 0 ? (double)(nblocks << 19) / (ms * 1e6) : 0.0;
    return QK_OK;
}

int qk_out_stats(int64_t* out, int n) {
    if (!out || n <= 0) return QK_EARG;
    std::lock_guard<std::mutex> lk(g_mu);
    const int64_t v[] = {g_stats.reserved, g_stats.reserve_failed, g_stats.map_failed, g_stats.live,
                         g_stats.live_bytes, g_stats.retired, g_stats.retired_bytes, g_stats.max_bytes,
                         g_stats.probe_pre_errors};
    const int m = (int)(sizeof v / sizeof v[0]);
    for (int i = 0; i < n; ++i) out[i] = i < m ? v[i] : 0;
    return QK_OK;
}

int qk_out_mapped_bytes(const void* ptr, int64_t* bytes) {
    if (!bytes) return QK_EARG;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_maps.find((uintptr_t)ptr);
    *bytes = it == g_maps.end() ? 0 : (int64_t)it->second.bytes;
    return it == g_maps.end() ? QK_EARG : QK_OK;
}

}  // extern "C"
