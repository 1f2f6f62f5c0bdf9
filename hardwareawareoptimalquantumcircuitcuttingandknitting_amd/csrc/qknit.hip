// qknit.hip — MI355X (gfx950 / CDNA4) kernels and C ABI of the circuit-knitting engine.
//
// Hot path of the reference (thangktran/HardwareAwareOptimalQuantumCircuitCuttingAndKnitting):
//   * qk_sweep          — batched exact statevector sweep of every cut instantiation of a
//                         fragment (replaces AerSimulator via third_party/qvm/qvm/run.py:36-58)
//   * qk_reduce_labels  — signed config-bit folding per label (virtual_gates.py:105-124,179-194)
//   * qk_gemm_keyed     — fp64 MFMA knit contraction with global-key scatter
//                         (replaces virtual_circuit.py:50-68,165-171,216-228, quasi_distr.py:55-60)
// Design notes: DESIGN.md §3 (sweep) and §4 (knit).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "internal.h"
#include "sweep_ops.h"

namespace {

constexpr int TILE = 1 << QK_TILE_BITS;  // 4096 amplitudes per tile (64 KiB complex128)
constexpr int NT = 256;                    // threads per sweep workgroup (TILE / NT = PER = 16)

int fail(qk_ctx* ctx, int code, const char* fmt, const char* detail = "") {
    if (ctx) {
        char buf[512];
        snprintf(buf, sizeof(buf), fmt, detail);
        ctx->err = buf;
    }
    return code;
}

#define QK_HIP(ctx, call)                                                     \
    do {                                                                      \
        hipError_t e_ = (call);                                               \
        if (e_ != hipSuccess) return fail(ctx, QK_EHIP, "%s", hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------------------------------------
// sweep: per-fiber ops (sweep_ops.h) and the interpreter's dispatch
// ------------------------------------------------------------------------------------------
using namespace qk_sweep_ops;

// Keeps the fiber in VGPRs: without it SimplifyCFG merges the per-position switch cases into
// loads/stores through a phi'd pointer and the whole fiber is demoted to scratch.
__device__ __forceinline__ void pin(double2 (&v)[PER]) {
#pragma unroll
    for (int r = 0; r < PER; ++r) asm volatile("" : "+v"(v[r].x), "+v"(v[r].y));
}

__device__ __forceinline__ void dispatch_u1(int a, double2 (&v)[PER], const double* m) {
    switch (a) {
        case 0: ap_u1<0>(v, m); pin(v); break;
        case 1: ap_u1<1>(v, m); pin(v); break;
        case 2: ap_u1<2>(v, m); pin(v); break;
        default: ap_u1<3>(v, m); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_u1r(int a, double2 (&v)[PER], const double* m) {
    switch (a) {
        case 0: ap_u1r<0>(v, m); pin(v); break;
        case 1: ap_u1r<1>(v, m); pin(v); break;
        case 2: ap_u1r<2>(v, m); pin(v); break;
        default: ap_u1r<3>(v, m); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_u1x(int a, double2 (&v)[PER], const double* m) {
    switch (a) {
        case 0: ap_u1x<0>(v, m); pin(v); break;
        case 1: ap_u1x<1>(v, m); pin(v); break;
        case 2: ap_u1x<2>(v, m); pin(v); break;
        default: ap_u1x<3>(v, m); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_d1r(int a, double2 (&v)[PER], const double* d) {
    switch (a) {
        case 0: ap_d1r<0>(v, d); pin(v); break;
        case 1: ap_d1r<1>(v, d); pin(v); break;
        case 2: ap_d1r<2>(v, d); pin(v); break;
        default: ap_d1r<3>(v, d); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_d1(int a, double2 (&v)[PER], const double* d) {
    switch (a) {
        case 0: ap_d1<0>(v, d); pin(v); break;
        case 1: ap_d1<1>(v, d); pin(v); break;
        case 2: ap_d1<2>(v, d); pin(v); break;
        default: ap_d1<3>(v, d); pin(v); break;
    }
}

// pair index for a<b in 0..3: (0,1)=0 (0,2)=1 (0,3)=2 (1,2)=3 (1,3)=4 (2,3)=5
__device__ __forceinline__ int pair_id(int a, int b) {
    return a == 0 ? b - 1 : (a == 1 ? b + 1 : 5);
}

__device__ __forceinline__ void dispatch_u2(int a, int b, double2 (&v)[PER], const double* m) {
    switch (pair_id(a, b)) {
        case 0: ap_u2<0, 1>(v, m); pin(v); break;
        case 1: ap_u2<0, 2>(v, m); pin(v); break;
        case 2: ap_u2<0, 3>(v, m); pin(v); break;
        case 3: ap_u2<1, 2>(v, m); pin(v); break;
        case 4: ap_u2<1, 3>(v, m); pin(v); break;
        default: ap_u2<2, 3>(v, m); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_d2(int a, int b, double2 (&v)[PER], const double* d) {
    switch (pair_id(a, b)) {
        case 0: ap_d2<0, 1>(v, d); pin(v); break;
        case 1: ap_d2<0, 2>(v, d); pin(v); break;
        case 2: ap_d2<0, 3>(v, d); pin(v); break;
        case 3: ap_d2<1, 2>(v, d); pin(v); break;
        case 4: ap_d2<1, 3>(v, d); pin(v); break;
        default: ap_d2<2, 3>(v, d); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_d2r(int a, int b, double2 (&v)[PER], const double* d) {
    switch (pair_id(a, b)) {
        case 0: ap_d2r<0, 1>(v, d); pin(v); break;
        case 1: ap_d2r<0, 2>(v, d); pin(v); break;
        case 2: ap_d2r<0, 3>(v, d); pin(v); break;
        case 3: ap_d2r<1, 2>(v, d); pin(v); break;
        case 4: ap_d2r<1, 3>(v, d); pin(v); break;
        default: ap_d2r<2, 3>(v, d); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_swap(int a, int b, double2 (&v)[PER]) {
    switch (pair_id(a, b)) {
        case 0: ap_swap<0, 1>(v); pin(v); break;
        case 1: ap_swap<0, 2>(v); pin(v); break;
        case 2: ap_swap<0, 3>(v); pin(v); break;
        case 3: ap_swap<1, 2>(v); pin(v); break;
        case 4: ap_swap<1, 3>(v); pin(v); break;
        default: ap_swap<2, 3>(v); pin(v); break;
    }
}

__device__ __forceinline__ void dispatch_cx(int c, int t, double2 (&v)[PER]) {
    switch (c * 4 + t) {
        case 1: ap_cx<0, 1>(v); pin(v); break;
        case 2: ap_cx<0, 2>(v); pin(v); break;
        case 3: ap_cx<0, 3>(v); pin(v); break;
        case 4: ap_cx<1, 0>(v); pin(v); break;
        case 6: ap_cx<1, 2>(v); pin(v); break;
        case 7: ap_cx<1, 3>(v); pin(v); break;
        case 8: ap_cx<2, 0>(v); pin(v); break;
        case 9: ap_cx<2, 1>(v); pin(v); break;
        case 11: ap_cx<2, 3>(v); pin(v); break;
        case 12: ap_cx<3, 0>(v); pin(v); break;
        case 13: ap_cx<3, 1>(v); pin(v); break;
        case 14: ap_cx<3, 2>(v); pin(v); break;
        default: break;
    }
}

// out = variant 0 of p (N doubles), or variant 1 where `b` (only if the op has that bit, `h`).
// `h` is wave-uniform, so the second variant's loads stay scalar; `b` is per lane.
template <int N>
__device__ __forceinline__ void select_variant(double (&out)[N], const double* p, bool h, bool b) {
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = p[k];
    if (h) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const double alt = p[N + k];
            out[k] = b ? alt : out[k];
        }
    }
}

// Variant index b1 + 2*b2 over up to four N-double variants (SCALE/SCALER encoding).
template <int N>
__device__ __forceinline__ void select_variant4(double (&out)[N], const double* p, bool h1, bool b1, bool h2,
                                                bool b2) {
    select_variant<N>(out, p, h1, b1);
    if (h2) {
        double hi[N];
        select_variant<N>(hi, p + 2 * N, h1, b1);
#pragma unroll
        for (int k = 0; k < N; ++k) out[k] = b2 ? hi[k] : out[k];
    }
}

struct SweepArgs {
    const qk_op* ops;
    const qk_group* groups;
    const double* mats;
    const double* job_slots;
    const double* job_sign;
    double2* state;  // SPLIT: [n_jobs][2^n]
    double* pjob;    // FINAL: [n_jobs][2^m]
    int64_t n_jobs;
    uint64_t tile_mask;
    uint64_t zero_mask;  // state elements with any of these bits set are known zero (not loaded)
    int init_sparse;     // SPLIT INIT pass launched on the |0..0>-containing tile of each job only
    int group_begin, group_end;
    int flags;
    uint32_t traced_local;
    int n, n_eff, m, n_slots;
};

// Deposit the low bits of `x` into the set bits of `mask` (mask has <= 64 bits).
__device__ __forceinline__ uint64_t pdep64(uint64_t x, uint64_t mask) {
    uint64_t r = 0;
    while (mask) {
        const uint64_t low = mask & (~mask + 1);
        if (x & 1) r |= low;
        x >>= 1;
        mask ^= low;
    }
    return r;
}

// One pass of the batched sweep. PACKED: a tile = 2^(12-n_eff) whole jobs. SPLIT: a tile =
// 12 state bits (tile_mask) of one job, 2^(n-12) tiles per job.
template <bool PACKED>
// The program (ops, groups, mats) comes in as separate __restrict__ read-only pointers so the
// compiler can prove it uniform and unclobbered: it then uses scalar (K$) loads instead of a
// vector-memory round trip per op.
__global__ __launch_bounds__(NT) void qk_sweep_pass_kernel(SweepArgs a, const qk_op* __restrict__ g_ops,
                                                           const qk_group* __restrict__ g_groups,
                                                           const double* __restrict__ g_mats) {
    __shared__ double2 lds[TILE];
    const int tid = threadIdx.x;
    const bool init = a.flags & 1;
    const bool final_ = a.flags & 2;

    int64_t job0;        // PACKED: first job of the tile; SPLIT: the job
    uint64_t tbase = 0;  // SPLIT: state bits outside the tile
    uint64_t outside = 0;
    int bitpos[QK_TILE_BITS];
    if (PACKED) {
        job0 = (int64_t)blockIdx.x << (QK_TILE_BITS - a.n_eff);
    } else {
        const int64_t tiles_per_job = a.init_sparse ? 1 : ((int64_t)1 << (a.n - QK_TILE_BITS));
        job0 = (int64_t)blockIdx.x / tiles_per_job;
        const uint64_t tj = (uint64_t)((int64_t)blockIdx.x % tiles_per_job);
        const uint64_t nmask = (a.n >= 64) ? ~0ull : ((1ull << a.n) - 1);
        outside = nmask & ~a.tile_mask;
        tbase = pdep64(tj, outside);
        uint64_t mk = a.tile_mask;
#pragma unroll
        for (int i = 0; i < QK_TILE_BITS; ++i) {
            bitpos[i] = __builtin_ctzll(mk);
            mk &= mk - 1;
        }
    }
    auto local_to_state = [&](int t) -> uint64_t {  // SPLIT only
        uint64_t s = tbase;
#pragma unroll
        for (int i = 0; i < QK_TILE_BITS; ++i) s |= (uint64_t)((t >> i) & 1) << bitpos[i];
        return s;
    };
    const int64_t njobs = a.n_jobs;
    const int64_t stride_job = PACKED ? 0 : ((int64_t)1 << a.n);

    // A SPLIT tile of |0..0> with a non-zero outside part is all zeros and stays zero under the
    // pass (tile-local unitaries + diagonal action): store zeros, skip the groups.
    bool zero_tile = false;
    if (!PACKED && init && tbase != 0) {
        if (!final_) {
            double2* dst = a.state + job0 * stride_job;
#pragma unroll
            for (int i = 0; i < PER; ++i) dst[local_to_state(tid + NT * i)] = make_double2(0.0, 0.0);
            return;
        }
        zero_tile = true;
    }

    // ---- load or initialise the tile
    if (init) {
        const int nmask = (1 << a.n_eff) - 1;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int t = tid + NT * i;
            const bool one = PACKED ? ((t & nmask) == 0) : (tbase == 0 && t == 0);
            lds[swz(t)] = make_double2(one ? 1.0 : 0.0, 0.0);
        }
    } else {
        const double2* src = a.state + job0 * stride_job;
        const uint64_t zm = a.zero_mask;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int t = tid + NT * i;
            const uint64_t s = local_to_state(t);
            lds[swz(t)] = (s & zm) ? make_double2(0.0, 0.0) : src[s];
        }
    }
    __syncthreads();

    // ---- fiber groups
    for (int g = a.group_begin; !zero_tile && g < a.group_end; ++g) {
        const qk_group grp = g_groups[g];
        const int p0 = grp.pos[0], p1 = grp.pos[1], p2 = grp.pos[2], p3 = grp.pos[3];
        const int fmask = (1 << p0) | (1 << p1) | (1 << p2) | (1 << p3);
        // base local index: deposit tid into the 8 non-fiber positions
        int base = 0;
        {
            int x = tid;
#pragma unroll
            for (int b = 0; b < QK_TILE_BITS; ++b) {
                if (!((fmask >> b) & 1)) {
                    base |= (x & 1) << b;
                    x >>= 1;
                }
            }
        }
        int idx[PER];
#pragma unroll
        for (int r = 0; r < PER; ++r)
            idx[r] = base | ((r & 1) << p0) | (((r >> 1) & 1) << p1) | (((r >> 2) & 1) << p2) |
                     (((r >> 3) & 1) << p3);
        double2 v[PER];
#pragma unroll
        for (int r = 0; r < PER; ++r) v[r] = lds[swz(idx[r])];

        uint64_t sbase;
        int64_t job;
        if (PACKED) {
            sbase = (uint64_t)(base & ((1 << a.n_eff) - 1));
            job = job0 + (base >> a.n_eff);
        } else {
            sbase = local_to_state(base);
            job = job0;
        }
        const int64_t job_c = job < njobs ? job : njobs - 1;  // padded tile slots reuse a valid row

        for (int o = grp.op_begin; o < grp.op_end; ++o) {
            const qk_op op = g_ops[o];
            // Matrix data is read at uniform addresses (scalar loads); a per-lane variant chosen by
            // external state bits is then picked with selects, never with per-lane addresses.
            const double* mp = g_mats + op.mat;
            const bool h1 = op.e1 >= 0, h2 = op.e2 >= 0;
            const bool b1 = h1 && ((sbase >> op.e1) & 1);
            const bool b2 = h2 && ((sbase >> op.e2) & 1);
            switch (op.kind) {
                case QK_U1: {
                    double m[8];
                    select_variant<8>(m, mp, h1, b1);
                    dispatch_u1(op.a, v, m);
                } break;
                case QK_D1: {
                    double m[4];
                    select_variant<4>(m, mp, h1, b1);
                    dispatch_d1(op.a, v, m);
                } break;
                case QK_SLOT:
                    dispatch_u1(op.a, v, a.job_slots + (job_c * a.n_slots + op.slot) * 8);
                    break;
                case QK_U2: dispatch_u2(op.a, op.b, v, mp); break;
                case QK_D2: dispatch_d2(op.a, op.b, v, mp); break;
                case QK_CX: dispatch_cx(op.a, op.b, v); break;
                case QK_SWAP: dispatch_swap(op.a, op.b, v); break;
                case QK_SCALE: {
                    double s[2];
                    select_variant4<2>(s, mp, h1, b1, h2, b2);
#pragma unroll
                    for (int r = 0; r < PER; ++r) v[r] = cmul(s[0], s[1], v[r]);
                    pin(v);
                } break;
                case QK_U1R: dispatch_u1r(op.a, v, mp); break;
                case QK_U1X: dispatch_u1x(op.a, v, mp); break;
                case QK_D1R: {
                    double m[2];
                    select_variant<2>(m, mp, h1, b1);
                    dispatch_d1r(op.a, v, m);
                } break;
                case QK_D2R: dispatch_d2r(op.a, op.b, v, mp); break;
                case QK_SCALER: {
                    double s[1];
                    select_variant4<1>(s, mp, h1, b1, h2, b2);
#pragma unroll
                    for (int r = 0; r < PER; ++r) v[r] = make_double2(s[0] * v[r].x, s[0] * v[r].y);
                    pin(v);
                } break;
                default: break;
            }
        }
#pragma unroll
        for (int r = 0; r < PER; ++r) lds[swz(idx[r])] = v[r];
        __syncthreads();
    }

    // ---- store the tile, or emit signed probabilities
    if (!final_) {
        double2* dst = a.state + job0 * stride_job;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int t = tid + NT * i;
            dst[local_to_state(t)] = lds[swz(t)];
        }
        return;
    }
    const uint32_t traced = a.traced_local;
    const uint64_t mmask = (a.m >= 64) ? ~0ull : ((1ull << a.m) - 1);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int t = tid + NT * i;
        if (t & traced) continue;
        double acc = 0.0;
        uint32_t sub = 0;
        do {
            const double2 z = lds[swz(t | (int)sub)];
            acc = fma(z.x, z.x, fma(z.y, z.y, acc));
            sub = (sub - traced) & traced;
        } while (sub != 0);
        int64_t job;
        uint64_t x;
        if (PACKED) {
            job = job0 + (t >> a.n_eff);
            x = (uint64_t)t & mmask;
        } else {
            job = job0;
            x = local_to_state(t) & mmask;
        }
        if (job < njobs) a.pjob[(job << a.m) + (int64_t)x] = a.job_sign[job] * acc;
    }
}

__global__ void qk_reduce_labels_kernel(int64_t n_labels, const int64_t* __restrict__ offsets,
                                        int64_t width, const double* __restrict__ pjob,
                                        double* __restrict__ q) {
    const int64_t total = n_labels * width;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t l = e / width, x = e - l * width;
        double s = 0.0;
        for (int64_t j = offsets[l]; j < offsets[l + 1]; ++j) s += pjob[j * width + x];
        q[e] = s;
    }
}

// ------------------------------------------------------------------------------------------
// knit: fp64 MFMA GEMM, out[keyA[i] + keyB[j]] = sum_k A[k][i] * B[k][j]
// ------------------------------------------------------------------------------------------
typedef double d4_t __attribute__((ext_vector_type(4)));

constexpr int GT = 128;      // workgroup tile (M and N)
constexpr int GK = 16;       // K chunk
constexpr int GPAD = 16;     // LDS row padding (doubles): 1152-B rows avoid the 2-way conflict

#ifndef QK_GEMM_GROUP
#define QK_GEMM_GROUP 8  // tile rows per L2 group (0 = plain column-major tile order)
#endif
#ifndef QK_GEMM_NT
#define QK_GEMM_NT 1     // non-temporal output stores (the 2^N output is written once)
#endif

typedef double d2_t __attribute__((ext_vector_type(2)));

// Loads this thread's share of chunk rows [k0, k0+GK): rows k0 + (tid>>6) + 4j, columns
// c0 + 2*(tid&63) + {0,1}. A wave reads one contiguous 1-KiB row segment per j (coalesced) and
// later writes it to LDS as one contiguous 1-KiB run (conflict-free ds_write_b128). `full` is
// workgroup-uniform (whole chunk in range, 16-B aligned), so the fast path is branch-free.
__device__ __forceinline__ void gemm_load(d2_t (&r)[4], const double* __restrict__ X, int64_t ld,
                                          int64_t k0, int64_t K, int64_t c0, int64_t cols, bool full) {
    // uniform chunk base and row steps, one per-lane offset
    const double* p = X + k0 * ld + c0;
    const int rl = threadIdx.x >> 6, cl = 2 * (threadIdx.x & 63);
    const int64_t off = (int64_t)rl * ld + cl;
    if (full) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const d2_t*>(p + 4 * j * ld + off);
    } else {
        const int kl = (int)(K - k0 < GK ? K - k0 : GK);
        const int cc = (int)(cols - c0 < GT ? cols - c0 : GT);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double* q = p + 4 * j * ld + off;
            const bool rv = rl + 4 * j < kl;
            r[j].x = (rv && cl < cc) ? q[0] : 0.0;
            r[j].y = (rv && cl + 1 < cc) ? q[1] : 0.0;
        }
    }
}

#ifndef QK_GEMM_STORE
#define QK_GEMM_STORE 1  // 0: per-element stores; 1: paired 16-B nt stores; 2: paired 16-B sc1 stores;
                         // 3: paired 16-B plain stores
// (LDS-DMA kernel, syc 32 5 contraction: nt 66.1 TF/s, sc1 65.4)
#endif

// Swap a 64-bit value with the neighbouring lane (lane ^ 1).
template <typename T>
__device__ __forceinline__ T dpp_swap_pair(T v) {
    static_assert(sizeof(T) == 8, "64-bit values only");
    int2 w = *reinterpret_cast<int2*>(&v);
    w.x = __builtin_amdgcn_mov_dpp(w.x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    w.y = __builtin_amdgcn_mov_dpp(w.y, 0xB1, 0xF, 0xF, false);
    return *reinterpret_cast<T*>(&w);
}

// 16-B store of two adjacent outputs. sc1 (write-through) stores do not keep the line in the
// XCD's L2, so the 2^N output stream does not evict the operand panels other tiles re-read.
__device__ __forceinline__ void gemm_store_pair(double* p, d2_t v) {
#if QK_GEMM_STORE == 2
    // s_nop 1: a >8-B store's data VGPRs must not be rewritten in the next cycle (the hazard
    // recogniser does not see inside inline asm)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
#elif QK_GEMM_STORE == 3
    *reinterpret_cast<d2_t*>(p) = v;
#else
    __builtin_nontemporal_store(v, reinterpret_cast<d2_t*>(p));
#endif
}

__device__ __forceinline__ void gemm_store_out(double* p, double v) {
#if QK_GEMM_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

#ifndef QK_GEMM_PERSIST
#define QK_GEMM_PERSIST 1  // persistent workgroups looping over tiles (stores overlap next tile)
#endif
#ifndef QK_GEMM_WG_PER_CU
#define QK_GEMM_WG_PER_CU 2
#endif

struct GemmArgs {
    int64_t M, N, K;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    const int64_t* __restrict__ keyA;
    int64_t strideA;
    const int64_t* __restrict__ keyB;
    int64_t strideB;
    double* __restrict__ out;
    int beta;
    int64_t tiles_m, tiles_n;
    const int32_t* skip = nullptr;  // DEVICE predicate: the launch does nothing when *skip > 0
};

// predicated launches (qk_gemm_keyed_pred): every workgroup reads the flag and leaves at once
__device__ __forceinline__ bool gemm_skipped(const GemmArgs& g) { return g.skip && *g.skip > 0; }

// Tile sequence index -> (bm, bn): QK_GEMM_GROUP tile rows x all tile columns, row fastest, so
// the ~64 tiles an XCD holds at once span 8 A panels x 8 B panels that stay in its 4 MiB L2.
__device__ __forceinline__ void gemm_tile_coords(int64_t seq, int64_t tiles_m, int64_t tiles_n,
                                                 int64_t& bm, int64_t& bn) {
    // 32-bit arithmetic (host guarantees tiles_m * tiles_n < 2^31): 64-bit division is a long
    // software sequence
    const uint32_t q = (uint32_t)seq, tm = (uint32_t)tiles_m, tn = (uint32_t)tiles_n;
#if QK_GEMM_GROUP
    const uint32_t per_group = (uint32_t)QK_GEMM_GROUP * tn;
    const uint32_t g = q / per_group, r = q - g * per_group;
    const uint32_t first = g * QK_GEMM_GROUP;
    const uint32_t gsize = tm - first < (uint32_t)QK_GEMM_GROUP ? tm - first : (uint32_t)QK_GEMM_GROUP;
    bm = first + r % gsize;
    bn = r / gsize;
#else
    bm = q % tm;
    bn = q / tm;
#endif
}

// Epilogue of one 128x128 tile: f64 16x16 C layout: col = lane & 15, row = (lane >> 4) + 4 * r.
// Output offsets are key(row) + key(col) (keys >= 0; -1 marks a row/column outside the matrix).
// FULL: the tile lies inside M x N and beta == 0 (the glds kernel's contract): no bounds checks,
// so the paired path issues exactly 32 stores per wave (its vmcnt accounting relies on that).
template <bool FULL>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, int64_t m0, int64_t n0, d4_t (&acc)[4][4]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t M = g.M, N = g.N;
    int64_t kcol[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * 64 + j * 16 + (lane & 15);
        kcol[j] = (FULL || col < N) ? (g.keyB ? g.keyB[col] : col * g.strideB) : -1;
    }
#if QK_GEMM_STORE
    // Paired 16-B stores: when every even column's right neighbour is the next output element
    // (key(c+1) = key(c) + 1, e.g. the fragment holding clbit 0 on the N side), lane pairs swap
    // one value (DPP quad_perm [1,0,3,2]) so each lane writes two adjacent outputs of one row.
    bool pairable = FULL || (!g.beta && n0 + GT <= N);
    if (pairable) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t nb = dpp_swap_pair(kcol[j]);
            ok = ok && ((lane & 1) ? nb + 1 == kcol[j] : kcol[j] + 1 == nb);
        }
        pairable = __all(ok);  // wave-uniform
    }
    if (pairable) {
        const bool odd = lane & 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int rp = 0; rp < 4; rp += 2) {
                // even lane writes row rp, odd lane row rp+1, both at the even column's key
                const int rr = rp + (odd ? 1 : 0);
                const int64_t row = m0 + wm * 64 + i * 16 + (lane >> 4) + 4 * rr;
                const int64_t krow = (FULL || row < M) ? (g.keyA ? g.keyA[row] : row * g.strideA) : -1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double x = odd ? acc[i][j][rp] : acc[i][j][rp + 1];
                    const double y = dpp_swap_pair(x);
                    d2_t v;
                    v.x = odd ? y : acc[i][j][rp];
                    v.y = odd ? acc[i][j][rp + 1] : y;
#ifdef QK_GEMM_NOSTORE
                    if (v.x != 1234.5678) continue;
#endif
                    if (FULL || krow >= 0) gemm_store_pair(g.out + krow + kcol[j] - (odd ? 1 : 0), v);
                }
            }
        }
        return;
    }
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int64_t krow[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = m0 + wm * 64 + i * 16 + (lane >> 4) + 4 * r;
            krow[r] = row < M ? (g.keyA ? g.keyA[row] : row * g.strideA) : -1;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#ifdef QK_GEMM_NOSTORE  // tuning experiment only: MFMA + operand traffic without the output
                if (acc[i][j][r] != 1234.5678) continue;
#endif
                if (krow[r] < 0 || kcol[j] < 0) continue;
                double* o = g.out + krow[r] + kcol[j];
                if (g.beta) *o += acc[i][j][r];
                else gemm_store_out(o, acc[i][j][r]);
            }
    }
}

// One 128x128 output tile by one 256-thread workgroup (2x2 waves of 64x64 = 4x4 MFMA 16x16x4
// f64 tiles each). K is streamed in 16-row chunks: the next chunk's global loads are issued into
// registers before the current chunk's MFMAs (software pipeline), LDS is double buffered so a
// chunk costs one barrier. `buf` carries the LDS buffer parity across the tiles of a persistent
// workgroup: the first store of the next tile goes to the buffer the last chunk did not read.
__device__ __forceinline__ bool gemm_vec(const double* X, int64_t ld, int64_t c0, int64_t cols) {
    return ((ld & 1) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) && c0 + GT <= cols;
}

// Chunk 0 of tile (bm, bn) into registers.
__device__ __forceinline__ void gemm_load_first(const GemmArgs& g, int64_t bm, int64_t bn, d2_t (&ra)[4],
                                                d2_t (&rb)[4]) {
    gemm_load(ra, g.A, g.lda, 0, g.K, bm * GT, g.M, gemm_vec(g.A, g.lda, bm * GT, g.M) && GK <= g.K);
    gemm_load(rb, g.B, g.ldb, 0, g.K, bn * GT, g.N, gemm_vec(g.B, g.ldb, bn * GT, g.N) && GK <= g.K);
}

// ra/rb hold chunk 0 of this tile on entry; during the last chunk the next tile's chunk 0 is
// prefetched into them (have_next), so a persistent workgroup never waits on a cold first load.
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int64_t bm, int64_t bn, bool have_next,
                                          int64_t nbm, int64_t nbn, d2_t (&ra)[4], d2_t (&rb)[4],
                                          double (*As)[GK][GT + GPAD], double (*Bs)[GK][GT + GPAD],
                                          int& buf) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t M = g.M, N = g.N, K = g.K;
    const int64_t m0 = bm * GT, n0 = bn * GT;

    d4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (d4_t){0.0, 0.0, 0.0, 0.0};

    const int lr = tid >> 6;        // first chunk row of this thread (rows lr + 4j)
    const int lc = 2 * (tid & 63);  // two columns per thread
    for (int64_t k0 = 0; k0 < K; k0 += GK) {
#ifdef QK_GEMM_NOLDSW  // tuning experiment only: LDS written and synchronised once per tile
        if (k0 == 0)
#endif
        {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            *reinterpret_cast<d2_t*>(&As[buf][lr + 4 * j][lc]) = ra[j];
            *reinterpret_cast<d2_t*>(&Bs[buf][lr + 4 * j][lc]) = rb[j];
        }
        __syncthreads();
        }
        // prefetch the next chunk (this tile's, else chunk 0 of the next tile) during the MFMAs
        const bool more = k0 + GK < K;
#ifdef QK_GEMM_NOLOAD  // tuning experiment only: no operand loads after a tile's first chunk
        if (!more && have_next) {
#else
        if (more || have_next) {
#endif
            const int64_t pk = more ? k0 + GK : 0;
            const int64_t pm = more ? m0 : nbm * GT, pn = more ? n0 : nbn * GT;
            const bool kfull = pk + GK <= K;
            gemm_load(ra, g.A, g.lda, pk, K, pm, M, gemm_vec(g.A, g.lda, pm, M) && kfull);
            gemm_load(rb, g.B, g.ldb, pk, K, pn, N, gemm_vec(g.B, g.ldb, pn, N) && kfull);
        }
#pragma unroll
        for (int kk = 0; kk < GK / 4; ++kk) {
            const int kr2 = kk * 4 + (lane >> 4);
            double fa[4], fb[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fa[t] = As[buf][kr2][wm * 64 + t * 16 + (lane & 15)];
                fb[t] = Bs[buf][kr2][wn * 64 + t * 16 + (lane & 15)];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        buf ^= 1;
    }
    gemm_epilogue<false>(g, m0, n0, acc);
}

// XCD-aware schedule: the dispatcher deals consecutive workgroup ids round-robin over the 8
// XCDs, so each XCD is handed a contiguous eighth of the (grouped) tile sequence. Persistent
// mode launches QK_GEMM_WG_PER_CU workgroups per CU; each walks its XCD's eighth with stride =
// the XCD's workgroup count, so one tile's output stores drain while the next tile's loads and
// MFMAs issue.
__global__ __launch_bounds__(256, 2) void qk_gemm_keyed_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) double As[2][GK][GT + GPAD];
    __shared__ __attribute__((aligned(16))) double Bs[2][GK][GT + GPAD];
    if (gemm_skipped(g)) return;
    const int64_t nblk = g.tiles_m * g.tiles_n;
    int buf = 0;
    int64_t bm, bn;
#if QK_GEMM_PERSIST
    const int64_t G = gridDim.x;  // multiple of 8 when nblk % 8 == 0 (host)
    const bool xcd = nblk % 8 == 0 && G % 8 == 0;
    const int64_t per_xcd = xcd ? nblk / 8 : nblk, stride = xcd ? G / 8 : G;
    const int64_t base = xcd ? (blockIdx.x % 8) * per_xcd : 0;
    int64_t li = xcd ? blockIdx.x / 8 : blockIdx.x;
    if (li >= per_xcd) return;
    d2_t ra[4], rb[4];
    gemm_tile_coords(base + li, g.tiles_m, g.tiles_n, bm, bn);
    gemm_load_first(g, bm, bn, ra, rb);
    for (; li < per_xcd; li += stride) {
        const bool have_next = li + stride < per_xcd;
        int64_t nbm = 0, nbn = 0;
        if (have_next) gemm_tile_coords(base + li + stride, g.tiles_m, g.tiles_n, nbm, nbn);
        gemm_tile(g, bm, bn, have_next, nbm, nbn, ra, rb, As, Bs, buf);
        bm = nbm;
        bn = nbn;
    }
#else
    int64_t bid = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (bid >= nblk) return;
    if (nblk % 8 == 0) bid = (bid % 8) * (nblk / 8) + bid / 8;
    gemm_tile_coords(bid, g.tiles_m, g.tiles_n, bm, bn);
    d2_t ra[4], rb[4];
    gemm_load_first(g, bm, bn, ra, rb);
    gemm_tile(g, bm, bn, false, 0, 0, ra, rb, As, Bs, buf);
#endif
}

// ------------------------------------------------------------------------------------------
// knit contraction, LDS-DMA pipeline (full tiles: M, N multiples of 128, K of 8, beta = 0)
// ------------------------------------------------------------------------------------------
// Every operand row goes global -> LDS directly (global_load_lds_dwordx4: one 1-KiB
// wave-instruction per 128-double row, SGPR row address + the lane's 16-B offset, no staging
// VGPRs, no ds_write), into a ring of G2S stages of G2K k-rows. One raw barrier per stage, the
// waits are counted (vmcnt(N), see gemm_ring_wait), and the MFMA fragments are double-buffered in
// registers so only a stage's first LDS read is exposed. Measured on syc 32 5's 65536^2 x 256
// contraction (tools/gemm_bench.py, random operands): the stage depth is the lever (G2K 4 / 8 / 16
// = 48 / 58-61 / 65 TF/s; more stages in flight at G2K = 8 change nothing), and G2K = 16 with two
// stages is what fits 2 workgroups per CU (73.7 KiB LDS each); the register-staged kernel above
// reaches 60.4 TF/s on the same shape.
#ifndef QK_GEMM_GLDS
#define QK_GEMM_GLDS 1  // full-tile contractions take the LDS-DMA pipeline
#endif
#ifndef QK_G2K
#define QK_G2K 16
#endif
#ifndef QK_G2S
#define QK_G2S 2
#endif
#ifndef QK_GLDS_WG_PER_CU
#define QK_GLDS_WG_PER_CU 2  // persistent workgroups per CU (LDS: 2 x 73.7 KiB at G2K = 16, G2S = 2)
#endif
#ifndef QK_GEMM_PRIO
#define QK_GEMM_PRIO 0  // raise wave priority around each k-step's MFMAs
#endif
constexpr int G2K = QK_G2K;  // k-rows per stage (multiple of 4)
constexpr int G2S = QK_G2S;  // stages in the ring (2 x 36.9 KiB per workgroup, 2 workgroups per CU)
constexpr int G2L = G2K / 2;  // glds per wave per stage (G2K/4 rows of A and of B)

struct GemmRing {
    double a[G2K][GT + GPAD];
    double b[G2K][GT + GPAD];
};

__device__ __forceinline__ void glds16(const double* src, double* lds_row) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                     reinterpret_cast<__attribute__((address_space(3))) void*>(
                                         reinterpret_cast<uintptr_t>(lds_row)),
                                     16, 0, 0);
}

// Wait until at most n of this wave's vector-memory operations are outstanding (n > 63 waits
// for 63: waiting for more is always safe).
__device__ __forceinline__ void gemm_ring_wait(int n) {
#define QK_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define QK_VMW8(k) QK_VMW(k) QK_VMW(k + 1) QK_VMW(k + 2) QK_VMW(k + 3) QK_VMW(k + 4) QK_VMW(k + 5) QK_VMW(k + 6) QK_VMW(k + 7)
    switch (n < 63 ? n : 63) {
        QK_VMW8(0) QK_VMW8(8) QK_VMW8(16) QK_VMW8(24) QK_VMW8(32) QK_VMW8(40) QK_VMW8(48)
        QK_VMW(56) QK_VMW(57) QK_VMW(58) QK_VMW(59) QK_VMW(60) QK_VMW(61) QK_VMW(62) QK_VMW(63)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#undef QK_VMW8
#undef QK_VMW
}

__global__ __launch_bounds__(256, 2) void qk_gemm_glds_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) GemmRing ring[G2S];
    if (gemm_skipped(g)) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int64_t nblk = g.tiles_m * g.tiles_n;
    const int64_t G = gridDim.x;
    const bool xcd = nblk % 8 == 0 && G % 8 == 0;
    const int64_t per_xcd = xcd ? nblk / 8 : nblk, stride = xcd ? G / 8 : G;
    const int64_t base = xcd ? (blockIdx.x % 8) * per_xcd : 0;
    const int64_t li0 = xcd ? blockIdx.x / 8 : blockIdx.x;
    if (li0 >= per_xcd) return;
    const int nct = (int)(g.K / G2K);                                  // stages per tile
    const int ntile = (int)((per_xcd - li0 + stride - 1) / stride);  // tiles of this workgroup
    const int total = ntile * nct;

    // issue side: the (tile, stage) the next glds batch belongs to
    int it = 0, ic = 0, issued = 0;
    int64_t ibm, ibn;
    gemm_tile_coords(base + li0, g.tiles_m, g.tiles_n, ibm, ibn);
    // this wave's two rows of the A and of the B stage, 16 B per lane
    // row addresses are wave-uniform (SGPR base + the lane's 16-B offset): no per-lane 64-bit
    // address arithmetic per load
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    const int src_off = 2 * lane;
    auto issue = [&]() {
        if (issued >= total) return;
        GemmRing& r = ring[issued % G2S];
        const int64_t k0 = (int64_t)ic * G2K;
#pragma unroll
        for (int q = 0; q < G2K / 4; ++q) {
            const int row = wave_s * (G2K / 4) + q;
            const double* pa = g.A + (k0 + row) * g.lda + ibm * GT;
            const double* pb = g.B + (k0 + row) * g.ldb + ibn * GT;
            glds16(pa + src_off, &r.a[row][0]);
            glds16(pb + src_off, &r.b[row][0]);
        }
        ++issued;
        if (++ic == nct) {
            ic = 0;
            ++it;
            if (it < ntile) gemm_tile_coords(base + li0 + (int64_t)it * stride, g.tiles_m, g.tiles_n, ibm, ibn);
        }
    };
    for (int s = 0; s < G2S - 1; ++s) issue();

    d4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (d4_t){0.0, 0.0, 0.0, 0.0};
    int64_t bm, bn;
    gemm_tile_coords(base + li0, g.tiles_m, g.tiles_n, bm, bn);
    int t = 0, c = 0;
    for (int gc = 0; gc < total; ++gc) {
        // VMEM operations this wave issued after stage gc's batch: the later batches in flight
        // (G2L each) and the 32 stores of every tile epilogue issued after it (tiles ending at
        // gc-3..gc-1, all of which followed batch gc)
        int after = G2L * ((total - 1 - gc) < (G2S - 2) ? (total - 1 - gc) : (G2S - 2));
#pragma unroll
        for (int d = 1; d < G2S; ++d)
            if (gc - d >= 0 && (gc - d + 1) % nct == 0) after += 32;
        gemm_ring_wait(after);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage gc landed for all waves; stage gc-1 fully read
        const GemmRing& r = ring[gc % G2S];
        // fragments double-buffered in registers: k-step kk+1's LDS reads are in flight during
        // k-step kk's MFMAs
        double fa[2][4], fb[2][4];
        auto frags = [&](int kk) {
            const int kr = kk * 4 + (lane >> 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                fa[kk & 1][q] = r.a[kr][wm * 64 + q * 16 + (lane & 15)];
                fb[kk & 1][q] = r.b[kr][wn * 64 + q * 16 + (lane & 15)];
            }
        };
        frags(0);  // first fragments in flight while the refill of stage gc-1 is issued
        issue();
#pragma unroll
        for (int kk = 0; kk < G2K / 4; ++kk) {
            if (kk + 1 < G2K / 4) frags(kk + 1);
#if QK_GEMM_PRIO
            __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[kk & 1][i], fb[kk & 1][j], acc[i][j], 0,
                                                                     0, 0);
#if QK_GEMM_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
        }
        if (++c == nct) {
            gemm_epilogue<true>(g, bm * GT, bn * GT, acc);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = (d4_t){0.0, 0.0, 0.0, 0.0};
            c = 0;
            if (++t < ntile) gemm_tile_coords(base + li0 + (int64_t)t * stride, g.tiles_m, g.tiles_n, bm, bn);
        }
    }
}

// ------------------------------------------------------------------------------------------
// knit contraction, wave-private LDS ring (full tiles, K = 4 * NKS, beta = 0)
// ------------------------------------------------------------------------------------------
// No barrier: each wave streams its own 64-row A slice and 64-column B slice of the k-step into
// its own LDS ring (global_load_lds_dwordx4, DW k-steps deep), so the four waves of a workgroup
// never wait for each other and a wave in its store epilogue leaves the SIMD's matrix pipe to its
// partner (the shared-ring kernel above stalls every wave at each stage's barrier). The price is
// that the two waves of a tile row both fetch its A slice (L2 traffic, not HBM).
// Fragment rows are permuted so every LDS read is a conflict-free ds_read_b128: MFMA fragment i
// holds tile rows m = 4 rho + i (rho: the A operand's row, lane & 15), fragment j of B holds
// columns n = 2 rho + (j & 1) + 32 (j >> 1). In the C layout (row rho_r = (lane >> 4) + 4 r,
// column rho) a lane then holds output columns n, n + 1 of fragments 2 jp, 2 jp + 1: one 16-B
// store per (i, r, jp), no lane swap. The tile's 64 row and 64 column keys ride in the ring as
// one more global_load_lds. Waits are counted by hand (the compiler does not count the stores
// in flight and would wait for them at every tile start): see the vmcnt comment in the loop.
#ifndef QK_GEMM_WAVE
#define QK_GEMM_WAVE 1  // K in {16, 32, 64} full-tile contractions take the wave-ring kernel
#endif
#ifndef QK_WAVE_WG_PER_CU
#define QK_WAVE_WG_PER_CU 2  // LDS: 4 waves x (4 x 4 KiB ring + 1 KiB keys) = 68 KiB per workgroup
#endif
constexpr int DW = 4;  // ring depth in k-steps (DW - 1 in flight while one is read)

struct WaveRing {
    double a[DW][4][64];  // k-step slot: 4 k-rows of the wave's 64 A columns (chunk-permuted)
    double b[DW][4][64];  // 4 k-rows of its 64 B columns
    int64_t key[2][64];   // row keys, column keys of the wave's 64 x 64 block
};

__device__ __forceinline__ void glds16_at(const void* src, void* lds_base) {
    __builtin_amdgcn_global_load_lds(src,
                                     reinterpret_cast<__attribute__((address_space(3))) void*>(
                                         reinterpret_cast<uintptr_t>(lds_base)),
                                     16, 0, 0);
}

template <int NKS>
__global__ __launch_bounds__(256, 2) void qk_gemm_wave_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) WaveRing rings[4];
    if (gemm_skipped(g)) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    WaveRing& ring = rings[__builtin_amdgcn_readfirstlane(wave)];
    const int64_t nblk = g.tiles_m * g.tiles_n;
    const int64_t G = gridDim.x;
    const bool xcd = nblk % 8 == 0 && G % 8 == 0;
    const int64_t per_xcd = xcd ? nblk / 8 : nblk, stride = xcd ? G / 8 : G;
    const int64_t base = xcd ? (blockIdx.x % 8) * per_xcd : 0;
    int64_t li = xcd ? blockIdx.x / 8 : blockIdx.x;
    if (li >= per_xcd) return;
    const int64_t lda = g.lda, ldb = g.ldb;
    // load side: lane t carries k-row (t >> 5) (+2 in the second load) and 16-B chunk position
    // p = t & 31 of it; A positions hold chunks 0, 2, .., 30, 1, 3, .., 31 (so a lane's two reads
    // are chunks 2 rho and 2 rho + 1), B positions the chunks in order
    const int p = lane & 31;
    const int chunkA = p < 16 ? 2 * p : 2 * (p - 16) + 1;
    const int64_t offA = (int64_t)(lane >> 5) * lda + wm * 64 + 2 * chunkA;
    const int64_t offB = (int64_t)(lane >> 5) * ldb + wn * 64 + 2 * p;
    // key load: lanes 0-31 two row keys each, lanes 32-63 two column keys (an unkeyed side reads
    // an in-bounds dummy and its keys are computed at the store)
    const int64_t* tabA = g.keyA ? g.keyA : reinterpret_cast<const int64_t*>(g.A);
    const int64_t* tabB = g.keyB ? g.keyB : reinterpret_cast<const int64_t*>(g.B);
    const int64_t keyOff = 2 * (lane & 31);

    int64_t bm, bn;
    gemm_tile_coords(base + li, g.tiles_m, g.tiles_n, bm, bn);
    const double* pa = g.A + bm * GT + offA;
    const double* pb = g.B + bn * GT + offB;
    const double* na = pa;
    const double* nb = pb;
    if (li + stride < per_xcd) {
        int64_t tbm, tbn;
        gemm_tile_coords(base + li + stride, g.tiles_m, g.tiles_n, tbm, tbn);
        na = g.A + tbm * GT + offA;
        nb = g.B + tbn * GT + offB;
    }
    // k-step ks of this tile into ring slot `slot` (ks >= NKS: the next tile's; the last tile's
    // overrun re-reads its own first k-steps: in bounds, never read back). Four VMEM ops.
    auto issue = [&](int slot, int ks) {
        const double* a = ks < NKS ? pa + (int64_t)(4 * ks) * lda : na + (int64_t)(4 * (ks - NKS)) * lda;
        const double* b = ks < NKS ? pb + (int64_t)(4 * ks) * ldb : nb + (int64_t)(4 * (ks - NKS)) * ldb;
        glds16_at(a, &ring.a[slot][0][0]);
        glds16_at(a + 2 * lda, &ring.a[slot][2][0]);
        glds16_at(b, &ring.b[slot][0][0]);
        glds16_at(b + 2 * ldb, &ring.b[slot][2][0]);
    };
#pragma unroll
    for (int s = 0; s < DW - 1; ++s) issue(s, s);

    // stores of the previous tile's epilogue still counted by vmcnt at this tile's first k-steps
    int prev_stores = 0;
    const int rho = lane & 15, kk = lane >> 4;
    auto tile = [&]() -> bool {
        d4_t acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (d4_t){0.0, 0.0, 0.0, 0.0};
        static_assert(NKS % DW == 0, "k-steps per tile must be a multiple of the ring depth");
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            issue((ks + DW - 1) % DW, ks + DW - 1);
            if (ks == 0) {
                const int64_t* t = lane < 32 ? tabA + (g.keyA ? bm * GT + wm * 64 : 0) + keyOff
                                             : tabB + (g.keyB ? bn * GT + wn * 64 : 0) + keyOff;
                glds16_at(t, &ring.key[0][0]);
            }
            // vmcnt: VMEM ops of this wave issued after slot ks's four: the later slots still
            // in flight, this k-step's refill, the key load (issued at k-step 0 after slot 3's
            // refill) and, for the slots filled during the previous tile, its epilogue stores
            //   ks = 0, 1, 2: 13 + prev_stores; ks = 3: 13; ks >= 4: 12 (DW = 4)
            static_assert(DW == 4, "wait counts below are for a 4-deep ring");
            if (ks <= DW - 2) {  // 13 + 0 / 32 / 64 (clamped to the field's 63: waits longer, safe)
                if (prev_stores == 0) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
                else if (prev_stores == 32) asm volatile("s_waitcnt vmcnt(45)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
            } else if (ks == DW - 1) {
                asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            }
            const int s = ks % DW;
            const d2_t a0 = *reinterpret_cast<const d2_t*>(&ring.a[s][kk][2 * rho]);
            const d2_t a1 = *reinterpret_cast<const d2_t*>(&ring.a[s][kk][32 + 2 * rho]);
            const d2_t b0 = *reinterpret_cast<const d2_t*>(&ring.b[s][kk][2 * rho]);
            const d2_t b1 = *reinterpret_cast<const d2_t*>(&ring.b[s][kk][32 + 2 * rho]);
            const double fa[4] = {a0.x, a0.y, a1.x, a1.y};
            const double fb[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[i], fb[j], acc[i][j], 0, 0, 0);
            // the next k-step's refill overwrites this slot's neighbour: keep program order
            __builtin_amdgcn_sched_barrier(0);
        }
        // keys: issued at k-step 0, followed by 4 (NKS - 1) refills
        static_assert(4 * (NKS - 1) <= 63, "vmcnt field");
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NKS - 1)) : "memory");
        const int64_t* keyR = &ring.key[0][0];  // row keys: [0, 64)
        const int64_t* keyC = &ring.key[0][0] + 64;
        // lane's rows m = 4 kk + 16 r + i, columns c_j = 2 rho + (j & 1) + 32 (j >> 1)
        int64_t kr[4][4], kc[4];
        if (g.keyA) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) kr[r][i] = keyR[4 * kk + 16 * r + i];
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) kr[r][i] = (bm * GT + wm * 64 + 4 * kk + 16 * r + i) * g.strideA;
        }
        if (g.keyB) {
#pragma unroll
            for (int j = 0; j < 4; ++j) kc[j] = keyC[2 * rho + (j & 1) + 32 * (j >> 1)];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) kc[j] = (bn * GT + wn * 64 + 2 * rho + (j & 1) + 32 * (j >> 1)) * g.strideB;
        }
        int64_t odd = (kc[0] | kc[2]) & 1;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 4; ++i) odd |= kr[r][i] & 1;
        // wave-uniform; out is 16-B aligned (host)
        const bool pair = __all(kc[1] == kc[0] + 1 && kc[3] == kc[2] + 1 && odd == 0);
        if (pair) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int jp = 0; jp < 2; ++jp) {
                        d2_t v;
                        v.x = acc[i][2 * jp][r];
                        v.y = acc[i][2 * jp + 1][r];
                        gemm_store_pair(g.out + kr[r][i] + kc[2 * jp], v);
                    }
            prev_stores = 32;
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) gemm_store_out(g.out + kr[r][i] + kc[j], acc[i][j][r]);
            prev_stores = 64;
        }
        li += stride;
        if (li >= per_xcd) return false;
        gemm_tile_coords(base + li, g.tiles_m, g.tiles_n, bm, bn);
        pa = na;
        pb = nb;
        if (li + stride < per_xcd) {
            int64_t tbm, tbn;
            gemm_tile_coords(base + li + stride, g.tiles_m, g.tiles_n, tbm, tbn);
            na = g.A + tbm * GT + offA;
            nb = g.B + tbn * GT + offB;
        }
        return true;
    };
    while (tile()) {
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the overrun refills land before the wave ends
}

// ------------------------------------------------------------------------------------------
// small-K contraction (K <= 8): output-write bound — syc 32 1's uncut knit is a K = 1 outer
// product that writes 34 GB from 1 MB of operands. A workgroup takes one output row at a time:
// the row's K values of A are read once (wave-uniform), each lane forms two adjacent outputs from
// 16-B reads of the B rows (L2-resident) and writes them with one 16-B nontemporal store.
// ------------------------------------------------------------------------------------------
constexpr int SK_MAX = 8;
#ifndef QK_SK_U
#define QK_SK_U 4
#endif
constexpr int SK_U = QK_SK_U;  // 512-output chunks per lane iteration

// KEYED: the output column of B column j is keyB[j] (caller contract of qk_gemm_outer_paired:
// keyB[2i + 1] = keyB[2i] + 1 and keyB[2i] even, i.e. the N side holds clbit 0), so each lane's
// two adjacent outputs are still one 16-B store; the key table (512 KiB at N = 2^16) is L2-resident.
template <bool KEYED>
__global__ __launch_bounds__(256) void qk_gemm_smallk_kernel(GemmArgs g) {
    if (gemm_skipped(g)) return;
    const int K = (int)g.K;
    for (int64_t row = blockIdx.x; row < g.M; row += gridDim.x) {
        double a[SK_MAX];
#pragma unroll
        for (int k = 0; k < SK_MAX; ++k) a[k] = k < K ? g.A[k * g.lda + row] : 0.0;
        const int64_t base = g.keyA ? g.keyA[row] : row * g.strideA;
        double* o = g.out + base;
        if ((base & 1) == 0) {  // 16-B aligned row start (wave-uniform)
            // SK_U chunks of 512 outputs per iteration: their B loads are all in flight before
            // the first store issues
            int64_t j0 = 2 * (int64_t)threadIdx.x;
            for (; j0 + 512 * (SK_U - 1) < g.N; j0 += 512 * SK_U) {
                d2_t acc[SK_U];
#pragma unroll
                for (int u = 0; u < SK_U; ++u) acc[u] = (d2_t){0.0, 0.0};
#pragma unroll
                for (int k = 0; k < SK_MAX; ++k) {
                    if (k < K) {
#pragma unroll
                        for (int u = 0; u < SK_U; ++u) {
                            const d2_t b = *reinterpret_cast<const d2_t*>(g.B + k * g.ldb + j0 + 512 * u);
                            acc[u].x = fma(a[k], b.x, acc[u].x);
                            acc[u].y = fma(a[k], b.y, acc[u].y);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < SK_U; ++u) {
                    const int64_t col = KEYED ? g.keyB[j0 + 512 * u] : j0 + 512 * u;
                    __builtin_nontemporal_store(acc[u], reinterpret_cast<d2_t*>(o + col));
                }
            }
            for (int64_t j = j0; j < g.N; j += 512) {
                d2_t acc = {0.0, 0.0};
                for (int k = 0; k < K; ++k) {
                    const d2_t b = *reinterpret_cast<const d2_t*>(g.B + k * g.ldb + j);
                    acc.x = fma(a[k], b.x, acc.x);
                    acc.y = fma(a[k], b.y, acc.y);
                }
                __builtin_nontemporal_store(acc, reinterpret_cast<d2_t*>(o + (KEYED ? g.keyB[j] : j)));
            }
        } else {
            for (int64_t j = threadIdx.x; j < g.N; j += 256) {
                double acc = 0.0;
                for (int k = 0; k < K; ++k) acc = fma(a[k], g.B[k * g.ldb + j], acc);
                __builtin_nontemporal_store(acc, o + (KEYED ? g.keyB[j] : j));
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// small-K knit as a streaming write (two fragments whose clbits cover all N output bits):
// out[o] = sum_k A[k][pext(o, maskA)] * B[k][pext(o, maskB)] for every o < 2^N, walked in output
// order, so each wave's 16-B nontemporal stores form one contiguous 1-KiB run (the keyed kernel
// above scatters a row over 128-B runs 2 KiB apart). Row / column indices come from per-byte pext
// tables in LDS (4 x 256 entries per side). Operands (K x 2^16 fp64 at syc 32 5: 1 MiB per side
// at K = 2) are L2-resident gathers.
// ------------------------------------------------------------------------------------------
#ifndef QK_OS_U
#define QK_OS_U 1  // 16-B stores per lane per iteration (syc 32 5, K = 2: U = 1 / 2 / 4 = 6.4-6.5 /
                   // 6.4-6.5 / 7.3-7.4 ms; 8 workgroups per CU vs 4 / 16 within noise; plain
                   // stores 7.2 ms; torch fill_ of the same 2^32 fp64 = 5.1 ms)
#endif
#ifndef QK_OS_NT
#define QK_OS_NT 1  // nontemporal output stores
#endif
#ifndef QK_OS_WG_PER_CU
#define QK_OS_WG_PER_CU 8
#endif
#ifndef QK_OS_P
#define QK_OS_P 1  // adjacent output pairs per lane (16 * P contiguous bytes per lane); P = 2 / 4: 17 /
                   // 46 ms on syc 32 5 (a wave store no longer covers whole lines), P = 1: 6.3 ms
#endif
constexpr int OS_U = QK_OS_U;
constexpr int OS_P = QK_OS_P;
constexpr int64_t OS_CHUNK = 2 * OS_P * 256 * OS_U;  // outputs per workgroup iteration

struct OuterStreamArgs {
    int nbits, K;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    double* __restrict__ out;
};

__device__ __forceinline__ uint32_t pext32(uint32_t x, uint32_t mask) {
    uint32_t r = 0, bit = 1;
    for (; mask; mask &= mask - 1, bit <<= 1)
        if (x & mask & (~mask + 1)) r |= bit;
    return r;
}

__global__ __launch_bounds__(256) void qk_knit_outer_stream_kernel(OuterStreamArgs a) {
    __shared__ uint32_t tab[2][4][256];  // [side][byte][value] -> that byte's pext contribution
    for (int i = threadIdx.x; i < 4 * 256; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), a.maskA);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), a.maskB);
    }
    __syncthreads();
    const int K = a.K;
    const int64_t total = int64_t(1) << a.nbits;
    for (int64_t c0 = (int64_t)blockIdx.x * OS_CHUNK; c0 < total; c0 += (int64_t)gridDim.x * OS_CHUNK) {
        d2_t v[OS_U * OS_P];
#pragma unroll
        for (int up = 0; up < OS_U * OS_P; ++up) {
            const int u = up / OS_P, pp = up % OS_P;
            const int64_t o = c0 + 512 * OS_P * u + 2 * (OS_P * threadIdx.x + pp);
            const uint32_t x = (uint32_t)o;
            uint32_t row = 0, col = 0;
#pragma unroll
            for (int byte = 0; byte < 4; ++byte) {
                const uint32_t b = (x >> (8 * byte)) & 255;
                row += tab[0][byte][b];
                col += tab[1][byte][b];
            }
            d2_t acc = {0.0, 0.0};
            if (o < total) {
#pragma unroll
                for (int k = 0; k < SK_MAX; ++k) {
                    if (k < K) {
                        const double av = a.A[k * a.lda + row];
                        const d2_t bv = *reinterpret_cast<const d2_t*>(a.B + k * a.ldb + col);
                        acc.x = fma(av, bv.x, acc.x);
                        acc.y = fma(av, bv.y, acc.y);
                    }
                }
            }
            v[up] = acc;
        }
#pragma unroll
        for (int up = 0; up < OS_U * OS_P; ++up) {
            const int u = up / OS_P, pp = up % OS_P;
            const int64_t o = c0 + 512 * OS_P * u + 2 * (OS_P * threadIdx.x + pp);
            if (o < total) {
#if QK_OS_NT
                __builtin_nontemporal_store(v[up], reinterpret_cast<d2_t*>(a.out + o));
#else
                *reinterpret_cast<d2_t*>(a.out + o) = v[up];
#endif
            }
        }
    }
}

// Blocked form of the same knit (the one used for outputs of >= 2^9 entries): the output is cut into
// tasks of 2^TB consecutive entries (TB <= 16); within a task the bits >= TB are fixed, so its A / B
// indices are pext(base) + pext(low bits): two short contiguous index ranges (K x 2^popcount(mask &
// (2^TB - 1)) values each: syc 32 5, K = 2, TB = 16: 2 x 256 per side, 8 KiB). A workgroup stages
// them in LDS once per task and then streams the task's 2^TB outputs with LDS reads only; a lane's
// low-byte pext is hoisted out of the loop (its two output bits 0..7 never change). Each wave's 16-B
// stores cover one 1-KiB run, a task one contiguous 2^(TB+3)-byte block. tools/write_ab:
// 6.5-6.8 TB/s on syc 32 5 (5.0-5.2 ms per 2^32-entry knit), above a grid-stride fill, where the
// per-output L2 gathers of qk_knit_outer_stream_kernel reach 5.25 (6.55 ms).
// Range form: outputs [o_begin, o_begin + o_count) (task-aligned) are written to out[o - o_begin]
// (a rank's contiguous slice of the distribution); kdev (DEVICE int, or NULL) overrides K at run time,
// and K <= 0 there skips the launch's work entirely (predicated knit, no host sync).
// Plain 16-B stores: 4% faster than nontemporal ones for this 34 GB write on the same box (tools/write_ab
// round 3: 6.01 vs 6.26 ms at 16 workgroups per CU; a plain grid-stride fill 6.41, nontemporal 6.75).
#ifndef QK_OB_NT
#define QK_OB_NT 0
#endif
struct OuterBlockedArgs {
    int K, TB;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA, maskB;
    int64_t task_begin, task_end;  // tasks [task_begin, task_end) of 2^TB outputs
    int64_t o_begin;
    const int32_t* kdev;
    double* __restrict__ out;
    int64_t spread;  // task order: the i-th task taken is (i % spread) * (n / spread) + i / spread
};

// BG: the B operand is read from global memory (L2: the task's B indices are one contiguous range
// of B's rows) instead of an LDS stage, for masks whose B range per task is too large to stage (syc
// 32 1: B holds all 16 low output bits, 2^16 values per task, A one value per task).
template <bool BG>
__global__ __launch_bounds__(256) void qk_knit_outer_blocked_kernel(OuterBlockedArgs a) {
    int K = a.K;
    if (a.kdev) {
        const int kd = *a.kdev;
        if (kd <= 0) return;
        K = kd < K ? kd : K;
    }
    __shared__ uint32_t tab[2][2][256];  // pext of bytes 0 / 1 of a task offset, per side
    extern __shared__ double stage[];    // [K][na] of A then (LDS mode) [K][nb] of B
    const uint32_t low = (1u << a.TB) - 1u;
    const uint32_t mAl = a.maskA & low, mBl = a.maskB & low;
    const int na = 1 << __builtin_popcount(mAl), nb = 1 << __builtin_popcount(mBl);
    double* sA = stage;
    double* sB = stage + (int64_t)a.K * na;
    for (int i = threadIdx.x; i < 512; i += 256) {
        const int byte = i >> 8, v = i & 255;
        tab[0][byte][v] = pext32((uint32_t)v << (8 * byte), mAl);
        tab[1][byte][v] = pext32((uint32_t)v << (8 * byte), mBl);
    }
    __syncthreads();
    const uint32_t r0 = tab[0][0][(2 * threadIdx.x) & 255], c0 = tab[1][0][(2 * threadIdx.x) & 255];
    const int iters = (1 << a.TB) / 512;
    const int64_t n_tasks = a.task_end - a.task_begin, per_part = n_tasks / a.spread;
    for (int64_t i = blockIdx.x; i < n_tasks; i += gridDim.x) {
        const int64_t t = a.task_begin + (i % a.spread) * per_part + i / a.spread;
        const uint32_t base = (uint32_t)(t << a.TB);
        const uint32_t ah = pext32(base, a.maskA), bh = pext32(base, a.maskB);
        __syncthreads();  // the previous task's readers are done with the stage
        for (int i = threadIdx.x; i < K * na; i += 256) {
            const int k = i / na;
            sA[i] = a.A[k * a.lda + ah + (i - k * na)];
        }
        if (!BG)
            for (int i = threadIdx.x; i < K * nb; i += 256) {
                const int k = i / nb;
                sB[i] = a.B[k * a.ldb + bh + (i - k * nb)];
            }
        __syncthreads();
        const double* Bg = a.B + bh;
        double* o = a.out + ((int64_t)base - a.o_begin);
#pragma unroll 4
        for (int it = 0; it < iters; ++it) {
            const uint32_t hi = (uint32_t)(2 * it + (threadIdx.x >> 7));  // byte 1 of the task offset
            const uint32_t row = r0 + tab[0][1][hi], col = c0 + tab[1][1][hi];
            d2_t acc = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < SK_MAX; ++k)
                if (k < K) {
                    const double av = sA[k * na + row];
                    const d2_t bv = BG ? *reinterpret_cast<const d2_t*>(Bg + k * a.ldb + col)
                                       : *reinterpret_cast<const d2_t*>(sB + k * nb + col);
                    acc.x = fma(av, bv.x, acc.x);
                    acc.y = fma(av, bv.y, acc.y);
                }
#if QK_OB_NT
            __builtin_nontemporal_store(acc, reinterpret_cast<d2_t*>(o + 512 * it + 2 * threadIdx.x));
#else
            *reinterpret_cast<d2_t*>(o + 512 * it + 2 * threadIdx.x) = acc;
#endif
        }
    }
}

// Rows form of the two-fragment knit (round 4), for masks whose B side holds the low C output bits
// (syc 32 1: B = the 16 low bits, A the 16 high ones, K = 1): the output is cut into pieces of 2^C
// consecutive entries; inside a piece the A index is fixed (pa = pext(piece, maskA >> C)) and the B
// indices are one contiguous run (pb << C .. + 2^C, pb = pext(piece, maskB >> C)). A workgroup holds
// its piece's B run in registers (lane: 2^(C - 9) adjacent pairs per k) and keeps it across the
// pieces it writes while pb stays the same — with a grid of a multiple of the pb count, always, so B
// is read once per workgroup — and multiplies by the piece's K scalars (scalar loads). The stores are
// the blocked kernel's (each wave-store one 1-KiB run, a piece 2^(C+3) contiguous bytes); nothing is
// staged in LDS and nothing re-read from L2 per output, where the B-from-global blocked form read B
// from L2 for every output (syc 32 1: 5.55 ms, 0.77 of HBM, round 4 first measurement).
// Outputs [o_begin, o_begin + o_count), piece-aligned, to out[o - o_begin]; kdev as the blocked kernel.
struct OuterRowsArgs {
    int K;
    const double* __restrict__ A;
    int64_t lda;
    const double* __restrict__ B;
    int64_t ldb;
    uint32_t maskA_hi, maskB_hi;  // the masks shifted right by C
    int64_t piece_begin, piece_end;
    int64_t o_begin;
    const int32_t* kdev;
    double* __restrict__ out;
    int64_t spread;  // piece order: the i-th piece taken is (i % spread) * (n / spread) + i / spread
};

template <int KR, int C>
__global__ __launch_bounds__(256) void qk_knit_outer_rows_kernel(OuterRowsArgs a) {
    constexpr int NP = 1 << (C - 9);  // output pairs per lane per piece
    int K = a.K;
    if (a.kdev) {
        const int kd = *a.kdev;
        if (kd <= 0) return;
        K = kd < K ? kd : K;
    }
    d2_t b[KR][NP];
    int64_t pb_loaded = -1;
    const int64_t n_pieces = a.piece_end - a.piece_begin, per_part = n_pieces / a.spread;
    for (int64_t i = blockIdx.x; i < n_pieces; i += gridDim.x) {
        const int64_t p = a.piece_begin + (i % a.spread) * per_part + i / a.spread;
        const uint32_t pl = (uint32_t)p;
        const int64_t pb = pext32(pl, a.maskB_hi);
        const uint32_t pa = pext32(pl, a.maskA_hi);
        if (pb != pb_loaded) {  // uniform: the piece's B run into registers
            const double* Bp = a.B + (pb << C) + 2 * threadIdx.x;
#pragma unroll
            for (int k = 0; k < KR; ++k)
#pragma unroll
                for (int i = 0; i < NP; ++i)
                    b[k][i] = k < K ? *reinterpret_cast<const d2_t*>(Bp + k * a.ldb + 512 * i) : (d2_t){0.0, 0.0};
            pb_loaded = pb;
        }
        double av[KR];
#pragma unroll
        for (int k = 0; k < KR; ++k) av[k] = k < K ? a.A[k * a.lda + pa] : 0.0;
        double* o = a.out + ((p << C) - a.o_begin) + 2 * threadIdx.x;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            d2_t acc = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < KR; ++k)
                if (k < K) {
                    acc.x = fma(av[k], b[k][i].x, acc.x);
                    acc.y = fma(av[k], b[k][i].y, acc.y);
                }
            *reinterpret_cast<d2_t*>(o + 512 * i) = acc;
        }
    }
}

// log2 outputs per piece of the rows kernel for K terms (B pairs held: K * 2^(C - 9) d2 per lane, at
// most 16: 64 VGPRs), 0 when the masks do not allow it: B must hold output bits 0 .. C-1, the range
// must be piece-aligned, and C >= 11 (4 wave-stores per lane per piece).
static int outer_rows_bits(int64_t K, uint64_t maskB, int align_bits) {
    static const int off = getenv("QKNIT_OB_ROWS") ? atoi(getenv("QKNIT_OB_ROWS")) : 1;
    if (!off || K < 1 || K > 8) return 0;
    const int low = __builtin_ctzll(~maskB);  // contiguous B bits from bit 0
    const int want = K <= 1 ? 13 : (K <= 2 ? 12 : 11);
    return (want <= low && want <= align_bits) ? want : 0;
}

// resident workgroups per CU of a rows-kernel instantiation (its B registers set the occupancy)
template <int KR, int C>
static int outer_rows_per_cu() {
    static int n = [] {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, qk_knit_outer_rows_kernel<KR, C>, 256, 0) != hipSuccess)
            b = 2;
        return b < 1 ? 1 : b;
    }();
    return n;
}

constexpr int64_t OB_STAGE_BYTES = 24 * 1024;  // LDS budget of the blocked kernel's operand stage
constexpr int OB_WG_PER_CU = 64;  // bench, one box: 5.82 ms per write at 64, 5.85 at 32, 5.90 at 16, 6.00 at 8, 5.83 one per task

// Widest task (TB <= 16 and <= align_bits, >= 9: one 512-output iteration) whose operand stage fits
// OB_STAGE_BYTES; 0: none. align_bits = trailing zero bits of the output range's begin and count.
// *b_global: stage only A and read B from global memory — taken when that allows a task of >= 2^14
// outputs while staging both does not (tasks below 2^14 outputs write measurably slower).
int outer_blocked_tile(int nbits, int64_t K, uint64_t maskA, uint64_t maskB, int align_bits, bool* b_global) {
    int top = nbits < 16 ? nbits : 16;
    top = align_bits < top ? align_bits : top;
    // QKNIT_OB_TB (A/B experiments, read at every call): cap the task width
    const char* cap_env = getenv("QKNIT_OB_TB");
    const int cap_tb = cap_env ? atoi(cap_env) : 16;
    top = cap_tb < top ? cap_tb : top;
    int both = 0, aonly = 0;
    for (int tb = top; tb >= 9; --tb) {
        const uint64_t low = (uint64_t(1) << tb) - 1;
        const int64_t sa = 8 * K * (int64_t(1) << __builtin_popcountll(maskA & low));
        const int64_t sb = 8 * K * (int64_t(1) << __builtin_popcountll(maskB & low));
        // B from global: the lane's 16-B reads need an even B range (bit 0 of the output is B's)
        if (!aonly && sa <= OB_STAGE_BYTES && (maskB & 1)) aonly = tb;
        if (!both && sa + sb <= OB_STAGE_BYTES) both = tb;
    }
    // QKNIT_OB_BGLOBAL=1 forces the B-from-global form wherever it applies (A/B experiments)
    static const int force = getenv("QKNIT_OB_BGLOBAL") ? atoi(getenv("QKNIT_OB_BGLOBAL")) : -1;
    *b_global = force >= 0 ? (force > 0 && aonly >= 9) : (both < 14 && aonly >= 14 && aonly > both);
    return *b_global ? aonly : both;
}

__global__ void qk_khatri_rao_kernel(int64_t K, int64_t M, int64_t N, const double* __restrict__ A,
                                     int64_t lda, const double* __restrict__ B, int64_t ldb,
                                     double* __restrict__ out) {
    const int64_t MN = M * N, total = K * MN;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = e / MN, c = e - k * MN, j = c / M, i = c - j * M;
        out[e] = A[k * lda + i] * B[k * ldb + j];
    }
}

__global__ void qk_gather_rows_kernel(int64_t R, int64_t width, const int64_t* __restrict__ idx,
                                      const double* __restrict__ coef, const double* __restrict__ src,
                                      double* __restrict__ dst) {
    const int64_t total = R * width;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / width, x = e - r * width;
        dst[e] = coef[r] * src[idx[r] * width + x];
    }
}

unsigned grid_for(int64_t total, int threads) {
    int64_t b = (total + threads - 1) / threads;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (unsigned)b;
}

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

const char* qk_version(void) { return "qknit 0.1 gfx950"; }

// CUs a stream may run on: the popcount of its CU mask (hipExtStreamCreateWithCUMask), or every CU
// of the device for unmasked streams / the null stream.
static int stream_cus(hipStream_t s, int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1)
        cus = 1;
    uint32_t mask[32] = {0};
    if (s && hipExtStreamGetCUMask(s, 32, mask) == hipSuccess) {
        int n = 0;
        for (uint32_t w : mask) n += __builtin_popcount(w);
        if (n > 0 && n < cus) return n;
    }
    return cus;
}

int qk_ctx_create(int device, qk_ctx** out) {
    if (!out) return QK_EARG;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return QK_EHIP;
    qk_ctx* c = new qk_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return QK_EHIP;
    }
    c->stream = c->own;
    c->cus = stream_cus(c->own, device);
    *out = c;
    return QK_OK;
}

int qk_ctx_destroy(qk_ctx* ctx) {
    if (!ctx) return QK_EARG;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->own);
    (void)hipStreamDestroy(ctx->own);
    delete ctx;
    return QK_OK;
}

int qk_ctx_set_stream(qk_ctx* ctx, void* s) {
    if (!ctx) return QK_EARG;
    if ((hipStream_t)s != ctx->stream || s == nullptr) ctx->cus = stream_cus((hipStream_t)s, ctx->device);
    ctx->stream = (hipStream_t)s;  // NULL = the device's null stream (torch's default stream)
    return QK_OK;
}

int qk_stream_create_cu_masked(int device, const uint32_t* cu_mask, int mask_words, void** stream) {
    if (!stream || !cu_mask || mask_words < 1 || mask_words > 32) return QK_EARG;
    *stream = nullptr;
    if (hipSetDevice(device) != hipSuccess) return QK_EHIP;
    int n = 0;
    for (int w = 0; w < mask_words; ++w) n += __builtin_popcount(cu_mask[w]);
    if (n == 0) return QK_EARG;
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask) != hipSuccess) return QK_EHIP;
    *stream = s;
    return QK_OK;
}

int qk_stream_destroy(void* stream) {
    if (!stream) return QK_EARG;
    (void)hipStreamSynchronize((hipStream_t)stream);
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? QK_OK : QK_EHIP;
}

int qk_stream_cu_count(int device, void* stream, int* cus) {
    if (!cus) return QK_EARG;
    *cus = stream_cus((hipStream_t)stream, device);
    return QK_OK;
}

int qk_ctx_synchronize(qk_ctx* ctx) {
    if (!ctx) return QK_EARG;
    QK_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return QK_OK;
}

const char* qk_last_error(qk_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int qk_sweep_workspace_bytes(const qk_program* p, int64_t n_jobs, int64_t* bytes) {
    if (!p || !bytes || n_jobs < 0) return QK_EARG;
    *bytes = p->packed ? 0 : n_jobs * ((int64_t)1 << p->n) * (int64_t)sizeof(double2);
    return QK_OK;
}

int qk_sweep(qk_ctx* ctx, const qk_program* p, int64_t n_jobs, const double* job_slots,
             const double* job_sign, void* workspace, int64_t workspace_bytes, double* pjob) {
    if (!ctx) return QK_EARG;
    if (!p || !p->passes || p->n_passes < 1) return fail(ctx, QK_EARG, "qk_sweep: empty program%s");
    if (n_jobs <= 0) return QK_OK;
    if (!job_sign || !pjob || (p->n_slots > 0 && !job_slots))
        return fail(ctx, QK_EARG, "qk_sweep: null buffer%s");
    if (p->m < 0 || p->m > p->n_eff || p->n_eff > 40)
        return fail(ctx, QK_EARG, "qk_sweep: bad widths%s");
    if (p->packed) {
        if (p->n_eff < QK_FIBER_BITS || p->n_eff > QK_TILE_BITS || p->n_passes != 1)
            return fail(ctx, QK_EARG, "qk_sweep: bad PACKED program%s");
    } else {
        if (p->n <= QK_TILE_BITS || p->n_eff != p->n) return fail(ctx, QK_EARG, "qk_sweep: bad SPLIT program%s");
        int64_t need = 0;
        qk_sweep_workspace_bytes(p, n_jobs, &need);
        if (!workspace || workspace_bytes < need) return fail(ctx, QK_EARG, "qk_sweep: workspace too small%s");
    }
    if (!(p->passes[p->n_passes - 1].flags & 2) || !(p->passes[0].flags & 1))
        return fail(ctx, QK_EARG, "qk_sweep: first pass must INIT and last must be FINAL%s");
    QK_HIP(ctx, hipSetDevice(ctx->device));
    SweepArgs a{};
    a.ops = p->ops;
    a.groups = p->groups;
    a.mats = p->mats;
    a.job_slots = job_slots;
    a.job_sign = job_sign;
    a.state = (double2*)workspace;
    a.pjob = pjob;
    a.n_jobs = n_jobs;
    a.n = p->n;
    a.n_eff = p->n_eff;
    a.m = p->m;
    a.n_slots = p->n_slots;
    for (int ip = 0; ip < p->n_passes; ++ip) {
        const qk_pass& ps = p->passes[ip];
        if (!p->packed && __builtin_popcountll(ps.tile_mask) != QK_TILE_BITS)
            return fail(ctx, QK_EARG, "qk_sweep: SPLIT tile must hold 12 state bits%s");
        a.tile_mask = ps.tile_mask;
        a.group_begin = ps.group_begin;
        a.group_end = ps.group_end;
        a.flags = ps.flags;
        a.traced_local = ps.traced_local;
        // A SPLIT INIT pass that is not also FINAL only needs the tile holding |0..0> of each job
        // (every other tile is zero and stays zero); the next pass then treats the elements
        // outside that tile as known zeros instead of reading them.
        const uint64_t nmask = (p->n >= 64) ? ~0ull : ((1ull << p->n) - 1);
        a.init_sparse = (!p->packed && ip == 0 && p->n_passes > 1) ? 1 : 0;
        a.zero_mask = (!p->packed && ip == 1) ? (nmask & ~p->passes[0].tile_mask) : 0;
        if (p->packed) {
            const int64_t per = (int64_t)1 << (QK_TILE_BITS - p->n_eff);
            const int64_t blocks = (n_jobs + per - 1) / per;
            if (blocks > 0x7fffffff) return fail(ctx, QK_EARG, "qk_sweep: too many jobs%s");
            hipLaunchKernelGGL(qk_sweep_pass_kernel<true>, dim3((unsigned)blocks), dim3(NT), 0, ctx->stream, a,
                               a.ops, a.groups, a.mats);
        } else {
            const int64_t blocks = a.init_sparse ? n_jobs : (n_jobs << (p->n - QK_TILE_BITS));
            if (blocks > 0x7fffffff) return fail(ctx, QK_EARG, "qk_sweep: too many tiles%s");
            hipLaunchKernelGGL(qk_sweep_pass_kernel<false>, dim3((unsigned)blocks), dim3(NT), 0, ctx->stream, a,
                               a.ops, a.groups, a.mats);
        }
        QK_HIP(ctx, hipGetLastError());
    }
    return QK_OK;
}

int qk_reduce_labels(qk_ctx* ctx, int64_t n_labels, const int64_t* offsets, int64_t width,
                     const double* pjob, double* q) {
    if (!ctx) return QK_EARG;
    if (n_labels < 0 || width < 0) return fail(ctx, QK_EARG, "qk_reduce_labels: negative size%s");
    if (n_labels == 0 || width == 0) return QK_OK;
    if (!offsets || !pjob || !q) return fail(ctx, QK_EARG, "qk_reduce_labels: null buffer%s");
    QK_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(qk_reduce_labels_kernel, dim3(grid_for(n_labels * width, 256)), dim3(256), 0,
                       ctx->stream, n_labels, offsets, width, pjob, q);
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_gemm_keyed(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                  const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                  const int64_t* keyB, int64_t strideB, double* out, int beta) {
    return qk_gemm_keyed_pred(ctx, M, N, K, A, lda, B, ldb, keyA, strideA, keyB, strideB, out, beta, nullptr);
}

int qk_gemm_keyed_pred(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                       const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                       const int64_t* keyB, int64_t strideB, double* out, int beta, const int32_t* skip) {
    if (!ctx) return QK_EARG;
    if (M < 0 || N < 0 || K < 0) return fail(ctx, QK_EARG, "qk_gemm_keyed: negative size%s");
    if (M == 0 || N == 0) return QK_OK;
    if (!out || (K > 0 && (!A || !B))) return fail(ctx, QK_EARG, "qk_gemm_keyed: null buffer%s");
    if (lda < M || ldb < N) return fail(ctx, QK_EARG, "qk_gemm_keyed: leading dimension too small%s");
    const int64_t tm = (M + GT - 1) / GT, tn = (N + GT - 1) / GT;
    const int64_t nblk = tm * tn;
    QK_HIP(ctx, hipSetDevice(ctx->device));
    if (nblk >= (int64_t(1) << 31)) return fail(ctx, QK_EARG, "qk_gemm_keyed: too many tiles%s");
    GemmArgs g{M, N, K, A, lda, B, ldb, keyA, strideA, keyB, strideB, out, beta, tm, tn, skip};
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0 &&
                           (lda % 2) == 0 && (ldb % 2) == 0;
    if (K >= 1 && K <= SK_MAX && !beta && !keyB && strideB == 1 && N % 2 == 0 && aligned16 &&
        (reinterpret_cast<uintptr_t>(out) & 15) == 0 && M * N >= (int64_t(1) << 16)) {
        const int cus = ctx->cus;
        const int64_t G = M < (int64_t)cus * 8 ? M : (int64_t)cus * 8;
        hipLaunchKernelGGL(qk_gemm_smallk_kernel<false>, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
        QK_HIP(ctx, hipGetLastError());
        return QK_OK;
    }
    if (QK_GEMM_WAVE && !beta && M % GT == 0 && N % GT == 0 && (K == 16 || K == 32 || K == 64) && aligned16 &&
        ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(keyA) | reinterpret_cast<uintptr_t>(keyB)) &
         15) == 0) {
        const int cus = ctx->cus;
        int64_t G = (int64_t)cus * QK_WAVE_WG_PER_CU;
        G = G < 8 ? 8 : G - G % 8;
        if (G > nblk) G = nblk;
        if (K == 16) hipLaunchKernelGGL(qk_gemm_wave_kernel<4>, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
        else if (K == 32) hipLaunchKernelGGL(qk_gemm_wave_kernel<8>, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
        else hipLaunchKernelGGL(qk_gemm_wave_kernel<16>, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
        QK_HIP(ctx, hipGetLastError());
        return QK_OK;
    }
    if (QK_GEMM_GLDS && !beta && M % GT == 0 && N % GT == 0 && K % G2K == 0 && K > 0 && aligned16) {
        const int cus = ctx->cus;
        int64_t G = (int64_t)cus * QK_GLDS_WG_PER_CU;
        G = G < 8 ? 8 : G - G % 8;
        if (G > nblk) G = nblk;
        hipLaunchKernelGGL(qk_gemm_glds_kernel, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
        QK_HIP(ctx, hipGetLastError());
        return QK_OK;
    }
#if QK_GEMM_PERSIST
    const int cus = ctx->cus;
    int64_t G = (int64_t)cus * QK_GEMM_WG_PER_CU;
    G = G < 8 ? 8 : G - G % 8;
    if (G > nblk) G = nblk;
    hipLaunchKernelGGL(qk_gemm_keyed_kernel, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
#else
    // grid.x * blockDim.x must stay below 2^32 work-items: spill tiles into grid.y
    const int64_t gx = nblk < (1 << 20) ? nblk : (1 << 20);
    const int64_t gy = (nblk + gx - 1) / gx;
    if (gy > 65535) return fail(ctx, QK_EARG, "qk_gemm_keyed: too many tiles%s");
    hipLaunchKernelGGL(qk_gemm_keyed_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, ctx->stream, g);
#endif
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_gemm_outer_paired(qk_ctx* ctx, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda,
                         const double* B, int64_t ldb, const int64_t* keyA, int64_t strideA,
                         const int64_t* keyB, double* out) {
    if (!ctx) return QK_EARG;
    if (M < 0 || N < 0 || K < 1 || K > SK_MAX) return fail(ctx, QK_EARG, "qk_gemm_outer_paired: bad size%s");
    if (M == 0 || N == 0) return QK_OK;
    if (!out || !A || !B || !keyB) return fail(ctx, QK_EARG, "qk_gemm_outer_paired: null buffer%s");
    if (lda < M || ldb < N) return fail(ctx, QK_EARG, "qk_gemm_outer_paired: leading dimension too small%s");
    if ((N & 1) || (ldb & 1) || ((reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(out)) & 15))
        return fail(ctx, QK_EARG, "qk_gemm_outer_paired: N, ldb even and 16-B aligned B/out required%s");
    GemmArgs g{M, N, K, A, lda, B, ldb, keyA, strideA, keyB, 0, out, 0, 0, 0};
    QK_HIP(ctx, hipSetDevice(ctx->device));
    const int cus = ctx->cus;
    const int64_t G = M < (int64_t)cus * 8 ? M : (int64_t)cus * 8;
    hipLaunchKernelGGL(qk_gemm_smallk_kernel<true>, dim3((unsigned)G), dim3(256), 0, ctx->stream, g);
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_knit_outer_stream(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B,
                         int64_t ldb, uint64_t maskA, uint64_t maskB, double* out) {
    if (!ctx) return QK_EARG;
    if (nbits < 2 || nbits > 32) return fail(ctx, QK_EARG, "qk_knit_outer_stream: need 2 <= nbits <= 32%s");
    return qk_knit_outer_stream_range(ctx, nbits, K, A, lda, B, ldb, maskA, maskB, 0, int64_t(1) << nbits,
                                      nullptr, out);
}

int qk_knit_outer_stream_range(qk_ctx* ctx, int nbits, int64_t K, const double* A, int64_t lda, const double* B,
                               int64_t ldb, uint64_t maskA, uint64_t maskB, int64_t o_begin, int64_t o_count,
                               const int32_t* k_dev, double* out) {
    if (!ctx) return QK_EARG;
    if (nbits < 2 || nbits > 32 || K < 1 || K > SK_MAX)
        return fail(ctx, QK_EARG, "qk_knit_outer_stream: need 2 <= nbits <= 32, 1 <= K <= 8%s");
    const uint64_t full = (uint64_t(1) << nbits) - 1;
    if ((maskA & maskB) || (maskA | maskB) != full || !(maskB & 1))
        return fail(ctx, QK_EARG, "qk_knit_outer_stream: masks must be disjoint, cover all bits, bit 0 in B%s");
    if (!out || !A || !B) return fail(ctx, QK_EARG, "qk_knit_outer_stream: null buffer%s");
    const int64_t M = int64_t(1) << __builtin_popcountll(maskA), N = int64_t(1) << __builtin_popcountll(maskB);
    if (lda < M || ldb < N || (ldb & 1) || ((reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(out)) & 15))
        return fail(ctx, QK_EARG, "qk_knit_outer_stream: leading dimension / alignment%s");
    if (o_begin < 0 || o_count < 0 || o_begin + o_count > (int64_t(1) << nbits))
        return fail(ctx, QK_EARG, "qk_knit_outer_stream: output range outside 0..2^nbits%s");
    if (o_count == 0) return QK_OK;
    QK_HIP(ctx, hipSetDevice(ctx->device));
    const int cus = ctx->cus;
    const int align = __builtin_ctzll((uint64_t)(o_begin | o_count));
    if (const int rc = outer_rows_bits(K, maskB, align)) {
        const int64_t pieces = o_count >> rc;
        // a grid of a multiple of the pb count (2^(|maskB| - C)) keeps every workgroup on one B run
        const int64_t nb = int64_t(1) << (__builtin_popcountll(maskB) - rc);
        const int per_cu = K <= 1 ? outer_rows_per_cu<1, 13>() : K <= 2 ? outer_rows_per_cu<2, 12>()
                           : K <= 4 ? outer_rows_per_cu<4, 11>() : outer_rows_per_cu<8, 11>();
        int64_t G = (int64_t)cus * per_cu;
        if (G >= nb) G -= G % nb;
        if (G > pieces) G = pieces;
        // piece order as the blocked kernel's task order (8 far-apart parts at once); a workgroup keeps
        // its B run when the grid is a multiple of 8 x the run count (then i % 8 and the run of i / 8 are
        // the same for all of its pieces). QKNIT_OR_SPREAD (A/B, read per launch) sets the part count.
        const char* rs_env = getenv("QKNIT_OR_SPREAD");
        int64_t spread = rs_env ? atoll(rs_env) : 8;
        if (spread < 1 || pieces % spread || G % (spread * nb) || pieces < 4 * G) spread = 1;
        OuterRowsArgs r{(int)K, A, lda, B, ldb, (uint32_t)(maskA >> rc), (uint32_t)(maskB >> rc), o_begin >> rc,
                        (o_begin >> rc) + pieces, o_begin, k_dev, out, spread};
        const dim3 grid((unsigned)(G < 1 ? 1 : G));
        if (K <= 1) {
            hipLaunchKernelGGL((qk_knit_outer_rows_kernel<1, 13>), grid, dim3(256), 0, ctx->stream, r);
        } else if (K <= 2) {
            hipLaunchKernelGGL((qk_knit_outer_rows_kernel<2, 12>), grid, dim3(256), 0, ctx->stream, r);
        } else if (K <= 4) {
            hipLaunchKernelGGL((qk_knit_outer_rows_kernel<4, 11>), grid, dim3(256), 0, ctx->stream, r);
        } else {
            hipLaunchKernelGGL((qk_knit_outer_rows_kernel<8, 11>), grid, dim3(256), 0, ctx->stream, r);
        }
        QK_HIP(ctx, hipGetLastError());
        return QK_OK;
    }
    bool bg = false;
    const int tb = outer_blocked_tile(nbits, K, maskA, maskB, align, &bg);
    if (tb) {
        const uint64_t low = (uint64_t(1) << tb) - 1;
        const size_t stage = 8 * (size_t)K * ((size_t(1) << __builtin_popcountll(maskA & low)) +
                                              (bg ? 0 : (size_t(1) << __builtin_popcountll(maskB & low))));
        const int64_t tasks = o_count >> tb;
        // workgroups per CU of the grid-stride launch; QKNIT_OB_WG_PER_CU=0: one workgroup per task
        // (workgroups retire as they finish, so work on other streams can take their slots)
        const char* wgpc_env = getenv("QKNIT_OB_WG_PER_CU");  // read at every launch (A/B experiments)
        const int wgpc = wgpc_env ? atoi(wgpc_env) : OB_WG_PER_CU;
        const int64_t G0 = wgpc > 0 ? (int64_t)cus * wgpc : tasks;
        // Task order: with >= 4 tasks per workgroup the i-th task taken is (i % 8) x (tasks / 8) + i / 8, so
        // consecutive workgroups write 8 far-apart parts of the range at once: 1% faster on syc 32 5's
        // 2^32 outputs (4.82-4.90 vs 4.85-4.96 ms on each of 4 buffers, tools/out_mapping_tb.py), slower
        // for one-task-per-workgroup slices (0.80 vs 0.75 ms at 2^29, tools/slice_write_bench.py).
        // QKNIT_OB_SPREAD (A/B experiments, read per launch) sets the part count.
        const char* spread_env = getenv("QKNIT_OB_SPREAD");
        int64_t spread = spread_env ? atoll(spread_env) : (tasks >= 4 * G0 ? 8 : 1);
        if (spread < 1 || tasks % spread) spread = 1;
        OuterBlockedArgs b{(int)K, tb, A, lda, B, ldb, (uint32_t)maskA, (uint32_t)maskB, o_begin >> tb,
                           (o_begin >> tb) + tasks, o_begin, k_dev, out, spread};
        const dim3 grid((unsigned)(tasks < G0 ? tasks : G0));
        if (bg)
            hipLaunchKernelGGL(qk_knit_outer_blocked_kernel<true>, grid, dim3(256), stage, ctx->stream, b);
        else
            hipLaunchKernelGGL(qk_knit_outer_blocked_kernel<false>, grid, dim3(256), stage, ctx->stream, b);
        QK_HIP(ctx, hipGetLastError());
        return QK_OK;
    }
    if (o_begin != 0 || o_count != (int64_t(1) << nbits) || k_dev)
        return fail(ctx, QK_EARG, "qk_knit_outer_stream: output ranges / device K need task-aligned ranges of >= 2^9%s");
    const int64_t chunks = (int64_t(1) << nbits) / OS_CHUNK;
    const int64_t G0 = (int64_t)cus * QK_OS_WG_PER_CU;
    const int64_t G = chunks < 1 ? 1 : (chunks < G0 ? chunks : G0);
    OuterStreamArgs a{nbits, (int)K, A, lda, B, ldb, (uint32_t)maskA, (uint32_t)maskB, out};
    hipLaunchKernelGGL(qk_knit_outer_stream_kernel, dim3((unsigned)G), dim3(256), 0, ctx->stream, a);
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_knit_outer_stream_kind(int nbits, int64_t K, uint64_t maskA, uint64_t maskB, int64_t o_begin,
                              int64_t o_count, int* kind, int* task_bits) {
    if (!kind || !task_bits || nbits < 2 || nbits > 32 || K < 1 || K > SK_MAX || o_count <= 0) return QK_EARG;
    const int align = __builtin_ctzll((uint64_t)(o_begin | o_count));
    if (const int rc = outer_rows_bits(K, maskB, align)) {
        *kind = 3;
        *task_bits = rc;
        return QK_OK;
    }
    bool bg = false;
    const int tb = outer_blocked_tile(nbits, K, maskA, maskB, align, &bg);
    *kind = tb ? (bg ? 2 : 1) : 0;
    *task_bits = tb;
    return QK_OK;
}

int qk_khatri_rao(qk_ctx* ctx, int64_t K, int64_t M, int64_t N, const double* A, int64_t lda,
                  const double* B, int64_t ldb, double* out) {
    if (!ctx) return QK_EARG;
    if (K < 0 || M < 0 || N < 0) return fail(ctx, QK_EARG, "qk_khatri_rao: negative size%s");
    if (K == 0 || M == 0 || N == 0) return QK_OK;
    if (!A || !B || !out) return fail(ctx, QK_EARG, "qk_khatri_rao: null buffer%s");
    QK_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(qk_khatri_rao_kernel, dim3(grid_for(K * M * N, 256)), dim3(256), 0, ctx->stream, K,
                       M, N, A, lda, B, ldb, out);
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

int qk_gather_rows(qk_ctx* ctx, int64_t R, int64_t width, const int64_t* idx, const double* coef,
                   const double* src, double* dst) {
    if (!ctx) return QK_EARG;
    if (R < 0 || width < 0) return fail(ctx, QK_EARG, "qk_gather_rows: negative size%s");
    if (R == 0 || width == 0) return QK_OK;
    if (!idx || !coef || !src || !dst) return fail(ctx, QK_EARG, "qk_gather_rows: null buffer%s");
    QK_HIP(ctx, hipSetDevice(ctx->device));
    hipLaunchKernelGGL(qk_gather_rows_kernel, dim3(grid_for(R * width, 256)), dim3(256), 0, ctx->stream, R,
                       width, idx, coef, src, dst);
    QK_HIP(ctx, hipGetLastError());
    return QK_OK;
}

}  // extern "C"
