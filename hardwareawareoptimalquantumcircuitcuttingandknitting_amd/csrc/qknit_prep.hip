// qknit_prep.hip — the data-rank step's operand preparation in three launches.
//
// Per step, the two-fragment knit R = A^T B needs, from the swept instance rows q_s [R_s][N_s]:
//   X_s = W_s^T q_s            [K][N_s]  the light-cone operands (W_s: [R_s][K] transform),
//   G_s = X_s X_s^T            [K][K]    their Gram matrices (qk_rank_factors' input),
//   U   = X_B P^T              [K][16]   the B operand against the 16 fixed Gaussian probes P [16][N_B],
// and, once qk_rank_factors has the factors T_A, T_B ([rmax][K]), the compressed operands
//   A'' = T_A X_A, B'' = T_B X_B  [rmax][N_s]  the write kernel streams from.
//
// qk_prep_operands_kernel does the first three in one pass over q: a workgroup (8 waves) takes
// 128-column tiles of both sides; each wave forms 16 columns of X with f64 MFMAs (16x16x4, K over
// the instance rows), the tile goes to LDS once, and the same workgroup adds the tile's Gram block
// (and, on the B side, its probe products) into register accumulators. Per-workgroup partial sums
// go to a workspace that qk_prep_reduce_kernel sums in workgroup order (deterministic, no atomics).
// Bound: fp64 MFMA and the stage loads' latency (syc 32 5 after row pruning, 65 swept rows per side: 1.1
// GFLOP of transforms + 0.8 of Grams (the 10 upper 16 x 16 blocks) and probe products, ~0.2 GB of HBM).
// qk_compress_kernel forms A'' / B'' (one column per thread, T in LDS): HBM-bound on reading X.
//
// The acceptance check (qk_probe_errors / qk_probe_accept) runs on the real operands, as the probe
// products would in torch, but without materialising them: V = B'' P^T ([rmax][16], MFMA, per-
// workgroup partials), then per column c of A: d_c = X_A[:, c]^T U - A''[:, c]^T V (the row c of
// (R - A''^T B'') P^T, formed by 16x16x4 MFMAs over K and then rmax) and e_p += d_{c,p}^2; the sums
// give ||(R - A''^T B'') p_j||^2 per probe. Forming T_A^T T_B first would square the factors'
// condition (their entries carry L^{-1}); A'' and B'' are balanced, so this keeps the fp64 floor.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "internal.h"

namespace {

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef double d2_t __attribute__((ext_vector_type(2)));

constexpr int PK = 64;          // largest K (light-cone terms)
constexpr int PCT = 128;        // columns per tile (8 waves x 16)
constexpr int PNP = 16;         // probes
constexpr int PTH = 512;        // threads per workgroup
constexpr int XLD = PCT + 2;    // X tile row stride (doubles): a Gram k-step's 16 rows x 2 columns hit distinct banks
// One workgroup's partial sums: the Gram's 10 upper 16 x 16 blocks (bi <= bj; the reduction mirrors the
// lower ones), and on the B side the probe products after them. Round 4 stored all 16 blocks and a zero
// U on the A side: 80 KiB per workgroup, 41 MiB per syc 32 5 step written and read back, now 48 KiB
constexpr int PG_BLK = 10;
constexpr int PPG = PG_BLK * 256;
constexpr int PPA = PPG;              // doubles of one A-side partial
constexpr int PPB = PPG + PK * PNP;   // doubles of one B-side partial
__host__ __device__ constexpr int prep_tri(int bi, int bj) { return bi * 4 - bi * (bi - 1) / 2 + (bj - bi); }

struct PrepSide {
    const double* Wt;  // [R][K]
    const double* q;   // [R][ldq], columns [0, N)
    int64_t ldq;
    int64_t N;
    int R;
    double* X;         // [K][N]
    const double* P;   // probes [16][N] (B side) or nullptr
};

struct PrepArgs {
    PrepSide s[2];
    int K;
    int split;     // 1: even workgroups take side 0's tiles, odd ones side 1's (prep_grid)
    double* part;  // [gridDim.x][PPA] (A side), then [gridDim.x][PPB] (B side)
};

// Stage ring of the transform phase: PRS instance rows of q (128 columns) and of Wt per stage, moved
// global -> LDS by global_load_lds (16 B per lane, no staging VGPRs); PNS stages in flight per
// workgroup (2 x 28.7 KiB) and two workgroups per CU cover the HBM latency. The ring and the X tile
// share the LDS (66.5 KiB per workgroup).
#ifndef QK_PREP_RS
#define QK_PREP_RS 16
#endif
constexpr int PRS = QK_PREP_RS;  // instance rows per stage (PRS / 4 MFMA k-steps; PRS / 8 rows loaded per wave)
constexpr int PRPW = PRS / 8;
static_assert(PRS % 8 == 0 && PRS >= 8, "stage rows: a multiple of 8 (8 waves)");
// tools/prep_bench.py, syc 32 5 shapes: 2 stages x 2 workgroups per CU 134 us; 1 workgroup per CU with
// 3 / 4 / 5 stages 167 / 160 / 160 us (the wider ring does not help: latency hiding needs more waves)
#ifndef QK_PREP_NS
#define QK_PREP_NS 2
#endif
#ifndef QK_PREP_WG_PER_CU
#define QK_PREP_WG_PER_CU 2  // 512-thread workgroups per CU (2 needs QK_PREP_NS <= 2: the LDS)
#endif
#ifndef QK_COMPRESS_COLS
#define QK_COMPRESS_COLS 1  // qk_compress_cols_kernel where the shapes allow (0: the K-split kernel)
#endif
#ifndef QK_PREP_EXP
#define QK_PREP_EXP 0  // tools/ timing experiments only: 1 skips the Gram phase, 2 the X store, 4 the transform
#endif
constexpr int PNS = QK_PREP_NS;  // stages in flight
#ifndef QK_PREP_QPAD
#define QK_PREP_QPAD 16
#endif
#ifndef QK_PREP_WPAD
#define QK_PREP_WPAD 16
#endif
constexpr int QLD = PCT + QK_PREP_QPAD;  // q stage row stride (doubles): rows 32 banks apart, a k-step's reads conflict-free
constexpr int WLD = PK + QK_PREP_WPAD;   // Wt stage row stride (same)
struct PrepStage {
    double q[PRS][QLD];
    double w[PRS][WLD];
};
union PrepLds {
    PrepStage st[PNS];
    double x[PK][XLD];
};

__device__ __forceinline__ void prep_glds(const double* src, double* lds_row) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                     reinterpret_cast<__attribute__((address_space(3))) void*>(
                                         reinterpret_cast<uintptr_t>(lds_row)),
                                     16, 0, 0);
}

// s_waitcnt vmcnt(n) for a run-time n (n > 15 waits for 15: always safe, only later loads in flight)
__device__ __forceinline__ void prep_vmwait(int n) {
    switch (n < 15 ? n : 15) {
#define QK_PW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
        QK_PW(0) QK_PW(1) QK_PW(2) QK_PW(3) QK_PW(4) QK_PW(5) QK_PW(6) QK_PW(7)
        QK_PW(8) QK_PW(9) QK_PW(10) QK_PW(11) QK_PW(12) QK_PW(13) QK_PW(14) QK_PW(15)
#undef QK_PW
    }
}

__global__ __launch_bounds__(PTH, 2 * QK_PREP_WG_PER_CU) void qk_prep_operands_kernel(PrepArgs a) {
    __shared__ __attribute__((aligned(16))) PrepLds L;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, l4 = lane >> 4;
    const int K = a.K;
    // Gram blocks of this wave: the 10 upper 16 x 16 blocks (the partials keep no others) dealt so each
    // SIMD (waves s and s + 4) issues at most 3 Gram MFMAs per k-step plus, on the B side, wave s's probe
    // block U(s) — round 4 gave every wave 2 of all 16 blocks: 4-5 MFMAs per SIMD and k-step. Waves 0-3
    // take the diagonal block (s, s), whose row block is also U's operand; waves 4-7 the off-diagonal ones.
    //   SIMD 0: (0,0) | (0,1) (0,2)    SIMD 1: (1,1) | (0,3) (1,2)    SIMD 2: (2,2) | (1,3)    SIMD 3: (3,3) | (2,3)
    int gi0, gj0, gi1 = -1, gj1 = -1;
    switch (wave) {
        case 4: gi0 = 0, gj0 = 1, gi1 = 0, gj1 = 2; break;
        case 5: gi0 = 0, gj0 = 3, gi1 = 1, gj1 = 2; break;
        case 6: gi0 = 1, gj0 = 3; break;
        case 7: gi0 = 2, gj0 = 3; break;
        default: gi0 = gj0 = wave; break;
    }
    gi0 = __builtin_amdgcn_readfirstlane(gi0), gj0 = __builtin_amdgcn_readfirstlane(gj0);
    gi1 = __builtin_amdgcn_readfirstlane(gi1), gj1 = __builtin_amdgcn_readfirstlane(gj1);
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    for (int sd = 0; sd < 2; ++sd) {
        const PrepSide& S = a.s[sd];
        const int R = S.R;
        const int nst = (R + PRS - 1) / PRS;
        const int64_t tiles = S.N / PCT;
        d4_t g0 = {0, 0, 0, 0}, g1 = {0, 0, 0, 0}, u = {0, 0, 0, 0};
        // split grids: a workgroup does one side's tile, so the two sides' serial stage chains (R / PRS
        // dependent stage loads each) run side by side instead of one after the other
        const bool mine = !a.split || (int)(blockIdx.x & 1) == sd;
        const int64_t t_first = a.split ? (int64_t)(blockIdx.x >> 1) : (int64_t)blockIdx.x;
        const int64_t t_step = a.split ? (int64_t)(gridDim.x >> 1) : (int64_t)gridDim.x;
        for (int64_t t = mine ? t_first : tiles; t < tiles; t += t_step) {
            const int64_t c0 = t * PCT;
            // stage loads: this wave moves q rows PRPW w + h (one 1-KiB wave-instruction each) and the
            // same Wt rows (lanes < K/2: 16 B each); rows >= R are not loaded (masked at use)
            int nload[PNS];  // loads this wave issued per ring slot (for the vmcnt accounting)
            auto issue = [&](int st) {
                PrepStage& P = L.st[st % PNS];
                int n = 0;
#pragma unroll
                for (int h = 0; h < PRPW; ++h) {
                    const int rl = PRPW * wave_s + h, r = st * PRS + rl;
                    if (r < R) {
                        prep_glds(S.q + (int64_t)r * S.ldq + c0 + 2 * lane, &P.q[rl][0]);
                        ++n;
                        if (2 * lane < K) prep_glds(S.Wt + (int64_t)r * K + 2 * lane, &P.w[rl][0]);
                        ++n;  // counted for every lane alike (wave-uniform accounting)
                    }
                }
                nload[st % PNS] = n;
            };
            // the previous tile's X readers are done with the LDS (bare barrier: a __syncthreads()
            // would wait for the previous tile's X stores as well)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            for (int st = 0; st < PNS - 1 && st < nst; ++st) issue(st);
            d4_t x[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = (d4_t){0, 0, 0, 0};
            for (int st = 0; st < ((QK_PREP_EXP & 4) ? 0 : nst); ++st) {
                int after = 0;  // loads of this wave issued after stage st's
                for (int d = st + 1; d < st + PNS - 1 && d < nst; ++d) after += nload[d % PNS];
                prep_vmwait(after);
                // stage st landed for every wave; stage st - 1 fully read. A bare s_barrier: the
                // release fence of __syncthreads() makes the compiler wait vmcnt(0) — for the
                // prefetched stages too — which serialised every stage's loads (round 3)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                // this stage's fragments into registers BEFORE the refill is issued: an LDS read
                // after a global_load_lds makes the compiler wait for that load (vmcnt(0)), which
                // serialised every refill with the stage's MFMAs (round 3)
                const PrepStage& P = L.st[st % PNS];
                double qb[PRS / 4], wa[PRS / 4][4];
#pragma unroll
                for (int kk = 0; kk < PRS / 4; ++kk) {
                    const int rl = 4 * kk + l4;
                    const bool rv = st * PRS + rl < R;
                    qb[kk] = rv ? P.q[rl][16 * wave + l16] : 0.0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int k = 16 * i + l16;
                        wa[kk][i] = (rv && k < K) ? P.w[rl][k] : 0.0;
                    }
                }
                if (st + PNS - 1 < nst) issue(st + PNS - 1);
#pragma unroll
                for (int kk = 0; kk < PRS / 4; ++kk)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(wa[kk][i], qb[kk], x[i], 0, 0, 0);
            }
            // probe columns of the tile (B side, waves 0-3): software-pipelined batches of PPB loads,
            // the first batch in flight across the X tile's LDS write (round 2 loaded one per k-step,
            // each waited for at once: 32 dependent global loads per tile)
            const bool probes = S.P != nullptr && wave < 4;
            constexpr int PPB = 8;
            const double* pp = probes ? S.P + (int64_t)l16 * S.N + c0 + l4 : nullptr;
            double pxn[PPB];
#pragma unroll
            for (int j = 0; j < PPB; ++j) pxn[j] = probes ? pp[4 * j] : 0.0;
            // bare barriers (no vmcnt(0): the probe batch stays in flight); every stage's LDS-DMA
            // landed at the last stage's wait
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave is done with the ring: the X tile takes its place
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) L.x[16 * i + l4 + 4 * rr][16 * wave + l16] = x[i][rr];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            // ---- Gram blocks and (B side) probe products over the tile's 128 columns
            for (int s8 = 0; s8 < ((QK_PREP_EXP & 1) ? 0 : PCT / 4); s8 += PPB) {
                double px[PPB];
#pragma unroll
                for (int j = 0; j < PPB; ++j) px[j] = pxn[j];
                if (probes && s8 + PPB < PCT / 4) {
#pragma unroll
                    for (int j = 0; j < PPB; ++j) pxn[j] = pp[4 * (s8 + PPB + j)];
                }
                if (wave < 4) {  // (s, s) and, on the B side, U(s): one operand read serves all three
#pragma unroll
                    for (int j = 0; j < PPB; ++j) {
                        const double av = L.x[16 * gi0 + l16][4 * (s8 + j) + l4];
                        g0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, av, g0, 0, 0, 0);
                        if (probes) u = __builtin_amdgcn_mfma_f64_16x16x4f64(av, px[j], u, 0, 0, 0);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < PPB; ++j) {
                        const int c = 4 * (s8 + j) + l4;
                        const double a0 = L.x[16 * gi0 + l16][c];
                        const double b0 = L.x[16 * gj0 + l16][c];
                        g0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, g0, 0, 0, 0);
                        if (gi1 >= 0) {
                            const double a1 = gi1 == gi0 ? a0 : L.x[16 * gi1 + l16][c];
                            const double b1 = L.x[16 * gj1 + l16][c];
                            g1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, g1, 0, 0, 0);
                        }
                    }
                }
            }
            // ---- X tile to HBM: wave w stores rows 8w .. 8w+7, one contiguous 1-KiB row per
            // wave-instruction (16 B per lane). Round 2 gave each thread 16 consecutive columns of one
            // row — every store instruction scattered 64 x 16 B at a 128-B stride — and then waited
            // for the stores (vmcnt(0)); the two cost 30 of the kernel's 126 us (tools/prep_bench.py)
            if (!(QK_PREP_EXP & 2)) {
                d2_t z[8];  // all eight rows read first: distinct registers, no store-data waits
#pragma unroll
                for (int v = 0; v < 8; ++v) z[v] = *reinterpret_cast<const d2_t*>(&L.x[8 * wave_s + v][2 * lane]);
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    if (8 * wave_s + v < K) *reinterpret_cast<d2_t*>(S.X + (int64_t)(8 * wave_s + v) * S.N + c0 + 2 * lane) = z[v];
            }
            // no vmcnt(0) here: the stores are older than every load of the next tile, and vector
            // memory operations complete in issue order, so the next tile's counted waits cover them
        }
        // ---- this workgroup's partial sums (zero if it took no tile)
        double* p = sd == 0 ? a.part + (int64_t)blockIdx.x * PPA
                            : a.part + (int64_t)gridDim.x * PPA + (int64_t)blockIdx.x * PPB;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int e = (l4 + 4 * rr) * 16 + l16;  // (row, column) inside the 16 x 16 block
            p[prep_tri(gi0, gj0) * 256 + e] = g0[rr];
            if (gi1 >= 0) p[prep_tri(gi1, gj1) * 256 + e] = g1[rr];
            if (sd == 1 && wave < 4) p[PPG + (16 * wave + l4 + 4 * rr) * PNP + l16] = u[rr];
        }
    }
}

// out (sums in a fixed order): GA [K][K], GB [K][K], U [K][16] (from the B side's partials). A
// workgroup takes 64 consecutive partial entries; its PRW waves sum every PRW-th partial (coalesced
// 512-B segments, PRW x more loads in flight than one thread per output), then LDS adds the PRW sums.
// Indexing the outputs by (row, column) instead read the mirrored blocks at a 128-B lane stride: 99 vs
// 43 us beside the 8-rank writes (profiles/r05w_*).
constexpr int PRW = 16;  // waves per reduction workgroup (each sums every 16th partial: 4 in-flight rounds
                         // of 8 loads at 512 partials; 4 waves took 16 rounds, 26 us)
__global__ __launch_bounds__(64 * PRW) void qk_prep_reduce_kernel(const double* __restrict__ part, int nblk,
                                                                  int K, double* __restrict__ GA,
                                                                  double* __restrict__ GB, double* __restrict__ U) {
    __shared__ double acc[PRW][64];
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    // outputs in the partials' own order (coalesced 512-B reads): the A Gram's upper blocks, the B Gram's,
    // then U; an off-diagonal block entry is written to both (r, c) and (c, r)
    const int e = blockIdx.x * 64 + lane;  // [0, 2 PPG + 16 K)
    int sd = -1, off = 0;
    double* dst = nullptr;
    double* mirror = nullptr;
    if (e < 2 * PPG) {
        sd = e < PPG ? 0 : 1;
        off = e - sd * PPG;
        const int blk = off >> 8;
        const int bi = blk < 4 ? 0 : blk < 7 ? 1 : blk < 9 ? 2 : 3;
        const int bj = bi + blk - prep_tri(bi, bi);
        const int r = 16 * bi + ((off >> 4) & 15), c = 16 * bj + (off & 15);
        if (r < K && c < K) {
            double* G = sd == 0 ? GA : GB;
            dst = G + r * K + c;
            if (bi != bj) mirror = G + c * K + r;
        }
    } else if (e < 2 * PPG + PNP * K) {
        const int f = e - 2 * PPG;
        sd = 1, off = PPG + f, dst = U + f;  // U rows k < K: [k][16]
    }
    if (!dst) sd = -1;  // entries past K: nothing to sum (the block stays uniform for the barrier)
    double s = 0.0;
    if (sd >= 0) {
        const int PPART = sd == 0 ? PPA : PPB;  // this side's partial stride
        const double* p = part + (sd == 0 ? 0 : (int64_t)nblk * PPA) + off;
        // 32 loads in flight per thread (one memory round trip for 512 partials; batches of 8 took four),
        // fixed summation order
        double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int b = grp;
        for (; b + 31 * PRW < nblk; b += 32 * PRW) {
            double v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) v[u] = p[(int64_t)(b + PRW * u) * PPART];
#pragma unroll
            for (int u = 0; u < 32; ++u) t[u & 7] += v[u];
        }
        for (; b < nblk; b += PRW) t[0] += p[(int64_t)b * PPART];
        s = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    }
    acc[grp][lane] = s;
    __syncthreads();
    if (grp == 0 && dst) {  // fixed-order pairwise sum over the waves
        double v[PRW];
#pragma unroll
        for (int w = 0; w < PRW; ++w) v[w] = acc[w][lane];
#pragma unroll
        for (int h = PRW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int w = 0; w < h; ++w) v[w] += v[w + h];
        *dst = v[0];
        if (mirror) *mirror = v[0];
    }
}

// out[j][c] = sum_k T[j][k] X[k][c] for j < rmax, both sides (blockIdx.y). A workgroup takes 64 columns
// per iteration; its four waves split K in quarters (16 rows each: every load of a thread in flight at
// once) and sum their partial products through LDS in a fixed order. Round 3: the X loads are issued
// before T is staged, and the grid is one 64-column block per workgroup (4 per CU per side: every
// load of the kernel in flight at once, no second round trip)
__global__ __launch_bounds__(256) void qk_compress_kernel(int K, int rmax, const double* __restrict__ TA,
                                                          const double* __restrict__ XA, int64_t NA, int64_t ldxa,
                                                          double* __restrict__ A2, int64_t lda2,
                                                          const double* __restrict__ TB,
                                                          const double* __restrict__ XB, int64_t NB, int64_t ldxb,
                                                          double* __restrict__ B2, int64_t ldb2) {
    __shared__ double T[8][PK];
    __shared__ double part[4][8][64];
    const bool bs = blockIdx.y == 1;
    const double* Tg = bs ? TB : TA;
    const double* X = bs ? XB : XA;
    double* out = bs ? B2 : A2;
    const int64_t N = bs ? NB : NA, ld = bs ? ldxb : ldxa, ldo = bs ? ldb2 : lda2;
    const int l = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR row bases
    auto load = [&](int64_t c0, double (&xv)[16]) {
        const int64_t c = c0 + l;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int k = 16 * q + u;
            const double* row = X + (int64_t)k * ld;  // uniform
            xv[u] = (k < K && c < N) ? row[c] : 0.0;
        }
    };
    double xv[16];
    int64_t c0 = (int64_t)blockIdx.x * 64;
    if (c0 < N) load(c0, xv);  // in flight while T is staged
    {  // T (at most 8 x 64): both loads of a thread in flight together
        const int n = rmax * K, e0 = threadIdx.x, e1 = threadIdx.x + 256;
        const double t0 = e0 < n ? Tg[e0] : 0.0, t1 = e1 < n ? Tg[e1] : 0.0;
        if (e0 < n) T[e0 / K][e0 % K] = t0;
        if (e1 < n) T[e1 / K][e1 % K] = t1;
    }
    __syncthreads();
    for (; c0 < N; c0 += (int64_t)gridDim.x * 64) {
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < rmax && 16 * q + u < K) acc[j] = fma(T[j][16 * q + u], xv[u], acc[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) part[q][j][l] = acc[j];
        __syncthreads();
        for (int e = threadIdx.x; e < 8 * 64; e += 256) {
            const int j = e >> 6, cc = e & 63;
            if (j < rmax && c0 + cc < N)
                out[(int64_t)j * ldo + c0 + cc] = (part[0][j][cc] + part[1][j][cc]) + (part[2][j][cc] + part[3][j][cc]);
        }
        __syncthreads();
        if (c0 + (int64_t)gridDim.x * 64 < N) load(c0 + (int64_t)gridDim.x * 64, xv);
    }
}

// Column form (round 3, the default when N is even and the rows 16-B aligned): one wave per 128
// columns, a lane takes two adjacent columns (16-B loads: every wave-instruction a contiguous 1-KiB row
// segment) over all K rows, T read as wave-uniform (scalar) operands, no LDS and no cross-wave sum.
// syc 32 5's two 64 x 2^16 operands are 1024 waves — one per SIMD — so each wave keeps its loads
// in flight in 16-row chunks, the next chunk issued before the current one is summed.
constexpr int PCW = 16;  // rows per load chunk
__global__ __launch_bounds__(64) void qk_compress_cols_kernel(int K, int rmax, const double* __restrict__ TA,
                                                              const double* __restrict__ XA, int64_t NA, int64_t ldxa,
                                                              double* __restrict__ A2, int64_t lda2,
                                                              const double* __restrict__ TB,
                                                              const double* __restrict__ XB, int64_t NB, int64_t ldxb,
                                                              double* __restrict__ B2, int64_t ldb2) {
    const bool bs = blockIdx.y == 1;
    const double* Tg = bs ? TB : TA;
    const double* X = bs ? XB : XA;
    double* out = bs ? B2 : A2;
    const int64_t N = bs ? NB : NA, ld = bs ? ldxb : ldxa, ldo = bs ? ldb2 : lda2;
    const int64_t c = ((int64_t)blockIdx.x * 64 + threadIdx.x) * 2;
    if ((int64_t)blockIdx.x * 128 >= N) return;  // the whole wave past this side's columns
    const int64_t cl = c < N ? c : N - 2;          // loads of lanes past the end: the last column pair
    d2_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (d2_t){0.0, 0.0};
    // T^T [PK][8] in LDS, zero beyond (K, rmax): the body is branch-free (rows k >= K re-read row K - 1
    // times a zero coefficient) — uniform-condition scalar T loads became branches, and the compiler
    // then waited vmcnt(0) at each of them
    __shared__ __attribute__((aligned(16))) double Tt[PK][8];
    d2_t buf[2][PCW];
    auto load = [&](int ch, d2_t (&b)[PCW]) {
#pragma unroll
        for (int u = 0; u < PCW; ++u) {
            const int k = min(ch * PCW + u, K - 1);
            b[u] = *reinterpret_cast<const d2_t*>(X + (int64_t)k * ld + cl);
        }
    };
    const int nch = (K + PCW - 1) / PCW;
    {
        // T first: loads complete in issue order, so its wait below does not wait for the X chunk
        double tv[PK * 8 / 64];  // clamped indices: every load unconditional, all in flight together
#pragma unroll
        for (int i = 0; i < PK * 8 / 64; ++i) {
            const int e = threadIdx.x + 64 * i, k = e >> 3, j = e & 7;
            tv[i] = Tg[min(j, rmax - 1) * K + min(k, K - 1)];
        }
        load(0, buf[0]);
#pragma unroll
        for (int i = 0; i < PK * 8 / 64; ++i) {
            const int e = threadIdx.x + 64 * i, k = e >> 3, j = e & 7;
            Tt[k][j] = (k < K && j < rmax) ? tv[i] : 0.0;
        }
    }
    __syncthreads();
    if (c >= N) return;  // after the T staging, which every lane of the wave takes part in
#pragma unroll
    for (int ch = 0; ch < PK / PCW; ++ch) {
        if (ch >= nch) break;
        if (ch + 1 < nch) load(ch + 1, buf[(ch + 1) & 1]);
#pragma unroll
        for (int u = 0; u < PCW; ++u) {
            const int k = ch * PCW + u;
            double t[8];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const d2_t tv = *reinterpret_cast<const d2_t*>(&Tt[k][2 * h]);
                t[2 * h] = tv.x;
                t[2 * h + 1] = tv.y;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc[j].x = fma(t[j], buf[ch & 1][u].x, acc[j].x);
                acc[j].y = fma(t[j], buf[ch & 1][u].y, acc[j].y);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < rmax) *reinterpret_cast<d2_t*>(out + (int64_t)j * ldo + c) = acc[j];
}

constexpr int PV_GRID = 128;  // workgroups of the V = B'' P^T partial sums (probe_d sums their partials)
constexpr int PV_PART = 8 * 16;  // doubles per V partial: rows j < 8 (rmax <= 8), 16 probes

// Compression with the probe check's V pass fused in (round 5): the column kernel's arithmetic (a lane: two
// adjacent columns over all K rows, T from LDS) in 4-wave workgroups of 512 columns; the first nA_wg
// workgroups take A's columns, the rest B's, and a B workgroup also forms its V partial
// vpart[b][j][p] = sum over its columns of B2[j][c] P[p][c] from the B2 values still in registers: each
// wave's 8 x 128 block goes through LDS into 16x16x4 f64 MFMAs against its 128 probe columns, and the
// four waves' sums are added in a fixed order. Replaces qk_probe_v_kernel's second read of B2 and its
// launch.
constexpr int CV_COLS = 512;  // columns per workgroup (4 waves x 128)
__global__ __launch_bounds__(256) void qk_compress_v_kernel(int K, int rmax, const double* __restrict__ TA,
                                                            const double* __restrict__ XA, int64_t NA, int64_t ldxa,
                                                            double* __restrict__ A2, int64_t lda2,
                                                            const double* __restrict__ TB,
                                                            const double* __restrict__ XB, int64_t NB, int64_t ldxb,
                                                            double* __restrict__ B2, int64_t ldb2,
                                                            const double* __restrict__ P, int64_t ldp,
                                                            double* __restrict__ vpart, int nA_wg) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool bs = (int)blockIdx.x >= nA_wg;  // uniform per workgroup
    const int64_t wg = bs ? (int64_t)blockIdx.x - nA_wg : (int64_t)blockIdx.x;
    const double* Tg = bs ? TB : TA;
    const double* X = bs ? XB : XA;
    double* out = bs ? B2 : A2;
    const int64_t N = bs ? NB : NA, ld = bs ? ldxb : ldxa, ldo = bs ? ldb2 : lda2;
    const int64_t base = wg * CV_COLS + wave * 128;
    const int64_t c = base + 2 * lane;
    const bool valid = c < N;
    const int64_t cl = valid ? c : N - 2;  // loads of lanes past the end: the last column pair
    __shared__ __attribute__((aligned(16))) double Tt[PK][8];
    __shared__ __attribute__((aligned(16))) double Bt[4][8][128 + 2];  // each wave's B2 block (B side)
    __shared__ double Vw[4][PV_PART];
    d2_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (d2_t){0.0, 0.0};
    d2_t buf[2][PCW];
    auto load = [&](int ch, d2_t (&b)[PCW]) {
#pragma unroll
        for (int u = 0; u < PCW; ++u) {
            const int k = min(ch * PCW + u, K - 1);
            b[u] = *reinterpret_cast<const d2_t*>(X + (int64_t)k * ld + cl);
        }
    };
    const int nch = (K + PCW - 1) / PCW;
    {
        double tv[2];  // T^T [PK][8]: 512 entries, two per thread
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + 256 * i, k = e >> 3, j = e & 7;
            tv[i] = Tg[min(j, rmax - 1) * K + min(k, K - 1)];
        }
        if (base < N) load(0, buf[0]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = tid + 256 * i, k = e >> 3, j = e & 7;
            Tt[k][j] = (k < K && j < rmax) ? tv[i] : 0.0;
        }
    }
    __syncthreads();
    if (base < N) {  // wave-uniform: the wave has columns
#pragma unroll
        for (int ch = 0; ch < PK / PCW; ++ch) {
            if (ch >= nch) break;
            if (ch + 1 < nch) load(ch + 1, buf[(ch + 1) & 1]);
#pragma unroll
            for (int u = 0; u < PCW; ++u) {
                const int k = ch * PCW + u;
                double t[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const d2_t tv = *reinterpret_cast<const d2_t*>(&Tt[k][2 * h]);
                    t[2 * h] = tv.x;
                    t[2 * h + 1] = tv.y;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    acc[j].x = fma(t[j], buf[ch & 1][u].x, acc[j].x);
                    acc[j].y = fma(t[j], buf[ch & 1][u].y, acc[j].y);
                }
            }
        }
        if (valid) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < rmax) *reinterpret_cast<d2_t*>(out + (int64_t)j * ldo + c) = acc[j];
        }
    }
    if (!bs) return;  // uniform per workgroup: no barrier below is split
    // ---- V partial of this workgroup's columns
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const d2_t v = (valid && j < rmax) ? acc[j] : (d2_t){0.0, 0.0};
        *reinterpret_cast<d2_t*>(&Bt[wave][j][2 * lane]) = v;
    }
    __syncthreads();
    const int i16 = lane & 15, k4 = lane >> 4;
    d4_t va = {0.0, 0.0, 0.0, 0.0};
    if (base < N) {
        // B operand: P[p = i16][base + 4 s + k4]; 8 steps of loads in flight per batch
        constexpr int VB = 8;
        const double* pr = P + (int64_t)i16 * ldp;
#pragma unroll
        for (int s0 = 0; s0 < 32; s0 += VB) {
            double pb[VB];
#pragma unroll
            for (int s = 0; s < VB; ++s) {
                const int64_t col = base + 4 * (s0 + s) + k4;
                pb[s] = col < N ? pr[col] : 0.0;
            }
#pragma unroll
            for (int s = 0; s < VB; ++s) {
                const double a = i16 < 8 ? Bt[wave][i16][4 * (s0 + s) + k4] : 0.0;
                va = __builtin_amdgcn_mfma_f64_16x16x4f64(a, pb[s], va, 0, 0, 0);
            }
        }
    }
    // C layout: row j = k4 + 4 r, column p = i16; rows j < 8 are r = 0, 1
#pragma unroll
    for (int r = 0; r < 2; ++r) Vw[wave][(k4 + 4 * r) * 16 + i16] = va[r];
    __syncthreads();
    if (tid < PV_PART)
        vpart[wg * PV_PART + tid] = (Vw[0][tid] + Vw[1][tid]) + (Vw[2][tid] + Vw[3][tid]);
}

// V partials: vpart[b][j][p] = sum over this workgroup's columns c of B2[j][c] P[p][c] (j < rmax), on the
// VALU: a lane takes one column per iteration (every load a coalesced 512-B row segment), wave w the
// probes 4w..4w+3, acc[j][q] in registers; then a wave reduction and one store per (j, p). The MFMA form
// before it fed a 16 x 4 operand block per instruction — 16 rows x 32 B per load, 4x the cache lines
// — and took 25 us for syc 32 5's 8 x 2^16 B'' against 16 probes.
__global__ __launch_bounds__(256) void qk_probe_v_kernel(int rmax, const double* __restrict__ B2, int64_t ldb2,
                                                         int64_t NB, const double* __restrict__ P, int64_t ldp,
                                                         double* __restrict__ vpart) {
    // loads are unconditional (rows >= rmax re-read row rmax - 1, zeroed at the end): conditional loads
    // became branches with a vmcnt(0) wait each (round 3)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double acc[8][4];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[jj][q] = 0.0;
    // the next column's 12 loads in flight while the current one is multiplied (two named buffers,
    // unconditional clamped prefetch: the round-2 loop waited for each iteration's loads in turn)
    struct Col {
        double b[8], pv[4];
    };
    const int64_t step = (int64_t)gridDim.x * 64;
    auto fetch = [&](int64_t c, Col& x) {
        const int64_t cc = c < NB ? c : NB - 1;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) x.b[jj] = B2[(int64_t)min(jj, rmax - 1) * ldb2 + cc];
#pragma unroll
        for (int q = 0; q < 4; ++q) x.pv[q] = P[(int64_t)(4 * wave + q) * ldp + cc];
    };
    auto mac = [&](const Col& x) {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[jj][q] = fma(x.b[jj], x.pv[q], acc[jj][q]);
    };
    int64_t c = (int64_t)blockIdx.x * 64 + lane;
    if (c < NB) {
        Col x0, x1;
        fetch(c, x0);
        for (;; c += 2 * step) {
            fetch(c + step, x1);
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issued ahead of the multiplies
            mac(x0);
            if (c + step >= NB) break;
            fetch(c + 2 * step, x0);
            __builtin_amdgcn_sched_barrier(0);
            mac(x1);
            if (c + 2 * step >= NB) break;
        }
    }
    // wave sums in a fixed order (xor butterfly: every lane ends with the total)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double v = acc[jj][q];
#pragma unroll
            for (int s = 1; s < 64; s <<= 1) v += __shfl_xor(v, s, 64);
            acc[jj][q] = jj < rmax ? v : 0.0;
        }
    // vpart layout [b][j][p], j < 8 (rows >= rmax zero): lane j * 4 + q (< 32) of wave w writes (j, 4w + q)
    double* out = vpart + (int64_t)blockIdx.x * PV_PART;
    if (lane < 32) {
        const int j8 = lane >> 2, q = lane & 3;
        double v = 0.0;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
                if (jj == j8 && qq == q) v = acc[jj][qq];
        out[j8 * 16 + 4 * wave + q] = v;
    }
}

// e2 partials over 16-column blocks of A: d = X_A^T U - A2^T V, epart[b][p] = sum of d[c][p]^2
__global__ __launch_bounds__(256) void qk_probe_d_kernel(int K, int rmax, const double* __restrict__ XA, int64_t ldx,
                                                         int64_t NA, const double* __restrict__ A2, int64_t lda2,
                                                         const double* __restrict__ U,
                                                         const double* __restrict__ vpart, int gv,
                                                         double* __restrict__ epart) {
    __shared__ double Us[PK][PNP];
    __shared__ double Vs[16][PNP];
    __shared__ double ep[4][2 * PNP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, l4 = lane >> 4;
    {  // V rows 0..7, a fixed-order fold of the partials: thread t takes entry t % 128 over the partials
       // b = t / 128 (mod 2), 16 loads in flight per batch (batches of 8 on half the threads took one
       // memory latency each); rows 8..15 stay zero
        __shared__ double vh[PV_PART];
        const int e = tid & (PV_PART - 1), h = tid >> 7;
        double t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) t[u] = 0.0;
        int b = h;
        for (; b + 30 < gv; b += 32) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = vpart[(int64_t)(b + 2 * u) * PV_PART + e];
#pragma unroll
            for (int u = 0; u < 16; ++u) t[u] += v[u];
        }
        for (; b < gv; b += 2) t[0] += vpart[(int64_t)b * PV_PART + e];
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int u = 0; u < w; ++u) t[u] += t[u + w];
        if (h == 1) vh[e] = t[0];
        __syncthreads();
        if (h == 0) Vs[e / 16][e % 16] = -(t[0] + vh[e]);
        else Vs[8 + e / 16][e % 16] = 0.0;
    }
    for (int e = tid; e < PK * PNP; e += 256) Us[e / PNP][e % PNP] = (e / PNP) < K ? U[e] : 0.0;
    __syncthreads();
    double e2 = 0.0, f2 = 0.0;  // squared errors and squared reference products (R p)
    // every operand load of a 16-column block in flight before its MFMAs (round 3: the k-loop waited
    // for each load in turn, 18 memory round trips per block); rows k >= K re-read row K - 1 against
    // the zero rows of Us, rows j >= rmax row rmax - 1 against the zero rows of Vs
    for (int64_t cb = (int64_t)blockIdx.x * 4 + wave; cb * 16 < NA; cb += (int64_t)gridDim.x * 4) {
        const int64_t c = cb * 16 + l16;
        double av[PK / 4], a2[2];
#pragma unroll
        for (int kk = 0; kk < PK / 4; ++kk) av[kk] = XA[(int64_t)min(4 * kk + l4, K - 1) * ldx + c];  // A[c][k]
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) a2[jj] = A2[(int64_t)min(4 * jj + l4, rmax - 1) * lda2 + c];
        d4_t acc = {0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < PK / 4; ++kk)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], Us[4 * kk + l4][l16], acc, 0, 0, 0);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) f2 = fma(acc[rr], acc[rr], f2);  // (X_A^T U)[c][p] = (R p)_c
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[jj], Vs[4 * jj + l4][l16], acc, 0, 0, 0);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) e2 = fma(acc[rr], acc[rr], e2);  // d[cb*16 + l4 + 4rr][l16]
    }
    e2 += __shfl_xor(e2, 16, 64);
    e2 += __shfl_xor(e2, 32, 64);
    f2 += __shfl_xor(f2, 16, 64);
    f2 += __shfl_xor(f2, 32, 64);
    if (l4 == 0) {
        ep[wave][l16] = e2;
        ep[wave][PNP + l16] = f2;
    }
    __syncthreads();
    if (tid < 2 * PNP)
        epart[(int64_t)blockIdx.x * 2 * PNP + tid] = ep[0][tid] + ep[1][tid] + ep[2][tid] + ep[3][tid];
}

// rows of 32: e2[p] (squared errors) then f2[p] (squared reference products ||R p||^2).
// e2_out[0..32) = sum_b epart[b][.]; with k_out: *err_out = sqrt(max_p e2), and the accepted rank
// *k_out = (r > 0 && err <= max(tol, rel_tol sqrt(max_p f2))) ? r : 0 — the bound scales with the knit
// itself (||R p|| ~ ||R||_F) above the absolute floor tol.
// 256 threads: thread t sums rows b = t / 32, + 8, ... of entry t % 32, then a fixed-order LDS tree.
constexpr int PE = 2 * PNP;

__global__ __launch_bounds__(256) void qk_probe_accept_kernel(const double* __restrict__ epart, int n,
                                                              const int32_t* __restrict__ r_dev, double tol,
                                                              double rel_tol, double* __restrict__ e2_out,
                                                              int32_t* __restrict__ k_out, double* __restrict__ err_out,
                                                              int64_t* __restrict__ tally = nullptr) {
    __shared__ double acc[256];
    const int tid = threadIdx.x, p = tid % PE;
    // eight independent partial sums (loads in flight together), combined in a fixed order
    constexpr int STEP = 256 / PE;
    double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int b = tid / PE;
    for (; b + 31 * STEP < n; b += 32 * STEP) {  // 32 loads in flight per batch (batches of 8: a round trip each)
        double v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = epart[(int64_t)(b + u * STEP) * PE + p];
#pragma unroll
        for (int u = 0; u < 32; ++u) s8[u & 7] += v[u];
    }
    for (; b < n; b += STEP) s8[0] += epart[(int64_t)b * PE + p];
    const double s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    acc[tid] = s;
    __syncthreads();
    for (int w = 128; w >= PE; w >>= 1) {
        if (tid < w) acc[tid] += acc[tid + w];
        __syncthreads();
    }
    if (tid < PE && e2_out) e2_out[tid] = acc[tid];
    if (tid == 0 && k_out) {
        double m = 0.0, f = 0.0;
        for (int q = 0; q < PNP; ++q) {
            m = fmax(m, acc[q]);
            f = fmax(f, acc[PNP + q]);
        }
        const double err = sqrt(m);
        const double bound = fmax(tol, rel_tol * sqrt(f));
        const int r = *r_dev;
        if (err_out) *err_out = err;
        const int k = (r > 0 && err <= bound) ? r : 0;
        *k_out = k;
        if (tally) {  // qk_rank_tally's update, fused (one dependent launch fewer per step)
            tally[0] += r == 0 ? 1 : 0;
            tally[1] += (r > 0 && k == 0) ? 1 : 0;
            tally[2] = k;
            tally[3] += 1;
        }
    }
}

// ================================================================================================
// q-space preparation (round 5): the same step without materialising X_s = W_s q_s (W_s = Wt_s^T).
// Every quantity the chain needs is a product of the swept rows q_s with small matrices:
//   G_s = X_s X_s^T = W_s (q_s q_s^T) W_s^T       Gq_s = q_s q_s^T  [R_s][R_s]   (qk_qgram_kernel)
//   U   = X_B P^T   = W_B (q_B P^T)               Pq   = q_B P^T    [R_B][16]
//   A'' = T_A X_A   = (T_A W_A) q_A = M_A q_A     M_s  = T_s W_s    [rmax][R_s]   (per workgroup, LDS)
//   R p = X_A^T U   = q_A^T (W_A^T U) = q_A^T Z_A Z_A  = W_A^T U    [R_A][16]
// so one pass over q gives the Grams (an MFMA SYRK over 128-column tiles, R <= 80 rows), and the
// compression and the probe check read q once more each: ~0.2 GB of HBM per syc 32 5 step instead of
// ~0.45 GB, and no 1.1-GFLOP transform. The check still runs on the MATERIALISED compressed operands
// (V = B'' P^T from the B'' the write reads; d = R p - A''^T V from the A'' it reads), as before.
constexpr int QG_T = 512;       // threads per qk_qgram workgroup (8 waves)
// LDS row stride (doubles) of a staged q tile: 146 = 292 dwords = 4 banks past a multiple of 32, so the
// MFMA operand reads (16 rows x 2 adjacent columns per 16-lane group, ds_read_b128) spread over the banks
// (2-way at most); a stride that is a multiple of 32 banks put all 16 rows on one bank group (16-way)
constexpr int QG_LD = PCT + 18;
constexpr int QG_NB = 5;        // 16-row blocks: R <= 80
constexpr int QG_RMAX = 16 * QG_NB;
constexpr int QG_UP = QG_NB * (QG_NB + 1) / 2;       // upper-triangle Gram blocks
constexpr int QG_PART = (QG_UP + QG_NB) * 256;        // one workgroup's partial sums per side (+ probe blocks)

// Global -> LDS staging of n doubles by nthreads threads, 16 loads of a thread in flight per round (a
// plain loop waits for each load in turn: ~40 dependent L2 round trips per thread, tens of us)
template <typename F>
__device__ __forceinline__ void stage16(const double* __restrict__ src, int n, int nthreads, F store) {
    for (int e0 = threadIdx.x; e0 < n; e0 += 16 * nthreads) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = e0 + u * nthreads;
            v[u] = e < n ? src[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = e0 + u * nthreads;
            if (e < n) store(e, v[u]);
        }
    }
}

struct QGramSide {
    const double* q;  // [R][ldq], columns [0, N)
    int64_t ldq, N;
    int R;
    const double* P;  // probes [16][N] (B side) or nullptr
};

struct QGramArgs {
    QGramSide s[2];
    int split;      // 1: even workgroups take side 0's tiles, odd ones side 1's
    int slots;      // partial slots per side
    double* part;   // [2][slots][QG_PART]
};

__device__ __forceinline__ void qg_block(int b, int& bi, int& bj) {  // upper block b -> (bi <= bj)
    bi = 0;
    int n = QG_NB;
    while (b >= n) {
        b -= n;
        ++bi;
        --n;
    }
    bj = bi + b;
}

__global__ __launch_bounds__(QG_T, 2) void qk_qgram_kernel(QGramArgs a) {
    extern __shared__ __attribute__((aligned(16))) double qs[];  // [R][QG_LD]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, l4 = lane >> 4;
    const int wave_s = __builtin_amdgcn_readfirstlane(wave);
    for (int sd = 0; sd < 2; ++sd) {
        const QGramSide& S = a.s[sd];
        const int R = S.R, nb = (R + 15) / 16;
        // this wave's blocks: slots wave, wave + 8, wave + 16 of [upper blocks | probe blocks]
        int bi[3], bj[3];
        bool live[3], probe[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int b = wave + 8 * t;
            probe[t] = b >= QG_UP;
            if (!probe[t]) qg_block(b, bi[t], bj[t]);
            else bi[t] = b - QG_UP, bj[t] = 0;
            live[t] = b < QG_UP + QG_NB && bi[t] < nb && (probe[t] ? S.P != nullptr : bj[t] < nb);
        }
        d4_t acc[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = (d4_t){0, 0, 0, 0};
        const bool mine = !a.split || (int)(blockIdx.x & 1) == sd;
        const int64_t t_first = a.split ? (int64_t)(blockIdx.x >> 1) : (int64_t)blockIdx.x;
        const int64_t t_step = a.split ? (int64_t)(gridDim.x >> 1) : (int64_t)gridDim.x;
        const int64_t tiles = S.N / PCT;
        const bool want_p = (live[0] && probe[0]) || (live[1] && probe[1]) || (live[2] && probe[2]);
        for (int64_t t = mine ? t_first : tiles; t < tiles; t += t_step) {
            const int64_t c0 = t * PCT;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // the previous tile's readers are done with the LDS
            for (int r = wave_s; r < R; r += QG_T / 64) prep_glds(S.q + (int64_t)r * S.ldq + c0 + 2 * lane, &qs[r * QG_LD]);
            // this lane's probe operands (the B operand of a probe block: columns 8 s + 2 l4 and + 1 of P row l16)
            d2_t pv[PCT / 8];
            if (want_p) {
                const double* pp = S.P + (int64_t)l16 * S.N + c0 + 2 * l4;
#pragma unroll
                for (int s8 = 0; s8 < PCT / 8; ++s8) pv[s8] = *reinterpret_cast<const d2_t*>(pp + 8 * s8);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave's rows landed
            // a k-step pair per 16-B read: lane (l16, l4) takes columns 8 s + 2 l4, + 1 (the Gram sums over
            // columns in any order; A and B operands take the same columns)
#pragma unroll
            for (int t3 = 0; t3 < 3; ++t3) {
                if (!live[t3]) continue;  // wave-uniform
                const int ra = 16 * bi[t3] + l16, rb = 16 * bj[t3] + l16;
                const d2_t* xa = reinterpret_cast<const d2_t*>(&qs[(ra < R ? ra : R - 1) * QG_LD + 2 * l4]);
                const d2_t* xb = reinterpret_cast<const d2_t*>(&qs[(rb < R ? rb : R - 1) * QG_LD + 2 * l4]);
                const double ma = ra < R ? 1.0 : 0.0, mb = rb < R ? 1.0 : 0.0;
                d4_t g = acc[t3];
                if (probe[t3]) {
#pragma unroll
                    for (int s8 = 0; s8 < PCT / 8; ++s8) {
                        const d2_t x = xa[4 * s8];
                        g = __builtin_amdgcn_mfma_f64_16x16x4f64(ma * x.x, pv[s8].x, g, 0, 0, 0);
                        g = __builtin_amdgcn_mfma_f64_16x16x4f64(ma * x.y, pv[s8].y, g, 0, 0, 0);
                    }
                } else {
#pragma unroll 4
                    for (int s8 = 0; s8 < PCT / 8; ++s8) {
                        const d2_t x = xa[4 * s8], y = xb[4 * s8];
                        g = __builtin_amdgcn_mfma_f64_16x16x4f64(ma * x.x, mb * y.x, g, 0, 0, 0);
                        g = __builtin_amdgcn_mfma_f64_16x16x4f64(ma * x.y, mb * y.y, g, 0, 0, 0);
                    }
                }
                acc[t3] = g;
            }
        }
        const int slot = a.split ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
        if (a.split && !mine) continue;  // a split workgroup owns one side's slot only
        double* p = a.part + ((int64_t)sd * a.slots + slot) * QG_PART;
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3) {
            const int b = wave + 8 * t3;
            if (b >= QG_UP + QG_NB) continue;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) p[b * 256 + (l4 + 4 * rr) * 16 + l16] = live[t3] ? acc[t3][rr] : 0.0;
        }
    }
}

// gq (zero-padded): Gq_A [QG_RMAX][QG_RMAX], Gq_B [QG_RMAX][QG_RMAX], Pq [QG_RMAX][16]; sums over the
// partial slots in a fixed order (as qk_prep_reduce_kernel), mirrored from the upper blocks
__global__ __launch_bounds__(64 * PRW) void qk_qgram_reduce_kernel(const double* __restrict__ part, int slots,
                                                                   double* __restrict__ gq) {
    __shared__ double acc[PRW][64];
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;  // [0, 2 * QG_PART): side e / QG_PART, entry e % QG_PART
    const int sd = e / QG_PART, f = e % QG_PART;
    double s = 0.0;
    if (sd < 2) {
        const double* p = part + (int64_t)sd * slots * QG_PART + f;
        double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int b = grp;
        for (; b + 31 * PRW < slots; b += 32 * PRW) {
            double v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) v[u] = p[(int64_t)(b + PRW * u) * QG_PART];
#pragma unroll
            for (int u = 0; u < 32; ++u) t[u & 7] += v[u];
        }
        for (; b < slots; b += PRW) t[0] += p[(int64_t)b * QG_PART];
        s = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
    }
    acc[grp][lane] = s;
    __syncthreads();
    if (grp == 0 && sd < 2) {
        double v[PRW];
#pragma unroll
        for (int w = 0; w < PRW; ++w) v[w] = acc[w][lane];
#pragma unroll
        for (int h = PRW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int w = 0; w < h; ++w) v[w] += v[w + h];
        const int blk = f / 256, in = f % 256, r = in / 16, c = in % 16;
        if (blk < QG_UP) {
            int bi, bj;
            qg_block(blk, bi, bj);
            double* G = gq + (int64_t)sd * QG_RMAX * QG_RMAX;
            G[(16 * bi + r) * QG_RMAX + 16 * bj + c] = v[0];
            if (bi != bj) G[(16 * bj + c) * QG_RMAX + 16 * bi + r] = v[0];
        } else if (sd == 1) {
            gq[2 * QG_RMAX * QG_RMAX + (16 * (blk - QG_UP) + r) * 16 + c] = v[0];
        }
    }
}

// The projections, 2 x (K / 16) + 1 workgroups: workgroup (s, cb) forms columns 16 cb .. 16 cb + 15 of
// H_s = Gq_s Wt_s [R][K] and of G_s = Wt_s^T H_s [K][K]; the last one U = Wt_B^T Pq [K][16]. Operands
// staged in LDS (16 loads in flight per thread), every sum in a fixed order.
constexpr int QP_CB = PK / 16;  // column blocks per side
__global__ __launch_bounds__(256) void qk_qproject_kernel(int K, int RA, const double* __restrict__ WtA, int RB,
                                                          const double* __restrict__ WtB, const double* __restrict__ gq,
                                                          double* __restrict__ GA, double* __restrict__ GB,
                                                          double* __restrict__ U) {
    __shared__ double Wt[QG_RMAX][PK + 1];
    __shared__ double Gs[QG_RMAX][QG_RMAX + 1];
    __shared__ double H[QG_RMAX][17];
    const int tid = threadIdx.x;
    const int bx = blockIdx.x;
    const bool proj_u = bx == 2 * QP_CB;
    const int sd = proj_u ? 1 : bx / QP_CB, cb = bx % QP_CB;
    if (!proj_u && 16 * cb >= K) return;
    const int R = sd ? RB : RA;
    const double* W = sd ? WtB : WtA;
    stage16(W, R * K, 256, [&](int e, double v) { Wt[e / K][e % K] = v; });
    if (!proj_u) {
        const double* Gq = gq + (int64_t)sd * QG_RMAX * QG_RMAX;
        stage16(Gq, R * QG_RMAX, 256, [&](int e, double v) { Gs[e / QG_RMAX][e % QG_RMAX] = v; });
    } else {
        const double* Pq = gq + 2 * QG_RMAX * QG_RMAX;
        stage16(Pq, R * PNP, 256, [&](int e, double v) { Gs[e / PNP][e % PNP] = v; });
    }
    __syncthreads();
    if (!proj_u) {
        const int nc = K - 16 * cb < 16 ? K - 16 * cb : 16;
        for (int e = tid; e < R * 16; e += 256) {  // H[:, 16 cb + y] = Gq Wt[:, 16 cb + y]
            const int i = e >> 4, y = e & 15;
            double h = 0.0;
            if (y < nc)
                for (int j = 0; j < R; ++j) h = fma(Gs[i][j], Wt[j][16 * cb + y], h);
            H[i][y] = h;
        }
        __syncthreads();
        double* G = sd ? GB : GA;
        for (int e = tid; e < K * 16; e += 256) {  // G[x][16 cb + y] = Wt[:, x]^T H[:, y]
            const int x = e >> 4, y = e & 15;
            if (y >= nc) continue;
            double g = 0.0;
            for (int i = 0; i < R; ++i) g = fma(Wt[i][x], H[i][y], g);
            G[x * K + 16 * cb + y] = g;
        }
    } else {
        for (int e = tid; e < K * PNP; e += 256) {  // U = Wt_B^T Pq  [K][16]
            const int x = e / PNP, p = e % PNP;
            double u = 0.0;
            for (int i = 0; i < R; ++i) u = fma(Wt[i][x], Gs[i][p], u);
            U[e] = u;
        }
    }
}

// The staged operands of a compress workgroup: T [8][K] and Wt [R][K] (then M^T [R][8] = (T Wt^T)^T), and
// on the A side U [K][16] (then Z = Wt U [R][16]); loaded with 16 loads in flight per thread, then formed
// from LDS. Rows j >= rmax of M are zero.
struct QcStage {
    double T[8][PK + 1];
    double W[QG_RMAX][PK + 1];
    double U[PK][PNP + 1];
};

__device__ __forceinline__ void qc_stage(int K, int rmax, int R, const double* __restrict__ T,
                                         const double* __restrict__ Wt, const double* __restrict__ U, QcStage& st,
                                         double (*Mt)[8], double (*Zt)[PNP], int nthreads) {
    stage16(T, rmax * K, nthreads, [&](int e, double v) { st.T[e / K][e % K] = v; });
    stage16(Wt, R * K, nthreads, [&](int e, double v) { st.W[e / K][e % K] = v; });
    if (U) stage16(U, K * PNP, nthreads, [&](int e, double v) { st.U[e / PNP][e % PNP] = v; });
    __syncthreads();
    for (int e = threadIdx.x; e < R * 8; e += nthreads) {
        const int i = e >> 3, j = e & 7;
        double m = 0.0;
        if (j < rmax)
            for (int x = 0; x < K; ++x) m = fma(st.T[j][x], st.W[i][x], m);
        Mt[i][j] = m;
    }
    if (U)
        for (int e = threadIdx.x; e < R * PNP; e += nthreads) {
            const int i = e / PNP, p = e % PNP;
            double z = 0.0;
            for (int x = 0; x < K; ++x) z = fma(st.W[i][x], st.U[x][p], z);
            Zt[i][p] = z;
        }
}

constexpr int QC_CH = 16;            // q rows per load chunk
constexpr int QV_PART = 8 * PNP;     // one workgroup's V partial [8][16]
constexpr int QB_T = 256;            // compress_b: threads (4 waves), 2 columns per lane per iteration
constexpr int QB_COLS = 2 * QB_T;    // columns per iteration
constexpr int QB_SPAN = 2 * QB_COLS; // columns per workgroup (2 iterations): few V partials to fold
constexpr int QA_T = 128;            // compress_a: threads (2 waves), 2 columns per lane
constexpr int QA_COLS = 2 * QA_T;

// B'' = M_B q_B (written) and this workgroup's V partial = B'' P^T over its columns, from the B'' just
// formed (staged in LDS per iteration; thread t sums (j, p) = (t / 16 % 8, t % 16) over half h = t / 128 of
// each iteration's columns, the halves added at the end: a fixed order)
__global__ __launch_bounds__(QB_T) void qk_qcompress_b_kernel(int K, int rmax, int R, const double* __restrict__ T,
                                                              const double* __restrict__ Wt, const double* __restrict__ q,
                                                              int64_t ldq, int64_t N, const double* __restrict__ P,
                                                              double* __restrict__ B2, double* __restrict__ vpart) {
    __shared__ double Mt[QG_RMAX][8];
    __shared__ __attribute__((aligned(16))) double b2s[8][QB_COLS];
    __shared__ __attribute__((aligned(16))) double ps[PNP][QB_COLS];
    __shared__ QcStage st;
    __shared__ double vh[QV_PART];
    const int tid = threadIdx.x;
    qc_stage(K, rmax, R, T, Wt, nullptr, st, Mt, nullptr, QB_T);
    __syncthreads();
    const int vj = (tid >> 4) & 7, vp = tid & 15, vhalf = tid >> 7;
    double vacc = 0.0;
    const int nch = (R + QC_CH - 1) / QC_CH;
    const int64_t s0 = (int64_t)blockIdx.x * QB_SPAN, s1 = s0 + QB_SPAN < N ? s0 + QB_SPAN : N;
    for (int64_t c0 = s0; c0 < s1; c0 += QB_COLS) {
        const int64_t c = c0 + 2 * tid;
        // the iteration's probes (coalesced 16-B rows) in flight with the q loads
        d2_t pvv[PNP * QB_COLS / 2 / QB_T];
#pragma unroll
        for (int u = 0; u < PNP * QB_COLS / 2 / QB_T; ++u) {
            const int e = tid + u * QB_T, p = e / (QB_COLS / 2), cc = 2 * (e % (QB_COLS / 2));
            pvv[u] = *reinterpret_cast<const d2_t*>(P + (int64_t)p * N + c0 + cc);
        }
        d2_t acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = (d2_t){0.0, 0.0};
        d2_t buf[2][QC_CH];
        auto load = [&](int ch, d2_t (&bb)[QC_CH]) {
#pragma unroll
            for (int u = 0; u < QC_CH; ++u) {
                const int i = min(ch * QC_CH + u, R - 1);
                bb[u] = *reinterpret_cast<const d2_t*>(q + (int64_t)i * ldq + c);
            }
        };
        load(0, buf[0]);
#pragma unroll
        for (int ch = 0; ch < QG_RMAX / QC_CH; ++ch) {  // compile-time buffer indices (no scratch)
            if (ch >= nch) break;
            if (ch + 1 < nch) load(ch + 1, buf[(ch + 1) & 1]);
#pragma unroll
            for (int u = 0; u < QC_CH; ++u) {
                const int i = ch * QC_CH + u;
                const double w = i < R ? 1.0 : 0.0;  // rows past R re-read row R - 1: zero weight
                const d2_t x = buf[ch & 1][u];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double m = w * Mt[i < R ? i : R - 1][j];
                    acc[j].x = fma(m, x.x, acc[j].x);
                    acc[j].y = fma(m, x.y, acc[j].y);
                }
            }
        }
        __syncthreads();  // the previous iteration's V readers are done with b2s / ps
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < rmax) *reinterpret_cast<d2_t*>(B2 + (int64_t)j * N + c) = acc[j];
            *reinterpret_cast<d2_t*>(&b2s[j][2 * tid]) = acc[j];
        }
#pragma unroll
        for (int u = 0; u < PNP * QB_COLS / 2 / QB_T; ++u) {
            const int e = tid + u * QB_T, p = e / (QB_COLS / 2), cc = 2 * (e % (QB_COLS / 2));
            *reinterpret_cast<d2_t*>(&ps[p][cc]) = pvv[u];
        }
        __syncthreads();
        const int h0 = vhalf * (QB_COLS / 2);
        double v0 = 0.0, v1 = 0.0;
        for (int cc = h0; cc < h0 + QB_COLS / 2; cc += 2) {
            v0 = fma(b2s[vj][cc], ps[vp][cc], v0);
            v1 = fma(b2s[vj][cc + 1], ps[vp][cc + 1], v1);
        }
        vacc += v0 + v1;
    }
    if (vhalf) vh[vj * PNP + vp] = vacc;
    __syncthreads();
    if (!vhalf) vpart[(int64_t)blockIdx.x * QV_PART + vj * PNP + vp] = vj < rmax ? vacc + vh[vj * PNP + vp] : 0.0;
}

// A'' = M_A q_A (written) and the probe check over these columns: ref = q_A^T Z_A (= (R p)_c, Z_A = W_A^T U)
// and d = ref - A''^T V (V: the fixed-order fold of the B-side partials); epart[wg] = (sum d^2, sum ref^2)
__global__ __launch_bounds__(QA_T) void qk_qcompress_a_kernel(int K, int rmax, int R, const double* __restrict__ T,
                                                              const double* __restrict__ Wt, const double* __restrict__ q,
                                                              int64_t ldq, int64_t N, const double* __restrict__ U,
                                                              const double* __restrict__ vpart, int gv,
                                                              double* __restrict__ A2, double* __restrict__ epart) {
    __shared__ double Mt[QG_RMAX][8];
    __shared__ double Zt[QG_RMAX][PNP];
    __shared__ double Vs[8][PNP];
    __shared__ double red[QA_T / 64][2 * PNP];
    __shared__ QcStage st;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t c = (int64_t)blockIdx.x * QA_COLS + 2 * tid;
    {  // V = sum of the gv partials, fixed order: thread t < 128 takes entry t over every partial
        const int e = tid;
        double t8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int b = 0;
        for (; b + 31 < gv; b += 32) {
            double v[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) v[u] = vpart[(int64_t)(b + u) * QV_PART + e];
#pragma unroll
            for (int u = 0; u < 32; ++u) t8[u & 7] += v[u];
        }
        for (; b < gv; ++b) t8[0] += vpart[(int64_t)b * QV_PART + e];
        Vs[e / PNP][e % PNP] = ((t8[0] + t8[1]) + (t8[2] + t8[3])) + ((t8[4] + t8[5]) + (t8[6] + t8[7]));
    }
    qc_stage(K, rmax, R, T, Wt, U, st, Mt, Zt, QA_T);  // Z = Wt_A U  [R][16]
    __syncthreads();
    d2_t a2[8], ref[PNP];
#pragma unroll
    for (int j = 0; j < 8; ++j) a2[j] = (d2_t){0.0, 0.0};
#pragma unroll
    for (int p = 0; p < PNP; ++p) ref[p] = (d2_t){0.0, 0.0};
    d2_t buf[2][QC_CH];
    auto load = [&](int ch, d2_t (&bb)[QC_CH]) {
#pragma unroll
        for (int u = 0; u < QC_CH; ++u) {
            const int i = min(ch * QC_CH + u, R - 1);
            bb[u] = *reinterpret_cast<const d2_t*>(q + (int64_t)i * ldq + c);
        }
    };
    const int nch = (R + QC_CH - 1) / QC_CH;
    load(0, buf[0]);
#pragma unroll
    for (int ch = 0; ch < QG_RMAX / QC_CH; ++ch) {  // compile-time buffer indices (no scratch)
        if (ch >= nch) break;
        if (ch + 1 < nch) load(ch + 1, buf[(ch + 1) & 1]);
#pragma unroll
        for (int u = 0; u < QC_CH; ++u) {
            const int i = ch * QC_CH + u;
            const double w = i < R ? 1.0 : 0.0;
            const int ii = i < R ? i : R - 1;
            const d2_t x = buf[ch & 1][u];
            const d2_t xw = (d2_t){w * x.x, w * x.y};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double m = Mt[ii][j];
                a2[j].x = fma(m, xw.x, a2[j].x);
                a2[j].y = fma(m, xw.y, a2[j].y);
            }
#pragma unroll
            for (int p = 0; p < PNP; ++p) {
                const double z = Zt[ii][p];
                ref[p].x = fma(z, xw.x, ref[p].x);
                ref[p].y = fma(z, xw.y, ref[p].y);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < rmax) *reinterpret_cast<d2_t*>(A2 + (int64_t)j * N + c) = a2[j];
    // d = ref - A''^T V per probe, squared; the reference products squared
    double e2[PNP], f2[PNP];
#pragma unroll
    for (int p = 0; p < PNP; ++p) {
        d2_t d = ref[p];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            d.x = fma(-a2[j].x, Vs[j][p], d.x);
            d.y = fma(-a2[j].y, Vs[j][p], d.y);
        }
        e2[p] = fma(d.x, d.x, d.y * d.y);
        f2[p] = fma(ref[p].x, ref[p].x, ref[p].y * ref[p].y);
    }
#pragma unroll
    for (int p = 0; p < PNP; ++p) {
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            e2[p] += __shfl_xor(e2[p], s, 64);
            f2[p] += __shfl_xor(f2[p], s, 64);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int p = 0; p < PNP; ++p) {
            red[wave][p] = e2[p];
            red[wave][PNP + p] = f2[p];
        }
    }
    __syncthreads();
    if (tid < 2 * PNP) epart[(int64_t)blockIdx.x * PE + tid] = red[0][tid] + red[1][tid];
}

int probe_grid_d(qk_ctx* ctx, int64_t NA) {
    const int64_t blocks = (NA + 63) / 64;  // 4 waves x 16 columns
    const int64_t cap = (int64_t)(ctx->cus > 0 ? ctx->cus : 256) * 2;
    return (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
}

int fail(qk_ctx* ctx, int code, const char* msg) {
    ctx->err = msg;
    return code;
}

// Workgroups of qk_prep_operands_kernel. A workgroup takes a tile of each side in turn; when both
// sides' tiles fit the resident workgroups at once (slice mode: 64 tiles per side at 8 ranks on the
// 96 preparation CUs) the grid is split, one side per workgroup (prep_split): 114 -> ? us at 8 ranks.
#ifndef QK_PREP_SPLIT
#define QK_PREP_SPLIT 1
#endif
bool prep_split(qk_ctx* ctx, int64_t NA, int64_t NB) {
    const int64_t tiles = (NA > NB ? NA : NB) / PCT;
    const int64_t g = (int64_t)(ctx->cus > 0 ? ctx->cus : 256) * QK_PREP_WG_PER_CU;
    return QK_PREP_SPLIT && tiles > 0 && 2 * tiles <= g;
}

int prep_grid(qk_ctx* ctx, int64_t NA, int64_t NB) {
    const int64_t tiles = (NA > NB ? NA : NB) / PCT;
    if (prep_split(ctx, NA, NB)) return (int)(2 * tiles);
    const int64_t g = (int64_t)(ctx->cus > 0 ? ctx->cus : 256) * QK_PREP_WG_PER_CU;
    return (int)(tiles < g ? (tiles > 0 ? tiles : 1) : g);
}

}  // namespace

extern "C" {

int qk_prep_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t NB, int64_t* bytes) {
    if (!ctx || !bytes) return QK_EARG;
    *bytes = (int64_t)prep_grid(ctx, NA, NB) * (PPA + PPB) * (int64_t)sizeof(double);
    return QK_OK;
}

int qk_prep_operands(qk_ctx* ctx, int K, int RA, const double* WtA, const double* qA, int64_t ldqA, int64_t NA,
                     double* XA, int RB, const double* WtB, const double* qB, int64_t ldqB, int64_t NB, double* XB,
                     const double* probes, double* GA, double* GB, double* U, double* work, int64_t work_bytes) {
    if (!ctx) return QK_EARG;
    if (K < 2 || K > PK || (K & 1) || RA < 1 || RB < 1)
        return fail(ctx, QK_EARG, "qk_prep_operands: need even 2 <= K <= 64 and R >= 1 on both sides");
    if (((reinterpret_cast<uintptr_t>(WtA) | reinterpret_cast<uintptr_t>(WtB) | reinterpret_cast<uintptr_t>(qA) |
          reinterpret_cast<uintptr_t>(qB)) & 15) || (ldqA & 1) || (ldqB & 1))
        return fail(ctx, QK_EARG, "qk_prep_operands: 16-B aligned Wt / q and even ldq required");
    if (NA < PCT || NB < PCT || NA % PCT || NB % PCT || ldqA < NA || ldqB < NB)
        return fail(ctx, QK_EARG, "qk_prep_operands: columns must be a positive multiple of 128 (ldq >= N)");
    if (!WtA || !qA || !XA || !WtB || !qB || !XB || !probes || !GA || !GB || !U || !work)
        return fail(ctx, QK_EARG, "qk_prep_operands: null buffer");
    const int G = prep_grid(ctx, NA, NB);
    if (work_bytes < (int64_t)G * (PPA + PPB) * (int64_t)sizeof(double))
        return fail(ctx, QK_EARG, "qk_prep_operands: workspace too small (qk_prep_workspace_bytes)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_prep_operands: hipSetDevice");
    PrepArgs args;
    args.s[0] = PrepSide{WtA, qA, ldqA, NA, RA, XA, nullptr};
    args.s[1] = PrepSide{WtB, qB, ldqB, NB, RB, XB, probes};
    args.K = K;
    args.split = prep_split(ctx, NA, NB) ? 1 : 0;
    args.part = work;
    hipLaunchKernelGGL(qk_prep_operands_kernel, dim3(G), dim3(PTH), 0, ctx->stream, args);
    const int outs = 2 * PPG + PNP * K;
    hipLaunchKernelGGL(qk_prep_reduce_kernel, dim3((outs + 63) / 64), dim3(64 * PRW), 0, ctx->stream, work, G, K, GA,
                       GB, U);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, QK_EHIP, (std::string("qk_prep_operands: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

/* q-space preparation (rows R <= 80 per side): the Grams G_A, G_B [K][K] and U = X_B P^T [K][16] of
 * X_s = Wt_s^T q_s without forming X (qknit_prep.hip "q-space preparation"). */
int qk_qprep_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t NB, int64_t* bytes) {
    if (!ctx || !bytes) return QK_EARG;
    const int G = prep_grid(ctx, NA, NB);
    const int64_t gb = (NB + QB_SPAN - 1) / QB_SPAN, ga = (NA + QA_COLS - 1) / QA_COLS;
    const int64_t grams = (int64_t)2 * G * QG_PART + 2 * QG_RMAX * QG_RMAX + QG_RMAX * PNP;
    const int64_t check = gb * QV_PART + ga * PE;
    *bytes = (grams > check ? grams : check) * (int64_t)sizeof(double);
    return QK_OK;
}

int qk_qprep_grams(qk_ctx* ctx, int K, int RA, const double* WtA, const double* qA, int64_t ldqA, int64_t NA, int RB,
                   const double* WtB, const double* qB, int64_t ldqB, int64_t NB, const double* probes, double* GA,
                   double* GB, double* U, double* work, int64_t work_bytes) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || RA < 1 || RB < 1 || RA > QG_RMAX || RB > QG_RMAX)
        return fail(ctx, QK_EARG, "qk_qprep_grams: need 1 <= K <= 64 and 1 <= R <= 80 on both sides");
    if (((reinterpret_cast<uintptr_t>(qA) | reinterpret_cast<uintptr_t>(qB) | reinterpret_cast<uintptr_t>(probes)) & 15) ||
        (ldqA & 1) || (ldqB & 1))
        return fail(ctx, QK_EARG, "qk_qprep_grams: 16-B aligned q / probes and even ldq required");
    if (NA < PCT || NB < PCT || NA % PCT || NB % PCT || ldqA < NA || ldqB < NB)
        return fail(ctx, QK_EARG, "qk_qprep_grams: columns must be a positive multiple of 128 (ldq >= N)");
    if (!WtA || !qA || !WtB || !qB || !probes || !GA || !GB || !U || !work)
        return fail(ctx, QK_EARG, "qk_qprep_grams: null buffer");
    int64_t need = 0;
    qk_qprep_workspace_bytes(ctx, NA, NB, &need);
    if (work_bytes < need) return fail(ctx, QK_EARG, "qk_qprep_grams: workspace too small (qk_qprep_workspace_bytes)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_qprep_grams: hipSetDevice");
    const int G = prep_grid(ctx, NA, NB);
    QGramArgs args;
    args.s[0] = QGramSide{qA, ldqA, NA, RA, nullptr};
    args.s[1] = QGramSide{qB, ldqB, NB, RB, probes};
    args.split = prep_split(ctx, NA, NB) ? 1 : 0;
    args.slots = args.split ? G / 2 : G;
    args.part = work;
    double* gq = work + (int64_t)2 * G * QG_PART;
    const size_t lds = (size_t)(RA > RB ? RA : RB) * QG_LD * sizeof(double);
    hipLaunchKernelGGL(qk_qgram_kernel, dim3(G), dim3(QG_T), lds, ctx->stream, args);
    hipLaunchKernelGGL(qk_qgram_reduce_kernel, dim3((2 * QG_PART + 63) / 64), dim3(64 * PRW), 0, ctx->stream, work,
                       args.slots, gq);
    hipLaunchKernelGGL(qk_qproject_kernel, dim3(2 * QP_CB + 1), dim3(256), 0, ctx->stream, K, RA, WtA, RB, WtB, gq, GA,
                       GB, U);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, QK_EHIP, (std::string("qk_qprep_grams: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

/* q-space compression + acceptance check: A2 = TA Wt_A^T q_A, B2 = TB Wt_B^T q_B ([rmax][N], rmax <= 8),
 * e2 / accepted rank exactly as qk_probe_errors over every column of A (U from qk_qprep_grams). */
int qk_qprep_compress_check(qk_ctx* ctx, int K, int rmax, int RA, const double* WtA, const double* qA, int64_t ldqA,
                            int64_t NA, int RB, const double* WtB, const double* qB, int64_t ldqB, int64_t NB,
                            const double* TA, const double* TB, const double* U, const double* probes, double* A2,
                            double* B2, double* e2, const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out,
                            double* err_out, double* work, int64_t work_bytes) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || rmax < 1 || rmax > 8 || RA < 1 || RB < 1 || RA > QG_RMAX || RB > QG_RMAX)
        return fail(ctx, QK_EARG, "qk_qprep_compress_check: need 1 <= K <= 64, 1 <= rmax <= 8, 1 <= R <= 80");
    if (NA % QA_COLS || NB % QB_COLS || NA < QA_COLS || NB < QB_COLS || ldqA < NA || ldqB < NB || (ldqA & 1) || (ldqB & 1))
        return fail(ctx, QK_EARG, "qk_qprep_compress_check: column counts must be positive multiples of 512");
    if (((reinterpret_cast<uintptr_t>(qA) | reinterpret_cast<uintptr_t>(qB) | reinterpret_cast<uintptr_t>(A2) |
          reinterpret_cast<uintptr_t>(B2) | reinterpret_cast<uintptr_t>(probes)) & 15))
        return fail(ctx, QK_EARG, "qk_qprep_compress_check: 16-B aligned buffers required");
    if (!WtA || !qA || !WtB || !qB || !TA || !TB || !U || !probes || !A2 || !B2 || !work || (k_out && !r_dev))
        return fail(ctx, QK_EARG, "qk_qprep_compress_check: null buffer");
    const int64_t gb = (NB + QB_SPAN - 1) / QB_SPAN, ga = NA / QA_COLS;
    if (work_bytes < (gb * QV_PART + ga * PE) * (int64_t)sizeof(double))
        return fail(ctx, QK_EARG, "qk_qprep_compress_check: workspace too small (qk_qprep_workspace_bytes)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_qprep_compress_check: hipSetDevice");
    double* vpart = work;
    double* epart = work + gb * QV_PART;
    hipLaunchKernelGGL(qk_qcompress_b_kernel, dim3((unsigned)gb), dim3(QB_T), 0, ctx->stream, K, rmax, RB, TB, WtB, qB,
                       ldqB, NB, probes, B2, vpart);
    hipLaunchKernelGGL(qk_qcompress_a_kernel, dim3((unsigned)ga), dim3(QA_T), 0, ctx->stream, K, rmax, RA, TA, WtA, qA,
                       ldqA, NA, U, vpart, (int)gb, A2, epart);
    hipLaunchKernelGGL(qk_probe_accept_kernel, dim3(1), dim3(256), 0, ctx->stream, epart, (int)ga, r_dev, tol, rel_tol,
                       e2, k_out, err_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(ctx, QK_EHIP, (std::string("qk_qprep_compress_check: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

int qk_compress_operands(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, double* A2,
                         const double* TB, const double* XB, int64_t NB, double* B2) {
    return qk_compress_operands_ld(ctx, K, rmax, TA, XA, NA, NA, A2, NA, TB, XB, NB, NB, B2, NB);
}

int qk_compress_operands_ld(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, int64_t ldxa,
                            double* A2, int64_t lda2, const double* TB, const double* XB, int64_t NB, int64_t ldxb,
                            double* B2, int64_t ldb2) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || rmax < 1 || rmax > 8 || NA < 1 || NB < 1)
        return fail(ctx, QK_EARG, "qk_compress_operands: need 1 <= K <= 64, 1 <= rmax <= 8, N >= 1");
    if (ldxa < NA || lda2 < NA || ldxb < NB || ldb2 < NB)
        return fail(ctx, QK_EARG, "qk_compress_operands: leading dimension below the width");
    if (!TA || !XA || !A2 || !TB || !XB || !B2) return fail(ctx, QK_EARG, "qk_compress_operands: null buffer");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_compress_operands: hipSetDevice");
    const int64_t N = NA > NB ? NA : NB;
    const bool cols = QK_COMPRESS_COLS && NA % 2 == 0 && NB % 2 == 0 && ldxa % 2 == 0 && lda2 % 2 == 0 &&
                      ldxb % 2 == 0 && ldb2 % 2 == 0 &&
                      !((reinterpret_cast<uintptr_t>(XA) | reinterpret_cast<uintptr_t>(XB) |
                         reinterpret_cast<uintptr_t>(A2) | reinterpret_cast<uintptr_t>(B2)) & 15);
    if (cols) {
        hipLaunchKernelGGL(qk_compress_cols_kernel, dim3((unsigned)((N + 127) / 128), 2), dim3(64), 0, ctx->stream, K,
                           rmax, TA, XA, NA, ldxa, A2, lda2, TB, XB, NB, ldxb, B2, ldb2);
    } else {
        int64_t gx = (N + 63) / 64;
        const int64_t cap = (int64_t)(ctx->cus > 0 ? ctx->cus : 256) * 4;  // x 2 sides: up to 8 workgroups per CU
        gx = gx < cap ? gx : cap;
        hipLaunchKernelGGL(qk_compress_kernel, dim3((unsigned)gx, 2), dim3(256), 0, ctx->stream, K, rmax, TA, XA, NA,
                           ldxa, A2, lda2, TB, XB, NB, ldxb, B2, ldb2);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(ctx, QK_EHIP, (std::string("qk_compress_operands: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

int qk_compress_probe_v(qk_ctx* ctx, int K, int rmax, const double* TA, const double* XA, int64_t NA, int64_t ldxa,
                        double* A2, int64_t lda2, const double* TB, const double* XB, int64_t NB, int64_t ldxb,
                        double* B2, int64_t ldb2, const double* probes, int64_t ldp, double* vpart,
                        int64_t vpart_doubles) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || rmax < 1 || rmax > 8 || NA < 2 || NB < 2 || (NA | NB | ldxa | lda2 | ldxb | ldb2) & 1)
        return fail(ctx, QK_EARG, "qk_compress_probe_v: need 1 <= K <= 64, 1 <= rmax <= 8, even widths and strides");
    if (ldxa < NA || lda2 < NA || ldxb < NB || ldb2 < NB || ldp < NB)
        return fail(ctx, QK_EARG, "qk_compress_probe_v: leading dimension below the width");
    if (!TA || !XA || !A2 || !TB || !XB || !B2 || !probes || !vpart)
        return fail(ctx, QK_EARG, "qk_compress_probe_v: null buffer");
    if ((reinterpret_cast<uintptr_t>(XA) | reinterpret_cast<uintptr_t>(XB) | reinterpret_cast<uintptr_t>(A2) |
         reinterpret_cast<uintptr_t>(B2)) & 15)
        return fail(ctx, QK_EARG, "qk_compress_probe_v: operands must be 16-B aligned");
    const int64_t ga = (NA + CV_COLS - 1) / CV_COLS, gb = (NB + CV_COLS - 1) / CV_COLS;
    if (vpart_doubles < gb * PV_PART) return fail(ctx, QK_EARG, "qk_compress_probe_v: vpart too small");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_compress_probe_v: hipSetDevice");
    hipLaunchKernelGGL(qk_compress_v_kernel, dim3((unsigned)(ga + gb)), dim3(256), 0, ctx->stream, K, rmax, TA, XA, NA,
                       ldxa, A2, lda2, TB, XB, NB, ldxb, B2, ldb2, probes, ldp, vpart, (int)ga);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(ctx, QK_EHIP, (std::string("qk_compress_probe_v: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

int qk_probe_errors_vpart(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                          int64_t lda2, const double* U, const double* vpart, int64_t gv, double* e2,
                          const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out, double* err_out,
                          double* work, int64_t work_bytes, int64_t* tally) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || rmax < 1 || rmax > 8 || NA < 16 || NA % 16 || gv < 1)
        return fail(ctx, QK_EARG, "qk_probe_errors_vpart: need 1 <= K <= 64, 1 <= rmax <= 8, NA % 16 == 0, gv >= 1");
    if (!XA || !A2 || !U || !vpart || !work || (k_out && !r_dev) || (tally && !k_out))
        return fail(ctx, QK_EARG, "qk_probe_errors_vpart: null buffer");
    if (ldx < NA) return fail(ctx, QK_EARG, "qk_probe_errors_vpart: leading dimension");
    const int gd = probe_grid_d(ctx, NA);
    if (work_bytes < (int64_t)(PV_GRID * PV_PART + gd * PE) * (int64_t)sizeof(double))
        return fail(ctx, QK_EARG, "qk_probe_errors_vpart: workspace too small (qk_probe_workspace_bytes)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_probe_errors_vpart: hipSetDevice");
    double* epart = work + PV_GRID * PV_PART;
    hipLaunchKernelGGL(qk_probe_d_kernel, dim3(gd), dim3(256), 0, ctx->stream, K, rmax, XA, ldx, NA, A2, lda2, U, vpart,
                       (int)gv, epart);
    hipLaunchKernelGGL(qk_probe_accept_kernel, dim3(1), dim3(256), 0, ctx->stream, epart, gd, r_dev, tol, rel_tol, e2,
                       k_out, err_out, tally);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(ctx, QK_EHIP, (std::string("qk_probe_errors_vpart: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

int qk_probe_workspace_bytes(qk_ctx* ctx, int64_t NA, int64_t* bytes) {
    if (!ctx || !bytes) return QK_EARG;
    *bytes = (int64_t)(PV_GRID * PV_PART + probe_grid_d(ctx, NA) * PE) * (int64_t)sizeof(double);
    return QK_OK;
}

int qk_probe_errors(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                    int64_t lda2, const double* U, const double* B2, int64_t ldb2, int64_t NB, const double* probes,
                    int64_t ldp, double* e2, const int32_t* r_dev, double tol, double rel_tol, int32_t* k_out,
                    double* err_out, double* work, int64_t work_bytes) {
    return qk_probe_errors_tally(ctx, K, rmax, XA, ldx, NA, A2, lda2, U, B2, ldb2, NB, probes, ldp, e2, r_dev, tol,
                                 rel_tol, k_out, err_out, work, work_bytes, nullptr);
}

int qk_probe_errors_tally(qk_ctx* ctx, int K, int rmax, const double* XA, int64_t ldx, int64_t NA, const double* A2,
                          int64_t lda2, const double* U, const double* B2, int64_t ldb2, int64_t NB,
                          const double* probes, int64_t ldp, double* e2, const int32_t* r_dev, double tol,
                          double rel_tol, int32_t* k_out, double* err_out, double* work, int64_t work_bytes,
                          int64_t* tally) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > PK || rmax < 1 || rmax > 8 || NA < 16 || NA % 16 || NB < 4 || NB % 4)
        return fail(ctx, QK_EARG, "qk_probe_errors: need 1 <= K <= 64, 1 <= rmax <= 8, NA % 16 == 0, NB % 4 == 0");
    if (!XA || !A2 || !U || !B2 || !probes || !work || (k_out && !r_dev) || (tally && !k_out))
        return fail(ctx, QK_EARG, "qk_probe_errors: null buffer");
    if (ldx < NA || ldb2 < NB || ldp < NB) return fail(ctx, QK_EARG, "qk_probe_errors: leading dimension");
    const int gd = probe_grid_d(ctx, NA);
    if (work_bytes < (int64_t)(PV_GRID * PV_PART + gd * PE) * (int64_t)sizeof(double))
        return fail(ctx, QK_EARG, "qk_probe_errors: workspace too small (qk_probe_workspace_bytes)");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_probe_errors: hipSetDevice");
    double* vpart = work;
    double* epart = work + PV_GRID * PV_PART;
    hipLaunchKernelGGL(qk_probe_v_kernel, dim3(PV_GRID), dim3(256), 0, ctx->stream, rmax, B2, ldb2, NB, probes, ldp,
                       vpart);
    hipLaunchKernelGGL(qk_probe_d_kernel, dim3(gd), dim3(256), 0, ctx->stream, K, rmax, XA, ldx, NA, A2, lda2, U, vpart,
                       PV_GRID, epart);
    hipLaunchKernelGGL(qk_probe_accept_kernel, dim3(1), dim3(256), 0, ctx->stream, epart, gd, r_dev, tol, rel_tol, e2,
                       k_out, err_out, tally);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, QK_EHIP, (std::string("qk_probe_errors: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

// Per-step statistics of the device data rank kept on the device (qk_rank_tally): acc[0] += (r == 0)
// (no factorisation of rank <= rmax), acc[1] += (r > 0 && k == 0) (probe check rejected), acc[2] = k
// (the last accepted rank), acc[3] += 1 (steps). The host reads acc only when asked
// (KnitPipeline.sync_stats), so a loop of steps never waits for the device.
__global__ __launch_bounds__(64) void qk_rank_tally_kernel(const int32_t* __restrict__ r, const int32_t* __restrict__ k,
                                                          int64_t* __restrict__ acc) {
    if (threadIdx.x == 0) {
        const int rv = *r, kv = *k;
        acc[0] += rv == 0 ? 1 : 0;
        acc[1] += (rv > 0 && kv == 0) ? 1 : 0;
        acc[2] = kv;
        acc[3] += 1;
    }
}

int qk_rank_tally(qk_ctx* ctx, const int32_t* r_dev, const int32_t* k_dev, int64_t* acc) {
    if (!ctx) return QK_EARG;
    if (!r_dev || !k_dev || !acc) return fail(ctx, QK_EARG, "qk_rank_tally: null buffer");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_rank_tally: hipSetDevice");
    hipLaunchKernelGGL(qk_rank_tally_kernel, dim3(1), dim3(64), 0, ctx->stream, r_dev, k_dev, acc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, QK_EHIP, (std::string("qk_rank_tally: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

int qk_probe_accept(qk_ctx* ctx, const double* e2, int n, const int32_t* r_dev, double tol, double rel_tol,
                    int32_t* k_out, double* err_out) {
    if (!ctx) return QK_EARG;
    if (!e2 || !r_dev || !k_out || n < 1) return fail(ctx, QK_EARG, "qk_probe_accept: null buffer or n < 1");
    if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, QK_EHIP, "qk_probe_accept: hipSetDevice");
    hipLaunchKernelGGL(qk_probe_accept_kernel, dim3(1), dim3(256), 0, ctx->stream, e2, n, r_dev, tol, rel_tol, nullptr,
                       k_out, err_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ctx, QK_EHIP, (std::string("qk_probe_accept: ") + hipGetErrorString(e)).c_str());
    return QK_OK;
}

}  // extern "C"
