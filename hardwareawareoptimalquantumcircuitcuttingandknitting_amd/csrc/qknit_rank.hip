// qknit_rank.hip — data-rank factors of a two-fragment knit on the GPU, one workgroup, no host trip.
//
// Device form of data_rank.rank_factors (see that module for the math): pivoted Cholesky of the two
// Gram matrices GA = A A^T, GB = B B^T (one wave per side, stopped on the residual trace), core
// C = L_A^T L_B, its rank-revealing LU with complete pivoting C ~= X Y^T (balanced columns), the rank r
// = pivots above the cut, and T_A = X^T L_A[P_A]^{-1}, T_B = Y^T L_B[P_B]^{-1} in the pivot columns,
// written as [rmax][K] (rows >= r zero)
// with r in *r_out. r_out = 0 means "no usable factorisation" (R = 0, no convergence within 32 pivot
// steps, or r > rmax): the caller's exact contraction then runs (predicated on the same int).
// The step that consumes these verifies the compressed product on the real operands
// (qk_probe_check, csrc/qknit_prep.hip) before trusting it, on the device too.
#include <hip/hip_runtime.h>

#include <cmath>

#include "internal.h"

namespace {

constexpr int RK_K = 64;   // operand rows (K) the kernel handles
constexpr int RK_RC = 32;  // pivoted-Cholesky steps per side
constexpr int RK_R = 8;    // largest rank written (rows of TA / TB)
constexpr int RK_THREADS = 128;

#ifdef QK_RANK_DEBUG  // tuning builds only (tools/build_variants.py): phase clocks + Jacobi sweep count
__device__ long long qk_rank_dbg[8];
#define RK_STAMP(i) \
    if (threadIdx.x == 0) qk_rank_dbg[i] = wall_clock64();
#else
#define RK_STAMP(i)
#endif

struct RankArgs {
    int K, rmax;
    const double* GA;
    const double* GB;
    double lam_tol, s_tol, s_abs;
    double* TA;
    double* TB;
    int32_t* r_out;
};

// Cross-lane reductions with DPP row operations (a few cycles each) and v_readlane across the four
// 16-lane rows, instead of ds_bpermute shuffles (~100+ cycles of LDS latency per step, serialised by
// the reduction's dependency chain: those made a Jacobi round cost ~1.5 us).
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
    int2 w = *reinterpret_cast<int2*>(&v);
    w.x = __builtin_amdgcn_mov_dpp(w.x, CTRL, 0xF, 0xF, false);
    w.y = __builtin_amdgcn_mov_dpp(w.y, CTRL, 0xF, 0xF, false);
    return *reinterpret_cast<double*>(&w);
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    int2 w = *reinterpret_cast<int2*>(&v);
    w.x = __builtin_amdgcn_readlane(w.x, l);
    w.y = __builtin_amdgcn_readlane(w.y, l);
    return *reinterpret_cast<double*>(&w);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

// 1/x and 1/sqrt(x) from the hardware estimates refined by one Newton step
__device__ __forceinline__ double rcp_d(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsq_d(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    return fma(y * 0.5, fma(-x * y, y, 1.0), y);
}

// sum over aligned groups of `width` lanes (1, 2, 4, 8, 16, 32, 64); every lane of a group gets it
__device__ __forceinline__ double wsum(double v, int width = 64) {
    if (width >= 2) v += dppd<DPP_XOR1>(v);
    if (width >= 4) v += dppd<DPP_XOR2>(v);
    if (width >= 8) v += dppd<DPP_HALF_MIRROR>(v);
    if (width >= 16) v += dppd<DPP_MIRROR>(v);
    if (width == 32) {
        const double lo = readlane_d(v, 0) + readlane_d(v, 16), hi = readlane_d(v, 32) + readlane_d(v, 48);
        v = (threadIdx.x & 32) ? hi : lo;
    } else if (width == 64) {
        v = (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
    }
    return v;
}

// wave-wide argmax of v (lowest index on ties); every lane gets (v, idx)
__device__ __forceinline__ void wargmax(double& v, int& idx) {
    auto take = [&](double v2, int i2) {
        if (v2 > v || (v2 == v && i2 < idx)) {
            v = v2;
            idx = i2;
        }
    };
    take(dppd<DPP_XOR1>(v), dppi<DPP_XOR1>(idx));
    take(dppd<DPP_XOR2>(v), dppi<DPP_XOR2>(idx));
    take(dppd<DPP_HALF_MIRROR>(v), dppi<DPP_HALF_MIRROR>(idx));
    take(dppd<DPP_MIRROR>(v), dppi<DPP_MIRROR>(idx));
    double bv = readlane_d(v, 0);
    int bi = __builtin_amdgcn_readlane(idx, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double v2 = readlane_d(v, r);
        const int i2 = __builtin_amdgcn_readlane(idx, r);
        if (v2 > bv || (v2 == bv && i2 < bi)) {
            bv = v2;
            bi = i2;
        }
    }
    v = bv;
    idx = bi;
}

__global__ __launch_bounds__(RK_THREADS) void qk_rank_factors_kernel(RankArgs a) {
    __shared__ double G[2][RK_K][RK_K + 1];
    __shared__ double L[2][RK_K][RK_RC + 1];
    __shared__ double C[RK_RC][RK_RC + 1];   // core, then the LU's residual
    __shared__ double Xs[RK_RC][RK_R + 2];   // balanced LU factor columns x_t, y_t
    __shared__ double Ys[RK_RC][RK_R + 2];
    __shared__ double Y[2][RK_R][RK_RC];     // triangular-solve results
    __shared__ int piv[2][RK_RC], nsteps[2], conv[2], rank_s, chol_live[2][2];
    __shared__ double Ts[2][RK_R][RK_K];       // T_A, T_B

    const int tid = threadIdx.x, lane = tid & 63, side = tid >> 6, K = a.K;
    RK_STAMP(0)
    {  // raw copy: wave 0 loads GA, wave 1 GB (lane = column), all K rows of a lane in flight at once
       // (round 3: unconditional loads with clamped indices; the round-2 loop of 16-row batches took one
       // memory round trip per batch, ~10 of the kernel's 26 us in the step where the Grams are cold)
       // — the symmetrisation 0.5 (G + G^T) happens where the Cholesky reads a column
        const double* Gs = side ? a.GB : a.GA;
        const int col = lane < K ? lane : K - 1;
        double v[RK_K];
#pragma unroll
        for (int u = 0; u < RK_K; ++u) v[u] = Gs[(u < K ? u : K - 1) * K + col];
#pragma unroll
        for (int u = 0; u < RK_K; ++u)
            if (u < K && lane < K) G[side][u][lane] = v[u];
        __syncthreads();
        RK_STAMP(4)
    }

    // ---- 1. pivoted Cholesky, wave `side` on Gram `side`, lane = row
    double d = lane < K ? G[side][lane][lane] : 0.0;
    bool alive = lane < K;
    double dmax = d;
    {
        int di = lane;
        wargmax(dmax, di);
    }
    bool active = dmax > 0.0, converged = !(dmax > 0.0);
    int steps = 0;
    for (int j = 0; j <= RK_RC; ++j) {  // both waves iterate alike: the barrier below is uniform
        if (active) {
            const double res = wsum(alive ? fmax(d, 0.0) : 0.0);
            if (res <= a.lam_tol * dmax) {
                converged = true;
                active = false;
            } else if (j == RK_RC) {
                active = false;
            } else {
                double v = alive ? d : -1.0;
                int idx = lane;
                wargmax(v, idx);  // lowest index on ties
                const int p = idx;
                const double dp = v;
                if (!(dp > 0.0)) {
                    active = false;
                } else {
                    double s = lane < K ? 0.5 * (G[side][lane][p] + G[side][p][lane]) : 0.0;
                    for (int i = 0; i < j; ++i) s -= L[side][lane][i] * L[side][p][i];
                    const double col = lane < K ? s / sqrt(dp) : 0.0;
                    if (lane < K) L[side][lane][j] = col;
                    d -= col * col;
                    if (lane == p) {
                        d = 0.0;
                        alive = false;
                        piv[side][j] = p;
                    }
                    steps = j + 1;
                }
            }
        }
        // both waves leave together once neither is active (double-buffered flags: no read/write race)
        if (lane == 0) chol_live[j & 1][side] = active ? 1 : 0;
        __syncthreads();
        if (!chol_live[j & 1][0] && !chol_live[j & 1][1]) break;
    }
    if (lane == 0) {
        nsteps[side] = steps;
        conv[side] = converged ? 1 : 0;
    }
    __syncthreads();
    const int ra = nsteps[0], rb = nsteps[1];
    bool ok = conv[0] && conv[1] && ra > 0 && rb > 0;
    RK_STAMP(1)

    // ---- 2. core C = L_A^T L_B
    if (ok) {
        for (int e = tid; e < ra * rb; e += RK_THREADS) {
            const int i = e / rb, j = e % rb;
            double s = 0.0;
            for (int k = 0; k < K; ++k) s += L[0][k][i] * L[1][k][j];
            C[i][j] = s;
        }
    }
    for (int e = tid; e < 2 * RK_R * RK_K; e += RK_THREADS) (&Ts[0][0][0])[e] = 0.0;
    __syncthreads();
    RK_STAMP(2)

    // ---- 3. complete-pivoting LU of the core (data_rank.cross_factors), wave 0: pivot t is the
    // residual's largest |entry| (lowest row-major index on ties), x_t = C[:, j] / sqrt|p|,
    // y_t = sign(p) C[i, :] / sqrt|p|, C -= x_t y_t^T; stop when the largest residual entry is at most
    // max(s_tol |p_0|, s_abs). At most rmax + 1 pivots: a (rmax + 1)-th one above the cut means r > rmax.
    // (Replaces round 2's one-sided Jacobi SVD of the core: ~9 sweeps x 7 rounds of serial rotations,
    // 25 us, for the same rank decision.)
    if (side == 0) {
        int r = 0;
        if (ok) {
            const int n = ra * rb;
            const int tmax = (ra < rb ? ra : rb) < a.rmax + 1 ? (ra < rb ? ra : rb) : a.rmax + 1;
            double cut = 0.0;
            for (int t = 0; t < tmax; ++t) {
                double v = -1.0;
                int idx = 1 << 30;
                for (int e = lane; e < n; e += 64) {
                    const double m = fabs(C[e / rb][e % rb]);
                    if (m > v) {  // ascending e: the first of equal entries stays
                        v = m;
                        idx = e;
                    }
                }
                wargmax(v, idx);
                if (t == 0) cut = fmax(a.s_tol * v, a.s_abs);
                if (!(v > cut)) break;
                const int pi = idx / rb, pj = idx % rb;
                const double p = C[pi][pj];
                const double sc = 1.0 / sqrt(fabs(p));
                const double xv = lane < ra ? C[lane][pj] * sc : 0.0;
                const double yv = lane < rb ? C[pi][lane] * (p > 0.0 ? sc : -sc) : 0.0;
                if (lane < ra) Xs[lane][t] = xv;
                if (lane < rb) Ys[lane][t] = yv;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                for (int e = lane; e < n; e += 64) {
                    const int i = e / rb, j = e % rb;
                    C[i][j] = fma(-Xs[i][t], Ys[j][t], C[i][j]);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                r = t + 1;
            }
            if (r > a.rmax || r > ra) r = 0;
        }
        if (lane == 0) rank_s = r;
    }
    __syncthreads();
    RK_STAMP(5)
    const int r = rank_s;

    // ---- 4. T_A[t][piv_A[i]] = y_i with L_A[P_A]^T y = x_t (T_B alike with y_t): back-substitution,
    // one thread per (side, t)
    if (tid < 2 * r) {
        const int sd = tid / r, t = tid % r;
        const int rx = sd ? rb : ra;
        double* y = Y[sd][t];
        for (int i = rx - 1; i >= 0; --i) {
            double v = sd ? Ys[i][t] : Xs[i][t];
            for (int k = i + 1; k < rx; ++k) v -= L[sd][piv[sd][k]][i] * y[k];
            y[i] = v / L[sd][piv[sd][i]][i];
        }
        for (int i = 0; i < rx; ++i) Ts[sd][t][piv[sd][i]] = y[i];
    }
    __syncthreads();
    for (int e = tid; e < a.rmax * K; e += RK_THREADS) {
        a.TA[e] = Ts[0][e / K][e % K];
        a.TB[e] = Ts[1][e / K][e % K];
    }
    if (tid == 0) *a.r_out = r;
    RK_STAMP(3)
#ifdef QK_RANK_DEBUG
    if (tid == 0) {
        qk_rank_dbg[6] = ra;
        qk_rank_dbg[7] = rb;
    }
#endif
}

}  // namespace

#ifdef QK_RANK_DEBUG
extern "C" int qk_rank_debug(long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(qk_rank_dbg), sizeof(long long) * 8) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int qk_rank_factors(qk_ctx* ctx, int64_t K, const double* GA, const double* GB, double lam_tol,
                               double s_tol, double s_abs, int rmax, double* TA, double* TB, int32_t* r_out) {
    if (!ctx) return QK_EARG;
    if (K < 1 || K > RK_K || rmax < 1 || rmax > RK_R) {
        ctx->err = "qk_rank_factors: need 1 <= K <= 64 and 1 <= rmax <= 8";
        return QK_EARG;
    }
    if (!GA || !GB || !TA || !TB || !r_out) {
        ctx->err = "qk_rank_factors: null buffer";
        return QK_EARG;
    }
    if (hipSetDevice(ctx->device) != hipSuccess) {
        ctx->err = "qk_rank_factors: hipSetDevice";
        return QK_EHIP;
    }
    RankArgs args{(int)K, rmax, GA, GB, lam_tol, s_tol, s_abs, TA, TB, r_out};
    hipLaunchKernelGGL(qk_rank_factors_kernel, dim3(1), dim3(RK_THREADS), 0, ctx->stream, args);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        ctx->err = std::string("qk_rank_factors: ") + hipGetErrorString(e);
        return QK_EHIP;
    }
    return QK_OK;
}
