// qknit_rank.hip — data-rank factors of a two-fragment knit on the GPU, one workgroup, no host trip.
//
// Device form of data_rank.rank_factors (see that module for the math): pivoted Cholesky of the two
// Gram matrices GA = A A^T, GB = B B^T (one wave per side, stopped on the residual trace), core
// C = L_A^T L_B, its SVD by one-sided (Hestenes) Jacobi rotations on C's columns, the numerical rank r,
// and T_X = S_r^{1/2} V_r^T L_X[P_X]^{-1} in the pivot columns, written as [rmax][K] (rows >= r zero)
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
constexpr int RK_MAX_SWEEPS = 40;

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
    __shared__ double C[RK_RC][RK_RC + 1];   // core, then U S in its columns
    __shared__ double W[RK_RC][RK_RC + 1];   // right rotations
    __shared__ double Y[2][RK_R][RK_RC];     // triangular-solve results
    __shared__ double sv[RK_RC];
    __shared__ int piv[2][RK_RC], nsteps[2], conv[2], order[RK_RC], rank_s, chol_live[2][2];
    __shared__ double cnorm2;
    __shared__ double Ts[2][RK_R][RK_K];       // T_A, T_B

    const int tid = threadIdx.x, lane = tid & 63, side = tid >> 6, K = a.K;
    RK_STAMP(0)
    {  // raw copy, wave w on rows w*16.. of [GA; GB] (lane = column), 16 loads in flight per lane and no
       // integer division in the index math (the divide-by-K form cost ~10 us); the symmetrisation
       // 0.5 (G + G^T) happens where the Cholesky reads a column
        const int wv = tid >> 6;
        for (int r0 = wv * 16; r0 < 2 * K; r0 += 32) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int rr = r0 + u;
                v[u] = (rr < 2 * K && lane < K) ? (rr < K ? a.GA[rr * K + lane] : a.GB[(rr - K) * K + lane]) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int rr = r0 + u;
                if (rr < 2 * K && lane < K) {
                    const int s = rr >= K ? 1 : 0;
                    G[s][rr - s * K][lane] = v[u];
                }
            }
        }
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

    // ---- 2. core C = L_A^T L_B, W = I
    if (ok) {
        for (int e = tid; e < ra * rb; e += RK_THREADS) {
            const int i = e / rb, j = e % rb;
            double s = 0.0;
            for (int k = 0; k < K; ++k) s += L[0][k][i] * L[1][k][j];
            C[i][j] = s;
        }
        for (int e = tid; e < rb * rb; e += RK_THREADS) W[e / rb][e % rb] = (e / rb == e % rb) ? 1.0 : 0.0;
    }
    __syncthreads();

    // ---- 3. one-sided Jacobi on C's columns (round-robin pairs, one thread group per pair). Pairs of
    // columns both below 1e-15 of the largest column norm are left alone: their singular values are
    // far under the rank cut (s_tol = 1e-13), and rotating rounding noise would keep the sweeps going
    if (ok && tid == 0) {
        double m = 0.0;
        for (int j = 0; j < rb; ++j) {
            double c2 = 0.0;
            for (int i = 0; i < ra; ++i) c2 += C[i][j] * C[i][j];
            m = fmax(m, c2);
        }
        cnorm2 = m;
    }
    __syncthreads();
    if (ok && rb > 1 && ra <= 8 && rb <= 8 && side == 0) {
        // Register form for cores of at most 8 x 8 (syc 32 5: the common case): lane 8 j + i holds
        // C[i][j] and W[i][j]; a round's partner column comes by one ds_bpermute per matrix and the
        // column sums by 3-step DPP reductions over the column's 8 lanes, so a round is a short
        // register chain instead of LDS round trips (same rotations, same pairing, same stopping rule
        // as the LDS form below)
        const int i = lane & 7, j = lane >> 3;
        const double floor2 = 1e-30 * cnorm2;
        double c = (i < ra && j < rb) ? C[i][j] : 0.0;
        double w = (i < rb && j < rb) ? W[i][j] : 0.0;
        const int n = rb + (rb & 1);
        auto perm = [](double v, int src_lane) {
            int2 x = *reinterpret_cast<int2*>(&v);
            x.x = __builtin_amdgcn_ds_bpermute(src_lane << 2, x.x);
            x.y = __builtin_amdgcn_ds_bpermute(src_lane << 2, x.y);
            return *reinterpret_cast<double*>(&x);
        };
        for (int sweep = 0; sweep < RK_MAX_SWEEPS; ++sweep) {
            bool rot = false;
            for (int round = 0; round < n - 1; ++round) {
                // partner of column j in this round (the LDS form's round-robin pairs)
                int pj;
                if (j == n - 1) pj = round;
                else if (j == round) pj = n - 1;
                else pj = (2 * round - j + 2 * (n - 1)) % (n - 1);
                const bool live = j < n && pj < rb && j < rb;
                const int src = (pj & 7) * 8 + i;
                const double cq = perm(c, src), wq = perm(w, src);
                double own = c * c, oth = cq * cq, cross = c * cq;
                own += dppd<DPP_XOR1>(own);
                oth += dppd<DPP_XOR1>(oth);
                cross += dppd<DPP_XOR1>(cross);
                own += dppd<DPP_XOR2>(own);
                oth += dppd<DPP_XOR2>(oth);
                cross += dppd<DPP_XOR2>(cross);
                own += dppd<DPP_HALF_MIRROR>(own);
                oth += dppd<DPP_HALF_MIRROR>(oth);
                cross += dppd<DPP_HALF_MIRROR>(cross);
                const bool lo = j < pj;  // column p of the pair (p < q)
                const double al = lo ? own : oth, be = lo ? oth : own, ga = cross;
                if (live && ga != 0.0 && fabs(ga) > 1e-13 * sqrt(al * be) && fmax(al, be) > floor2) {
                    const double zeta = (be - al) * 0.5 * rcp_d(ga);
                    const double ww = 1.0 + zeta * zeta;
                    const double tt = copysign(rcp_d(fabs(zeta) + ww * rsq_d(ww)), zeta);
                    const double cs = rsq_d(1.0 + tt * tt), sn = cs * tt;
                    // p: c' = cs c_p - sn c_q;  q: c' = sn c_p + cs c_q
                    c = lo ? cs * c - sn * cq : sn * cq + cs * c;
                    w = lo ? cs * w - sn * wq : sn * wq + cs * w;
                    rot = true;
                }
            }
#ifdef QK_RANK_DEBUG
            if (lane == 0) qk_rank_dbg[5] = sweep + 1;
#endif
            if (!__any(rot)) break;
        }
        if (i < ra && j < rb) C[i][j] = c;
        if (i < rb && j < rb) W[i][j] = w;
    } else if (ok && rb > 1 && side == 0) {  // wave 0 alone: rounds are ordered by the wave's own LDS traffic
        const double floor2 = 1e-30 * cnorm2;
        const int n = rb + (rb & 1), npair = n / 2;
        int tpp = 64 / npair;
        int pw = 1;
        while (pw * 2 <= tpp) pw *= 2;
        tpp = pw;  // power of two lanes per pair
        const int g = lane / tpp, t = lane % tpp;
        for (int sweep = 0; sweep < RK_MAX_SWEEPS; ++sweep) {
            bool rot = false;
            for (int round = 0; round < n - 1; ++round) {
                int p = -1, q = -1;
                if (g < npair) {
                    if (g == 0) {
                        p = round;
                        q = n - 1;
                    } else {
                        p = (round + g) % (n - 1);
                        q = (round - g + (n - 1)) % (n - 1);
                    }
                    if (p > q) {
                        const int x = p;
                        p = q;
                        q = x;
                    }
                }
                const bool live = g < npair && q < rb;
                double al = 0.0, be = 0.0, ga = 0.0;
                if (live)
                    for (int i = t; i < ra; i += tpp) {
                        const double cp = C[i][p], cq = C[i][q];
                        al += cp * cp;
                        be += cq * cq;
                        ga += cp * cq;
                    }
                al = wsum(al, tpp);
                be = wsum(be, tpp);
                ga = wsum(ga, tpp);
                // the factors only need to be good enough for the probe check that follows (1e-13
                // relative orthogonality instead of 1e-15: fewer sweeps chasing rounding)
                if (live && ga != 0.0 && fabs(ga) > 1e-13 * sqrt(al * be) && fmax(al, be) > floor2) {
                    // hardware reciprocal / reciprocal-sqrt seeds + one Newton step each (full double
                    // precision without the IEEE division / sqrt sequences): this is the serial chain
                    // of every Jacobi round
                    const double zeta = (be - al) * 0.5 * rcp_d(ga);
                    const double w = 1.0 + zeta * zeta;
                    const double tt = copysign(rcp_d(fabs(zeta) + w * rsq_d(w)), zeta);
                    const double c = rsq_d(1.0 + tt * tt), s = c * tt;
                    for (int i = t; i < ra; i += tpp) {
                        const double cp = C[i][p], cq = C[i][q];
                        C[i][p] = c * cp - s * cq;
                        C[i][q] = s * cp + c * cq;
                    }
                    for (int i = t; i < rb; i += tpp) {
                        const double wp = W[i][p], wq = W[i][q];
                        W[i][p] = c * wp - s * wq;
                        W[i][q] = s * wp + c * wq;
                    }
                    rot = true;
                }
                // this round's column writes land before the next round's reads (same wave: LDS is in order)
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
#ifdef QK_RANK_DEBUG
            if (lane == 0) qk_rank_dbg[5] = sweep + 1;
#endif
            if (!__any(rot)) break;
        }
    }
    __syncthreads();

    RK_STAMP(2)
    // ---- 4. singular values (column norms), descending order, rank
    if (ok && tid < rb) {
        double s = 0.0;
        for (int i = 0; i < ra; ++i) s += C[i][tid] * C[i][tid];
        sv[tid] = sqrt(s);
    }
    __syncthreads();
    if (tid == 0) {
        int r = 0;
        if (ok) {
            for (int j = 0; j < rb; ++j) order[j] = j;
            for (int j = 0; j < rb; ++j)  // selection sort, stable
                for (int k = j + 1; k < rb; ++k)
                    if (sv[order[k]] > sv[order[j]]) {
                        const int x = order[j];
                        order[j] = order[k];
                        order[k] = x;
                    }
            const double s0 = sv[order[0]];
            const double cut = fmax(a.s_tol * s0, a.s_abs);
            if (s0 > 0.0)
                for (int j = 0; j < rb; ++j) r += sv[order[j]] > cut ? 1 : 0;
            if (r > a.rmax || r > ra) r = 0;
        }
        rank_s = r;
    }
    for (int e = tid; e < 2 * RK_R * RK_K; e += RK_THREADS) (&Ts[0][0][0])[e] = 0.0;
    __syncthreads();
    const int r = rank_s;

    // ---- 5. T_X[j][piv_X[i]] = sqrt(s_j) y_i,  L_X[P_X]^T y = v_j  (back-substitution, one thread each)
    if (tid < 2 * r) {
        const int sd = tid / r, j = tid % r, col = order[j];
        const int rx = sd ? rb : ra;
        const double sj = sv[col];
        double* y = Y[sd][j];
        for (int i = rx - 1; i >= 0; --i) {
            double v = sd ? W[i][col] : C[i][col] / sj;
            for (int k = i + 1; k < rx; ++k) v -= L[sd][piv[sd][k]][i] * y[k];
            y[i] = v / L[sd][piv[sd][i]][i];
        }
        const double rs = sqrt(sj);
        for (int i = 0; i < rx; ++i) Ts[sd][j][piv[sd][i]] = rs * y[i];
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
