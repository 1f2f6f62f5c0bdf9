// sweep_ops.h — per-fiber amplitude updates of the batched sweep (shared by the interpreter
// kernel in qknit.hip and the per-program kernels sweep_codegen.py generates for hiprtc).
// A thread holds a fiber of PER = 16 amplitudes (4 tile positions) in registers; fiber bit A of
// the register index r is the op's qubit.
#ifndef QKNIT_SWEEP_OPS_H
#define QKNIT_SWEEP_OPS_H
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace qk_sweep_ops {

constexpr int PER = 16;

__device__ __forceinline__ double2 cmul(double ar, double ai, double2 b) {
    return make_double2(fma(ar, b.x, -ai * b.y), fma(ar, b.y, ai * b.x));
}
// m0 * a + m1 * b with m given as (re, im) pairs
__device__ __forceinline__ double2 cmac2(const double* m, double2 a, double2 b) {
    double re = m[0] * a.x;
    re = fma(-m[1], a.y, re);
    re = fma(m[2], b.x, re);
    re = fma(-m[3], b.y, re);
    double im = m[0] * a.y;
    im = fma(m[1], a.x, im);
    im = fma(m[2], b.y, im);
    im = fma(m[3], b.x, im);
    return make_double2(re, im);
}

// LDS swizzle: XOR the low nibble with the two higher nibbles (bank spread for strided fibers)
__device__ __forceinline__ int swz(int t) { return t ^ (((t >> 4) ^ (t >> 8)) & 15); }

template <int A>
__device__ __forceinline__ void ap_u1(double2 (&v)[PER], const double* m) {
    double mm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) mm[i] = m[i];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (r & (1 << A)) continue;
        const double2 a = v[r], b = v[r | (1 << A)];
        v[r] = cmac2(mm, a, b);
        v[r | (1 << A)] = cmac2(mm + 4, a, b);
    }
}

template <int A>
__device__ __forceinline__ void ap_d1(double2 (&v)[PER], const double* d) {
    const double d0r = d[0], d0i = d[1], d1r = d[2], d1i = d[3];
#pragma unroll
    for (int r = 0; r < PER; ++r) v[r] = (r & (1 << A)) ? cmul(d1r, d1i, v[r]) : cmul(d0r, d0i, v[r]);
}

template <int A, int B>
__device__ __forceinline__ void ap_u2(double2 (&v)[PER], const double* m) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (r & ((1 << A) | (1 << B))) continue;
        const int i0 = r, i1 = r | (1 << A), i2 = r | (1 << B), i3 = r | (1 << A) | (1 << B);
        const double2 x0 = v[i0], x1 = v[i1], x2 = v[i2], x3 = v[i3];
        double2 y[4];
#pragma unroll
        for (int row = 0; row < 4; ++row) {
            const double* mr = m + row * 8;
            double2 s = cmac2(mr, x0, x1);
            const double2 t = cmac2(mr + 4, x2, x3);
            y[row] = make_double2(s.x + t.x, s.y + t.y);
        }
        v[i0] = y[0];
        v[i1] = y[1];
        v[i2] = y[2];
        v[i3] = y[3];
    }
}

template <int A, int B>
__device__ __forceinline__ void ap_d2(double2 (&v)[PER], const double* d) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const int k = ((r >> A) & 1) | (((r >> B) & 1) << 1);
        v[r] = cmul(d[2 * k], d[2 * k + 1], v[r]);
    }
}

template <int C, int T>
__device__ __forceinline__ void ap_cx(double2 (&v)[PER]) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (!(r & (1 << C)) || (r & (1 << T))) continue;
        const double2 t = v[r];
        v[r] = v[r | (1 << T)];
        v[r | (1 << T)] = t;
    }
}

template <int A, int B>
__device__ __forceinline__ void ap_swap(double2 (&v)[PER]) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if ((r & (1 << A)) && !(r & (1 << B))) {
            const int o = (r ^ (1 << A)) | (1 << B);
            const double2 t = v[r];
            v[r] = v[o];
            v[o] = t;
        }
    }
}

// Real 2x2 [m00 m01; m10 m11]: 4 FMA per amplitude instead of 8.
template <int A>
__device__ __forceinline__ void ap_u1r(double2 (&v)[PER], const double* m) {
    const double m00 = m[0], m01 = m[1], m10 = m[2], m11 = m[3];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (r & (1 << A)) continue;
        const double2 a = v[r], b = v[r | (1 << A)];
        v[r] = make_double2(fma(m00, a.x, m01 * b.x), fma(m00, a.y, m01 * b.y));
        v[r | (1 << A)] = make_double2(fma(m10, a.x, m11 * b.x), fma(m10, a.y, m11 * b.y));
    }
}

// [m00, i p01; i p10, m11] with real m00, p01, p10, m11 (rx-type): 4 FMA per amplitude.
template <int A>
__device__ __forceinline__ void ap_u1x(double2 (&v)[PER], const double* m) {
    const double m00 = m[0], p01 = m[1], p10 = m[2], m11 = m[3];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (r & (1 << A)) continue;
        const double2 a = v[r], b = v[r | (1 << A)];
        v[r] = make_double2(fma(m00, a.x, -p01 * b.y), fma(m00, a.y, p01 * b.x));
        v[r | (1 << A)] = make_double2(fma(m11, b.x, -p10 * a.y), fma(m11, b.y, p10 * a.x));
    }
}

template <int A>
__device__ __forceinline__ void ap_d1r(double2 (&v)[PER], const double* d) {
    const double d0 = d[0], d1 = d[1];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const double s = (r & (1 << A)) ? d1 : d0;
        v[r] = make_double2(s * v[r].x, s * v[r].y);
    }
}

// Sign flip by XOR of the high dwords (mask 0x80000000 or 0): the +-1 diagonals and scalars the
// per-program kernels select from state bits cost two 32-bit ops instead of two f64 multiplies.
__device__ __forceinline__ double2 flip_sign(double2 z, unsigned m) {
    return make_double2(__hiloint2double(__double2hiint(z.x) ^ (int)m, __double2loint(z.x)),
                        __hiloint2double(__double2hiint(z.y) ^ (int)m, __double2loint(z.y)));
}

template <int A>
__device__ __forceinline__ void ap_d1s(double2 (&v)[PER], unsigned m0, unsigned m1) {
#pragma unroll
    for (int r = 0; r < PER; ++r) v[r] = flip_sign(v[r], (r & (1 << A)) ? m1 : m0);
}

template <int A, int B>
__device__ __forceinline__ void ap_d2r(double2 (&v)[PER], const double* d) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const double s = d[((r >> A) & 1) | (((r >> B) & 1) << 1)];
        v[r] = make_double2(s * v[r].x, s * v[r].y);
    }
}

// Cross-lane exchange of one fiber (register) bit with lane bit 4 or 5 (CDNA4 v_permlane16_swap /
// v_permlane32_swap: lanes 16-31 (48-63) of the first operand trade places with lanes 0-15 (32-47) of the
// second). Applied to the register pairs (r, r | 1 << I) it transposes register bit I with lane bit T:
// afterwards register bit I holds the qubit lane bit T held, and lane bit T the one register bit I held.
// The per-program kernels use it where the next fiber group needs at most two qubits that sit on lane
// bits 4 / 5 (a 1-2-bit butterfly boundary): 8 x 4 dword swaps per bit instead of the tile's round trip
// through LDS (16 writes, a barrier, 16 reads).
template <int T>
__device__ __forceinline__ void lane_swap(double& a, double& b) {
    static_assert(T == 4 || T == 5, "lane bit 4 or 5");
    const unsigned alo = (unsigned)__double2loint(a), ahi = (unsigned)__double2hiint(a);
    const unsigned blo = (unsigned)__double2loint(b), bhi = (unsigned)__double2hiint(b);
    if constexpr (T == 5) {
        const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
        a = __hiloint2double((int)hi[0], (int)lo[0]);
        b = __hiloint2double((int)hi[1], (int)lo[1]);
    } else {
        const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
        a = __hiloint2double((int)hi[0], (int)lo[0]);
        b = __hiloint2double((int)hi[1], (int)lo[1]);
    }
}

template <int I, int T>
__device__ __forceinline__ void xchg_lane_bit(double2 (&v)[PER]) {
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (r & (1 << I)) continue;
        lane_swap<T>(v[r].x, v[r | (1 << I)].x);
        lane_swap<T>(v[r].y, v[r | (1 << I)].y);
    }
}

// The same transposition for any lane bit L of the wave (0..5) through __shfl_xor (ds_bpermute / DPP):
// per dword one cross-lane move and three selects, where the swap instructions above take one. The
// FINAL passes use it for the positions that cannot be put on lane bits 4 / 5, so that no transition
// of theirs needs the LDS tile (QKNIT_SWEEP_LANE_XCHG=2).
template <int L>
__device__ __forceinline__ void lane_xor_swap(double& a, double& b, bool hi) {
    const double s = hi ? a : b;
    const double t = __shfl_xor(s, 1 << L, 64);
    a = hi ? t : a;
    b = hi ? b : t;
}

template <int I, int L>
__device__ __forceinline__ void xchg_lane_bit_any(double2 (&v)[PER]) {
    if constexpr (L == 4 || L == 5) {
        xchg_lane_bit<I, L>(v);
    } else {
        const bool hi = (__lane_id() >> L) & 1;
#pragma unroll
        for (int r = 0; r < PER; ++r) {
            if (r & (1 << I)) continue;
            lane_xor_swap<L>(v[r].x, v[r | (1 << I)].x, hi);
            lane_xor_swap<L>(v[r].y, v[r | (1 << I)].y, hi);
        }
    }
}

}  // namespace qk_sweep_ops

#endif  // QKNIT_SWEEP_OPS_H
