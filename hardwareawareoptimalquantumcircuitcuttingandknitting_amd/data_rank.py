"""Data-rank factors of a two-fragment knit ``R = A^T B`` from its Gram matrices.

The knit of two fragments is ``R[x_A, x_B] = sum_k A[k, x_A] B[k, x_B]`` (``A``, ``B``: the
``[K, 2^m]`` operands after the factored transforms; ``virtual_circuit.py:50-68`` in the reference).
Its numerical rank is often far below ``K`` (syc 32 5: K = 64, rank 2), and the write-bound
small-K knit then replaces the K = 64 MFMA contraction. This module is the host implementation of
the factorisation; ``qk_rank_factors`` (``csrc/qknit_rank.hip``) runs the same steps on the GPU in
one workgroup (no host round trip), so this is also the reference its tests compare against.

Steps, on ``GA = A A^T`` and ``GB = B B^T`` ([K, K]):

1. Pivoted Cholesky of each Gram: ``G ~= L L^T`` (``L``: [K, r_X]), greedy on the largest residual
   diagonal (ties: lowest index), stopped when the residual trace is at most ``lam_tol * max diag G``
   (the dropped part ``E = G - L L^T`` is PSD, so its largest eigenvalue is below its trace). In
   terms of the operand, ``A = L_A Q_A + E_A`` with orthonormal rows ``Q_A`` spanning the pivot rows
   of ``A`` and ``||E_A||_F^2 = trace(E)``; the pivot rows lie in that span exactly, so
   ``Q_A = L_A[P_A]^{-1} A[P_A]`` (``L_A[P_A]``: lower triangular).
2. Core ``C = L_A^T L_B`` ([r_A, r_B]): ``R ~= Q_A^T C Q_B``.
3. Rank-revealing LU of the core with complete pivoting (cross approximation): pivot ``t`` is the
   largest ``|entry|`` of the residual ``C_t`` (ties: lowest row-major index), ``x_t = C_t[:, j] /
   sqrt|p|``, ``y_t = sign(p) C_t[i, :] / sqrt|p|``, ``C_{t+1} = C_t - x_t y_t^T``; stop when the
   residual's largest entry is at most ``max(s_tol * |p_0|, s_abs)`` (its spectral norm is then at
   most ``sqrt(r_A r_B)`` times that, and so is every moved entry of ``R``). ``C ~= X Y^T`` with balanced
   columns, ``r`` = the pivots taken. (Earlier rounds took the core's SVD by one-sided Jacobi: 25 us
   of serial rotations on the device for the same rank decision; the probe check below is what
   certifies either.)
4. ``T_A = X^T L_A[P_A]^{-1}`` placed in the pivot columns (``[r, K]``), ``T_B = Y^T L_B[P_B]^{-1}``:
   ``R ~= (T_A A)^T (T_B B)``.

Nothing here is trusted for accuracy: the Grams square the condition number, so the caller verifies
the compressed product on the real operands against fixed Gaussian probes (``qk_probe_errors``,
``KnitPipeline``) and takes the exact contraction when the check fails. Returns None when there is nothing to compress to
(``R = 0``, the pivoting did not converge in ``rc_max`` steps, or ``r > rmax``).
"""
from __future__ import annotations

import numpy as np

LAM_TOL = 1e-12  # residual Gram trace / max diagonal at which the pivoted Cholesky stops
S_TOL = 1e-13    # singular values of the core kept above S_TOL * s_0 ...
S_ABS = 1e-15    # ... and above S_ABS (a dropped singular value moves entries of R by at most itself)
RC_MAX = 32      # pivoted-Cholesky steps per side (qknit_rank.hip keeps L in LDS: [64][32])
R_MAX = 8        # largest compressed rank the small-K knit kernels take
K_MAX = 64       # operand rows the device kernel handles


def pivoted_cholesky(G: np.ndarray, lam_tol: float = LAM_TOL, rc_max: int = RC_MAX):
    """``(L [K, r], pivots, converged)`` of a PSD matrix (see module doc, step 1)."""
    K = G.shape[0]
    d = np.diag(G).astype(np.float64).copy()
    dmax = float(d.max()) if K else 0.0
    if dmax <= 0:
        return np.zeros((K, 0)), [], True
    L = np.zeros((K, rc_max))
    alive = np.ones(K, dtype=bool)
    piv: list = []
    for j in range(rc_max + 1):
        if float(np.maximum(d[alive], 0.0).sum()) <= lam_tol * dmax:
            return L[:, :j], piv, True
        if j == rc_max:
            break
        cand = np.where(alive, d, -np.inf)
        p = int(np.argmax(cand))
        dp = d[p]
        if dp <= 0:
            break
        col = (G[:, p] - L[:, :j] @ L[p, :j]) / np.sqrt(dp)
        L[:, j] = col
        d -= col * col
        d[p] = 0.0
        alive[p] = False
        piv.append(p)
    return L[:, :len(piv)], piv, False


def cross_factors(C: np.ndarray, s_tol: float = S_TOL, s_abs: float = S_ABS, rmax: int = R_MAX):
    """``(X [r_A, r], Y [r_B, r])`` with ``C ~= X Y^T`` by complete-pivoting LU (module doc, step 3);
    ``r`` may exceed ``rmax`` by one (the caller rejects that), 0 when ``C = 0``."""
    R = np.array(C, dtype=np.float64)
    ra, rb = R.shape
    X, Y = [], []
    p0 = float(np.abs(R).max()) if R.size else 0.0
    if p0 <= 0:
        return np.zeros((ra, 0)), np.zeros((rb, 0))
    cut = max(s_tol * p0, s_abs)
    for _ in range(min(ra, rb, rmax + 1)):
        flat = int(np.argmax(np.abs(R)))  # first (row-major) on ties
        i, j = divmod(flat, rb)
        p = R[i, j]
        if not abs(p) > cut:
            break
        sc = 1.0 / np.sqrt(abs(p))
        x, y = R[:, j] * sc, R[i, :] * (sc if p > 0 else -sc)
        R = R - np.outer(x, y)
        X.append(x)
        Y.append(y)
    return np.array(X).T.reshape(ra, -1), np.array(Y).T.reshape(rb, -1)


def _side_factor(L: np.ndarray, piv: list, V: np.ndarray, K: int) -> np.ndarray:
    """``V^T L[P]^{-1}`` in the pivot columns of a [r, K] matrix."""
    LP = np.tril(L[piv])  # lower triangular up to rounding (a pivot row's later columns vanish)
    Y = np.linalg.solve(LP.T, V)  # L[P]^T Y = V  ->  Y^T = V^T L[P]^{-1}
    T = np.zeros((V.shape[1], K))
    T[:, piv] = Y.T
    return T


def rank_factors(GA: np.ndarray, GB: np.ndarray, lam_tol: float = LAM_TOL, s_tol: float = S_TOL,
                 s_abs: float = S_ABS, rmax: int = R_MAX, rc_max: int = RC_MAX):
    """``(T_A, T_B)`` ([r, K] each) with ``R = A^T B ~= (T_A A)^T (T_B B)``, or None."""
    K = GA.shape[0]
    GA = 0.5 * (GA + GA.T)
    GB = 0.5 * (GB + GB.T)
    LA, pa, oka = pivoted_cholesky(GA, lam_tol, rc_max)
    LB, pb, okb = pivoted_cholesky(GB, lam_tol, rc_max)
    if not (oka and okb) or not pa or not pb:
        return None
    X, Y = cross_factors(LA.T @ LB, s_tol, s_abs, rmax)
    r = X.shape[1]
    if r == 0 or r > rmax:
        return None
    return _side_factor(LA, pa, X, K), _side_factor(LB, pb, Y, K)


# the engine's historical name (pipeline host path, tests)
data_rank_factors = rank_factors
