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
2. Core ``C = L_A^T L_B`` ([r_A, r_B]): ``R ~= Q_A^T C Q_B``; SVD ``C = U S W^T``.
3. Rank ``r`` = singular values above ``max(s_tol * s_0, s_abs)``.
4. ``T_A = S_r^{1/2} U_r^T L_A[P_A]^{-1}`` placed in the pivot columns (``[r, K]``), ``T_B`` alike with
   ``W``: ``R ~= (T_A A)^T (T_B B)``.

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


def _side_factor(L: np.ndarray, piv: list, V: np.ndarray, s: np.ndarray, K: int) -> np.ndarray:
    """``S^{1/2} V^T L[P]^{-1}`` in the pivot columns of a [r, K] matrix."""
    LP = np.tril(L[piv])  # lower triangular up to rounding (a pivot row's later columns vanish)
    Y = np.linalg.solve(LP.T, V)  # L[P]^T Y = V  ->  Y^T = V^T L[P]^{-1}
    T = np.zeros((V.shape[1], K))
    T[:, piv] = (Y * np.sqrt(s)[None, :]).T
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
    U, s, Wt = np.linalg.svd(LA.T @ LB)
    if s.size == 0 or s[0] <= 0:
        return None
    r = int((s > max(s_tol * s[0], s_abs)).sum())
    if r == 0 or r > rmax:
        return None
    return _side_factor(LA, pa, U[:, :r], s[:r], K), _side_factor(LB, pb, Wt[:r].T, s[:r], K)


# the engine's historical name (pipeline host path, tests)
data_rank_factors = rank_factors
