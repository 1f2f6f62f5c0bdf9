"""Label algebra of the knit: global labels, coefficients, fragment row maps, keys.

Restates the label bookkeeping of ``third_party/qvm/qvm/virtual_circuit.py``
as index arrays, so the contraction can run as dense GEMMs:

* global labels ``l`` = ``itertools.product(range(n_0), ..., range(n_{K-1}))``,
  last gate fastest (``_global_inst_labels``, ``:133-137``);
* fragment row of ``l`` = position of ``_global_to_fragment_inst_label`` in
  ``get_instance_labels(fragment)`` (``:39-48,139-163``) = mixed-radix index
  over the gates touching the fragment;
* coefficient ``c_l = prod_j a_j(l_j)`` where ``a_j`` is the knit rule of gate
  ``j`` (``virtual_gates.py:105-124,179-194,262-286``), config-bit outcomes
  already folded into the fragment rows with sign ``(-1)^m``;
* output key of fragment outcome ``x_f`` = bit-deposit of ``x_f`` into the
  fragment's global ``meas`` clbits (the XOR merge of ``quasi_distr.py:55-60``
  with disjoint supports).

The knit is then ``R[sum_f key_f(x_f)] = sum_l c_l prod_f q_f[row_f(l)][x_f]``.

``factor_vgate`` implements the optional *factored* knit: per
virtual gate, instantiations whose side programs coincide are merged, which
turns the ``n_j``-term sum into a rank-``r_j`` one (4 for every gate type in
the reference); the contraction dimension drops from ``prod n_j`` to
``prod r_j`` with identical results up to fp64 rounding.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def deposit_keys(clbits: list, dtype=np.int64) -> np.ndarray:
    """key[x] for x in [0, 2^len(clbits)): bit i of x -> bit clbits[i] of the key."""
    m = len(clbits)
    keys = np.zeros(1 << m, dtype=dtype)
    for i, c in enumerate(clbits):
        keys[np.arange(1 << m) >> i & 1 == 1] += np.int64(1) << np.int64(c)
    return keys


@dataclass
class LabelSpace:
    n_inst: list  # instantiation count per virtual gate (circuit order)
    coefs: list  # per gate: list of a_j(i)

    @property
    def num_labels(self) -> int:
        return int(np.prod(self.n_inst)) if self.n_inst else 1

    def global_labels(self) -> np.ndarray:
        """[L, K] array, last gate fastest."""
        K = len(self.n_inst)
        if K == 0:
            return np.zeros((1, 0), dtype=np.int64)
        grids = np.meshgrid(*[np.arange(n) for n in self.n_inst], indexing="ij")
        return np.stack([g.ravel() for g in grids], axis=1).astype(np.int64)

    def coefficients(self) -> np.ndarray:
        labels = self.global_labels()
        c = np.ones(labels.shape[0], dtype=np.float64)
        for j, a in enumerate(self.coefs):
            c *= np.asarray(a, dtype=np.float64)[labels[:, j]]
        return c

    def fragment_rows(self, touches: list) -> np.ndarray:
        """Row of each global label in the fragment's label list (touches[j]: bool)."""
        labels = self.global_labels()
        rows = np.zeros(labels.shape[0], dtype=np.int64)
        for j, t in enumerate(touches):
            if t:
                rows = rows * self.n_inst[j] + labels[:, j]
        return rows


# ----------------------------------------------------------------------------- factored knit
def _signature(endpoint, inst_id: int) -> tuple:
    from .fragment_program import side_program

    side = side_program(endpoint, inst_id)
    sig = []
    for instr in side.data:
        op = instr.operation
        sig.append((op.name, tuple(round(float(p), 15) for p in getattr(op, "params", ()))))
    return tuple(sig)


def factor_vgate(ep0, ep1, coefs: list, tol: float = 1e-14):
    """Rank factorisation of one virtual gate's knit term.

    Returns ``(T0, T1)`` with shapes ``[r, n]`` such that for every pair of
    side-indexed vectors ``u_i`` (side 0) and ``v_i`` (side 1) that depend on
    the instantiation only through that side's program,
    ``sum_i a_i u_i (x) v_i == sum_r (T0 u)_r (x) (T1 v)_r``.
    """
    n = len(coefs)
    s0 = [_signature(ep0, i) for i in range(n)]
    s1 = [_signature(ep1, i) for i in range(n)]
    u0 = {s: k for k, s in enumerate(dict.fromkeys(s0))}
    u1 = {s: k for k, s in enumerate(dict.fromkeys(s1))}
    C = np.zeros((len(u0), len(u1)))
    for i in range(n):
        C[u0[s0[i]], u1[s1[i]]] += coefs[i]
    # exact-ish rank factorisation C = L @ R by complete pivoting (entries are small dyadics)
    Cw = C.copy()
    Ls, Rs = [], []
    while True:
        idx = np.unravel_index(np.argmax(np.abs(Cw)), Cw.shape)
        piv = Cw[idx]
        if abs(piv) <= tol:
            break
        col = Cw[:, idx[1]].copy()
        row = Cw[idx[0], :].copy() / piv
        Ls.append(col)
        Rs.append(row)
        Cw -= np.outer(col, row)
    r = len(Ls)
    Lm = np.stack(Ls, axis=1) if r else np.zeros((len(u0), 0))
    Rm = np.stack(Rs, axis=0) if r else np.zeros((0, len(u1)))
    # expand unique-side indices back to instantiation indices (first occurrence carries weight)
    T0 = np.zeros((r, n))
    T1 = np.zeros((r, n))
    first0, first1 = {}, {}
    for i in range(n):
        first0.setdefault(s0[i], i)
        first1.setdefault(s1[i], i)
    for s, k in u0.items():
        T0[:, first0[s]] = Lm[k, :]
    for s, k in u1.items():
        T1[:, first1[s]] = Rm[:, k]
    return T0, T1
