"""Exact branching statevector simulation (numpy) — TEST INFRASTRUCTURE ONLY.

Restates the semantics ``AerSimulator`` samples from at ``run.py:42``: a
circuit of 1/2-qubit gates, mid-circuit measurements (which the cut
instantiations use, ``virtual_gates.py:72-100,164-175,246-257``) and final
measurements, started in ``|0..0>``. Instead of sampling ``shots``, the exact
joint distribution over classical keys is returned, keyed like
``QuasiDistr.from_counts`` (``quasi_distr.py:12-20``): bit ``i`` of the key is
classical bit ``i`` in register order.

An op is ``(name, params, qubits, clbits)`` with integer qubit/clbit indices.
"""
import numpy as np

from .gates import matrix


def _apply(psi, n, mat, qubits):
    if len(qubits) == 1:
        ax = n - 1 - qubits[0]
        psi = np.tensordot(mat, psi, axes=([1], [ax]))
        return np.moveaxis(psi, 0, ax)
    q0, q1 = qubits
    u = mat.reshape(2, 2, 2, 2)  # (b1', b0', b1, b0)
    a0, a1 = n - 1 - q0, n - 1 - q1
    psi = np.tensordot(u, psi, axes=([2, 3], [a1, a0]))
    return np.moveaxis(psi, [0, 1], [a1, a0])


def _project(psi, n, q, bit):
    out = psi.copy()
    sl = [slice(None)] * n
    sl[n - 1 - q] = 1 - bit
    out[tuple(sl)] = 0
    return out


def simulate_branches(ops, n_qubits):
    """The branching simulation behind :func:`simulate`: ``(branches, final)`` with ``branches`` a
    list of ``(p, key)`` — ``p`` the probability vector over the state index (``sum b_q 2^q``) of one
    mid-circuit measurement branch, ``key`` that branch's measured bits — and ``final`` the map
    qubit -> clbit of the final measurements. Golden-vector generation restricts these to a few
    outcomes without building the whole dict (tests/golden/make_golden.py)."""
    last_touch = {}
    for i, (name, _, qs, _) in enumerate(ops):
        if name != "barrier":
            for q in qs:
                last_touch[q] = i
    psi = np.zeros((2,) * max(n_qubits, 1), dtype=complex) if n_qubits else np.ones(1, complex)
    if n_qubits:
        psi[(0,) * n_qubits] = 1.0
    branches = [(psi, 0)]  # (state, key bits from mid-circuit measurements)
    final = {}  # qubit -> clbit
    for i, (name, params, qs, cs) in enumerate(ops):
        if name == "barrier":
            continue
        if name == "measure":
            q, c = qs[0], cs[0]
            if last_touch.get(q) == i:  # nothing follows on this qubit: final measurement
                final[q] = c
                continue
            nb = []
            for st, key in branches:
                for bit in (0, 1):
                    pr = _project(st, n_qubits, q, bit)
                    k = (key & ~(1 << c)) | (bit << c)
                    nb.append((pr, k))
            branches = nb
            continue
        mat = matrix(name, params)
        branches = [(_apply(st, n_qubits, mat, qs), key) for st, key in branches]
    # index = sum b_q 2^q (C order, axis 0 = qubit n-1)
    return [(np.abs(st.reshape(-1)) ** 2, key) for st, key in branches], final


def simulate(ops, n_qubits, n_clbits=0):
    """Exact distribution ``{key: p}`` (entries with p == 0 are omitted)."""
    branches, final = simulate_branches(ops, n_qubits)
    out = {}
    for p, key in branches:
        if not n_qubits:
            out[key] = out.get(key, 0.0) + float(p[0])
            continue
        s = np.nonzero(p)[0].astype(np.int64)
        keys = np.full(s.shape, key, dtype=np.int64)
        for q, c in final.items():
            keys = (keys & ~np.int64(1 << c)) | (((s >> q) & 1) << c)
        for k, v in zip(keys.tolist(), p[s].tolist()):
            out[k] = out.get(k, 0.0) + v
    return out


def dense_probabilities(ops, n_qubits, n_clbits):
    """Dense vector over 2^n_clbits (for uncut circuits with final measurements only)."""
    d = simulate(ops, n_qubits, n_clbits)
    v = np.zeros(1 << n_clbits)
    for k, p in d.items():
        v[k] += p
    return v
