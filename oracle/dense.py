"""Dense numpy knit + uncut known answer — TEST INFRASTRUCTURE ONLY.

The dense form of the reference knit: with config outcomes
folded as ``(-1)^m`` per fragment row, ``R[key] = sum_l c_l prod_f q_f[l|f][x_f]``
where ``c_l = prod_j a_j(l_j)`` (``oracle.tables.coefficients``) — the same
linear map ``virtual_circuit.py:50-68`` evaluates with dicts.
"""
import numpy as np

from . import tables
from .qvm import CutView, circuit_ops, instance_distributions
from .statevector import simulate


def fold(distr: dict, n_clbits: int, clbits: list) -> np.ndarray:
    """Signed fold of config bits, data bits compressed onto ``clbits`` (ascending)."""
    pos = {c: i for i, c in enumerate(clbits)}
    out = np.zeros(1 << len(clbits))
    for key, v in distr.items():
        data, cfg = key & ((1 << n_clbits) - 1), key >> n_clbits
        x = 0
        for c in range(n_clbits):
            if data >> c & 1:
                x |= 1 << pos[c]
        out[x] += (-1.0) ** bin(cfg).count("1") * v
    return out


def fragment_clbits(view: CutView, frag) -> list:
    cl = set()
    for op in view.fragment_ops(frag):
        if op[0] == "measure":
            cl.update(op[3])
    return sorted(cl)


def fragment_q(view: CutView, frag):
    d = instance_distributions(view, frag, 0.0)
    if d is None:
        return None, []
    cl = fragment_clbits(view, frag)
    return np.stack([fold(x, view.num_clbits, cl) for x in d]), cl


def dense_knit(view: CutView, qs: dict, clbits: dict) -> np.ndarray:
    """``qs[frag] = [L_f, 2^m_f]``; returns the dense distribution over ``num_clbits`` bits."""
    N = view.num_clbits
    glabels = view.global_labels()
    coefs = [tables.coefficients(k, p) for k, p, _, _ in view.vgates]
    R = np.zeros(1 << N)
    frags = list(qs)
    keys = []
    rows = []
    for f in frags:
        cl = clbits[f]
        k = np.zeros(1 << len(cl), dtype=np.int64)
        for i, c in enumerate(cl):
            k[(np.arange(k.size) >> i) & 1 == 1] += 1 << c
        keys.append(k)
        lab = {l: r for r, l in enumerate(view.labels(list(f)))}
        rows.append([lab[tuple(g[j] if view.touches(j, list(f)) else -1 for j in range(len(g)))]
                     for g in glabels])
    for li, g in enumerate(glabels):
        c = 1.0
        for j, a in enumerate(coefs):
            c *= a[g[j]]
        if not frags:
            R[0] += c
            continue
        vec = c * qs[frags[0]][rows[0][li]]
        key = keys[0]
        for fi in range(1, len(frags)):
            v2 = qs[frags[fi]][rows[fi][li]]
            vec = np.outer(v2, vec).reshape(-1)
            key = (keys[fi][:, None] + key[None, :]).reshape(-1)
        np.add.at(R, key, vec)
    return R


def run_dense(circ):
    """Dense knit of exact instance distributions for a cut circuit."""
    view = CutView(circ)
    qs, cls = {}, {}
    for qreg in view.qregs:
        frag = list(qreg)
        if not frag:
            continue
        q, cl = fragment_q(view, frag)
        if q is None:
            continue
        qs[tuple(frag)] = q
        cls[tuple(frag)] = cl
    return dense_knit(view, qs, cls)


def uncut_distribution(circ) -> np.ndarray:
    """Exact distribution of the uncut circuit (independent dense statevector)."""
    ops = circuit_ops(circ)
    n_cl = sum(len(r) for r in circ.cregs)
    d = simulate(ops, circ.num_qubits, n_cl)
    v = np.zeros(1 << n_cl)
    for k, p in d.items():
        v[k] += p
    return v
