"""Uncut reference distribution and cut-vs-uncut fidelity on the GPU.

Mirrors the ideal half of the reference harness
``Utilities.compareOriginalCircWithCutCirc`` (``src/HwAwareCutter/Utilities.py:154-226``):
the uncut circuit's distribution (``getCircResultFromBackend``, ``:39-69``, Aer there) and the
knitted one, compared by Hellinger fidelity (``:222-224``). Here both are exact: the uncut
circuit is swept as ONE 0-cut fragment by the same HIP sweep (up to ~34 qubits fit one
MI355X: 2^34 complex128 = 256 GiB), the fidelity is a HIP reduction. Noisy fake-device runs
(``FakeKolkataV2``) stay out of scope.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import engine
from .cutting import CutSpec, cut_circuit
from .run import RunTimeInfo, run_virtual_circuit_dense
from .virtual_circuit import VirtualCircuit


def uncut_distribution(circ, device: int = 0):
    """Exact distribution of an uncut circuit as a dense device tensor over its clbits."""
    one = cut_circuit(circ, CutSpec([list(range(circ.num_qubits))]))
    out, _ = run_virtual_circuit_dense(VirtualCircuit(one), device=device)
    return out


def hellinger_fidelity_dense(p, q, device: int = 0) -> float:
    return engine.hellinger_fidelity(engine.get_context(device), p, q)


def hellinger_fidelity(dist_p: dict, dist_q: dict) -> float:
    """qiskit ``hellinger_fidelity`` on dicts (normalised, union of keys)."""
    sp = sum(dist_p.values())
    sq = sum(dist_q.values())
    s = 0.0
    for k in set(dist_p) | set(dist_q):
        a, b = max(dist_p.get(k, 0.0), 0.0) / sp, max(dist_q.get(k, 0.0), 0.0) / sq
        s += (a * b) ** 0.5
    return s * s


@dataclass
class Comparison:
    cut_vs_uncut_fidelity: float
    uncut: object  # dense device tensor
    cut: object  # dense device tensor
    cut_info: RunTimeInfo


def compare_original_with_cut(circ, cut_circ, device: int = 0, factored: bool = False) -> Comparison:
    """Ideal cut-vs-uncut comparison (``compareOriginalCircWithCutCirc``'s ``cutVsUncutFidelity``)."""
    cut, info = run_virtual_circuit_dense(VirtualCircuit(cut_circ), device=device, factored=factored)
    uncut = uncut_distribution(circ, device)
    return Comparison(hellinger_fidelity_dense(uncut, cut, device), uncut, cut, info)
