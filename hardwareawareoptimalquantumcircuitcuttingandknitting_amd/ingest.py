"""Cut-spec ingestion: adopt a foreign (e.g. qiskit) cut circuit into this package's IR.

The reference's cut circuit is a ``qiskit.QuantumCircuit`` produced by
``Cutter.getResultCircs()`` (``src/HwAwareCutter/Cutter.py:128-160``): ``frag{i}``
quantum registers (plus ``vmove`` qubits moved into them, ``Cutter.py:614-645``), the
original classical registers, standard gates after one ``decompose()`` and the reference's
own ``qvm.virtual_gates`` objects for the cuts. :func:`adopt` rebuilds such a circuit from
its duck-typed surface only — ``qregs`` / ``cregs`` (named, sized, iterable), instructions
with ``operation`` (``name``, ``params``, optional ``to_matrix()``), ``qubits``, ``clbits`` —
so no qiskit import is needed:

* registers keep their names and sizes, bits are mapped positionally;
* a virtual gate is recognised by its ``v_<gate>`` name and rebuilt as this package's class;
  ``VirtualCPhase`` has already rewritten its parameter to ``-lambda/2``
  (``virtual_gates.py:297``), so ``lambda = -2 * params[0]`` is recovered;
* standard gates keep name and parameters; anything else with ``to_matrix()`` becomes a
  :class:`MatrixGate`; ``measure`` / ``barrier`` map directly.
"""
from __future__ import annotations

import numpy as np

from . import gates as _g
from .circuit import (
    Barrier,
    ClassicalRegister,
    Gate,
    Measure,
    QuantumCircuit,
    QuantumRegister,
)
from .virtual_gates import VIRTUAL_GATE_TYPES, VirtualBinaryGate, VirtualMove


class MatrixGate(Gate):
    """A gate given by an explicit unitary (foreign gates outside the named table)."""

    def __init__(self, name: str, matrix: np.ndarray, label=None):
        m = np.asarray(matrix, dtype=np.complex128)
        nq = int(round(np.log2(m.shape[0])))
        super().__init__(name, nq, (), label)
        self._matrix = m

    def to_matrix(self) -> np.ndarray:
        return self._matrix


def _params(op) -> list:
    ps = getattr(op, "_params", None)
    if ps is None:
        ps = getattr(op, "params", [])
    return [float(p) for p in ps]


def _adopt_vgate(op):
    name = op.name
    kind = name[2:]
    label = getattr(op, "label", None) or ""
    if kind == "swap":
        return VirtualMove(Gate("swap", 2, (), label=label))
    if kind not in VIRTUAL_GATE_TYPES:
        raise ValueError(f"unknown virtual gate {name}")
    ps = _params(op)
    if kind == "cp":
        ps = [-2.0 * ps[0]]  # undo the in-place rewrite params[0] <- -lambda/2
    return VIRTUAL_GATE_TYPES[kind](Gate(kind, 2, ps), label)


def _adopt_op(op):
    name = getattr(op, "name", None)
    if isinstance(op, (VirtualBinaryGate, VirtualMove)):
        return op
    if name is None:
        raise ValueError(f"operation without a name: {op!r}")
    if name.startswith("v_") and name != "v_endpoint":
        return _adopt_vgate(op)
    if name == "measure":
        return Measure()
    if name == "barrier":
        return Barrier(getattr(op, "num_qubits", 1))
    if name in _g.ONE_QUBIT or name in _g.TWO_QUBIT:
        return Gate(name, _g.num_gate_qubits(name), _params(op), getattr(op, "label", None))
    if hasattr(op, "to_matrix"):
        return MatrixGate(name, op.to_matrix(), getattr(op, "label", None))
    raise ValueError(f"cannot adopt operation '{name}'")


def adopt(circuit) -> QuantumCircuit:
    """Return ``circuit`` as this package's :class:`QuantumCircuit` (identity if it already is)."""
    return adopt_with_map(circuit)[0]


def adopt_with_map(circuit) -> tuple[QuantumCircuit, dict]:
    """Like :func:`adopt`, also returning ``{foreign quantum register: adopted register}``."""
    if isinstance(circuit, QuantumCircuit):
        return circuit, {}
    qmap, cmap, reg_map = {}, {}, {}
    regs = []
    for r in circuit.qregs:
        mine = QuantumRegister(len(r), getattr(r, "name", None))
        regs.append(mine)
        reg_map[r] = mine
        for i, b in enumerate(r):
            qmap[b] = mine[i]
    for r in circuit.cregs:
        mine = ClassicalRegister(len(r), getattr(r, "name", None))
        regs.append(mine)
        for i, b in enumerate(r):
            cmap[b] = mine[i]
    out = QuantumCircuit(*regs)
    data = circuit.data if hasattr(circuit, "data") else list(circuit)
    for instr in data:
        op = _adopt_op(instr.operation)
        out.append(op, [qmap[q] for q in instr.qubits], [cmap[c] for c in instr.clbits])
    return out, reg_map
