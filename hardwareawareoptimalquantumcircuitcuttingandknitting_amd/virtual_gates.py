"""Cut-gate algebra: instantiation tables and per-gate knit rules.

Behavioural mirror of ``third_party/qvm/qvm/virtual_gates.py``:

* every virtual gate replaces one 2-qubit gate (gate cut) or one wire segment
  (``VirtualMove``, wire cut) by ``num_instantiations`` pairs of local 1-qubit
  programs, one per side, at most one of which measures into the gate's config
  clbit;
* ``knit(results, clbit_idx)`` recombines the ``num_instantiations``
  distributions of one label chunk into one (``QuasiDistr`` arithmetic, exactly
  the reference's linear combination);
* :meth:`VirtualBinaryGate.knit_coefficients` exposes the same linear
  combination as one coefficient per instantiation, with the understanding that
  every config-bit measurement contributes the sign ``(-1)^m`` — the form the
  dense GPU knit consumes (derivation in DESIGN.md §2).

Instantiation tables (reference line numbers): VirtualMove ``62-103``,
VirtualCZ ``154-177``, VirtualCX ``197-206``, VirtualCY ``209-220``,
VirtualRZZ ``230-260``, VirtualCPhase ``299-310``. Knit rules: ``105-124``,
``179-194``, ``262-286``.
"""
from __future__ import annotations

import abc
import threading
from contextlib import contextmanager
from math import cos, pi, sin

from .circuit import Barrier, CompositeInstruction, Gate, QuantumCircuit, QuantumRegister
from .quasi_distr import QuasiDistr

#: degenerate-angle threshold of VirtualRZZ, ``virtual_gates.py:223``
RZZ_ACCURACY = 0.00001


_memo = threading.local()


@contextmanager
def planning_memo():
    """Memoise endpoint side programs for the duration of one plan (per thread). Every query of a
    side (``side_circuit``, its branches, its signature) otherwise rebuilds the virtual gate's
    whole instantiation list (``virtual_gates.py:62-103,154-177``: circuits composed per call), and a
    plan asks hundreds of times (syc 32 5: ~580 instantiation lists). Scoped to the plan: the
    reference's gates alias their original gate's parameter list (``virtual_gates.py:22``), so a
    side may change between plans, never within one. Nested uses share the outer memo."""
    outer = getattr(_memo, "d", None)
    if outer is None:
        _memo.d = {}
    try:
        yield
    finally:
        if outer is None:
            _memo.d = None


def _memoised(kind: str, endpoint, inst_id: int, make):
    d = getattr(_memo, "d", None)
    if d is None:
        return make()
    key = (kind, id(endpoint), inst_id)
    hit = d.get(key)
    if hit is None or hit[0] is not endpoint:  # (the endpoint is held: its id is not reused meanwhile)
        hit = d[key] = (endpoint, make())
    return hit[1]


def _zero_like(r):
    """The empty accumulator of a knit: ``QuasiDistr({})`` for the dict results of the reference
    interface, ``r.zero_like()`` for device results (truncated.DenseQD)."""
    return r.zero_like() if hasattr(r, "zero_like") else QuasiDistr({})


def _inst(side0=(), side1=()) -> QuantumCircuit:
    """Build a 2-qubit / 1-clbit instantiation circuit from per-side op lists.

    An op is ``"name"``, ``("name", param)`` or ``"M"`` (measure into clbit 0).
    Ops are appended side 0 first, then side 1; only the per-qubit order is
    observable (each endpoint keeps the ops of its own qubit).
    """
    qc = QuantumCircuit(2, 1)
    for q, ops in ((0, side0), (1, side1)):
        for op in ops:
            if op == "M":
                qc.measure(q, 0)
            elif isinstance(op, tuple):
                getattr(qc, op[0])(*op[1:], q)
            else:
                getattr(qc, op)(q)
    return qc


def _wrap(inner: QuantumCircuit, before: QuantumCircuit, after: QuantumCircuit) -> QuantumCircuit:
    return before.compose(inner).compose(after)


class WireCut(Barrier):
    """Wire-cut marker placed by the cutter (``virtual_gates.py:9-14``)."""

    def __init__(self, num_qubits: int = 1, label=None):
        super().__init__(num_qubits, label)
        self.name = "wire_cut"


class VirtualBinaryGate(Barrier, abc.ABC):
    """Base class of all cut gates (``virtual_gates.py:17-55``)."""

    def __init__(self, original_gate: Gate, label: str = ""):
        self._original_gate = original_gate
        super().__init__(original_gate.num_qubits, label if label else f"v_{original_gate.name}")
        self.name = f"v_{original_gate.name}"
        # aliases the original gate's parameter list, as the reference does (:22)
        self._params = original_gate.params
        for inst in self._instantiations():
            self._check_instantiation(inst)

    @property
    def original_gate(self) -> Gate:
        return self._original_gate

    @property
    def num_instantiations(self) -> int:
        return len(self._instantiation_list())

    def _instantiation_list(self) -> list:
        """``_instantiations()``, built once per plan inside :func:`planning_memo` (read-only there)."""
        return _memoised("insts", self, 0, self._instantiations)

    @abc.abstractmethod
    def _instantiations(self) -> list[QuantumCircuit]:
        ...

    @abc.abstractmethod
    def knit(self, results: list[QuasiDistr], clbit_idx: int) -> QuasiDistr:
        ...

    @abc.abstractmethod
    def knit_coefficients(self) -> list[float]:
        """Coefficient ``a_i`` per instantiation; config-bit outcomes fold as ``(-1)^m``."""

    def instantiate(self, inst_id: int) -> QuantumCircuit:
        return self._instantiation_list()[inst_id]

    @staticmethod
    def _check_instantiation(inst: QuantumCircuit) -> None:
        assert inst.num_qubits == 2
        assert inst.num_clbits == 1
        for instr in inst.data:
            assert len(instr.qubits) == 1
            assert len(instr.clbits) <= 1

    @staticmethod
    def _signed(r: QuasiDistr, clbit_idx: int) -> QuasiDistr:
        zero, one = r.split(clbit_idx)
        return zero - one


class VirtualMove(VirtualBinaryGate):
    """Wire cut: measure-and-prepare over the Pauli bases (``virtual_gates.py:58-124``)."""

    _SIGNS = (1, 1, 1, -1, 1, -1, 1, -1)

    def __init__(self, original_gate: Gate):
        super().__init__(original_gate, label=f"VirtualMove {original_gate.label}")

    def _instantiations(self) -> list[QuantumCircuit]:
        # side 0 measures the source qubit in the I / X / Y / Z basis,
        # side 1 prepares the matching eigenstates on the fresh move qubit.
        return [
            _inst((), ()),
            _inst((), ("x",)),
            _inst(("h", "M"), ("h",)),
            _inst(("h", "M"), ("x", "h")),
            _inst(("sdg", "h", "M"), ("h", "s")),
            _inst(("sdg", "h", "M"), ("x", "h", "s")),
            _inst(("M",), ()),
            _inst(("M",), ("x",)),
        ]

    def knit(self, results: list[QuasiDistr], clbit_idx: int) -> QuasiDistr:
        acc = _zero_like(results[0])
        for sign, r in zip(self._SIGNS, results):
            term = self._signed(r, clbit_idx)
            acc = acc + term if sign > 0 else acc - term
        return 0.5 * acc

    def knit_coefficients(self) -> list[float]:
        return [0.5 * s for s in self._SIGNS]


class VirtualGateEndpoint(Barrier):
    """One side of a virtual gate inside a fragment (``virtual_gates.py:127-150``)."""

    def __init__(self, virtual_gate: VirtualBinaryGate, vgate_idx: int, qubit_idx: int):
        self._virtual_gate = virtual_gate
        self.vgate_idx = vgate_idx
        self.qubit_idx = qubit_idx
        super().__init__(1, label=f"v_{virtual_gate.name}_{vgate_idx}_{qubit_idx}")
        self.name = "v_endpoint"

    @property
    def virtual_gate(self) -> VirtualBinaryGate:
        return self._virtual_gate

    def side_circuit(self, inst_id: int) -> QuantumCircuit:
        """The 1-qubit / 1-clbit program of this side for instantiation ``inst_id``."""
        assert 0 <= inst_id < self._virtual_gate.num_instantiations
        inst = self._virtual_gate.instantiate(inst_id)
        qreg = QuantumRegister(1)
        side = QuantumCircuit(qreg, *inst.cregs)
        mine = inst.qubits[self.qubit_idx]
        for instr in inst.data:
            if len(instr.qubits) == 1 and instr.qubits[0] == mine:
                side.append(instr.operation, [side.qubits[0]], list(instr.clbits))
        return side

    def instantiate(self, inst_id: int) -> CompositeInstruction:
        return self.side_circuit(inst_id).to_instruction()


class VirtualCZ(VirtualBinaryGate):
    """Gate cut of CZ (``virtual_gates.py:153-194``)."""

    _SIGNS = (1, 1, 1, -1, 1, -1)

    def _instantiations(self) -> list[QuantumCircuit]:
        return [
            _inst(("sdg",), ("sdg",)),
            _inst(("s",), ("s",)),
            _inst(("M",), ()),
            _inst(("M",), ("z",)),
            _inst((), ("M",)),
            _inst(("z",), ("M",)),
        ]

    def knit(self, results: list[QuasiDistr], clbit_idx: int) -> QuasiDistr:
        acc = _zero_like(results[0])
        for sign, r in zip(self._SIGNS, results):
            term = self._signed(r, clbit_idx)
            acc = acc + term if sign > 0 else acc - term
        return 0.5 * acc

    def knit_coefficients(self) -> list[float]:
        return [0.5 * s for s in self._SIGNS]


class VirtualCX(VirtualCZ):
    """CZ instantiations conjugated by H on the target (``virtual_gates.py:197-206``)."""

    def _instantiations(self) -> list[QuantumCircuit]:
        h1 = _inst((), ("h",))
        return [_wrap(i, h1, h1) for i in super()._instantiations()]


class VirtualCY(VirtualCX):
    """CX instantiations conjugated by RZ(-/+pi/2) on the target (``virtual_gates.py:209-220``)."""

    def _instantiations(self) -> list[QuantumCircuit]:
        pre, post = _inst((), (("rz", -pi / 2),)), _inst((), (("rz", pi / 2),))
        return [_wrap(i, pre, post) for i in super()._instantiations()]


class VirtualRZZ(VirtualBinaryGate):
    """Gate cut of RZZ (``virtual_gates.py:226-291``)."""

    def __init__(self, original_gate: Gate, label: str = ""):
        super().__init__(original_gate, label)

    def _cs(self) -> tuple[float, float]:
        m_theta = -self._params[0]
        return cos(m_theta / 2), sin(m_theta / 2)

    def _instantiations(self) -> list[QuantumCircuit]:
        c, s = self._cs()
        if abs(c) < RZZ_ACCURACY:
            return [_inst(("z",), ("z",))]
        if abs(s) < RZZ_ACCURACY:
            return [_inst((), ())]
        return [
            _inst((), ()),
            _inst(("z",), ("z",)),
            _inst((("rz", -pi / 2),), ("M",)),
            _inst(("M",), (("rz", -pi / 2),)),
            _inst((("rz", pi / 2),), ("M",)),
            _inst(("M",), (("rz", pi / 2),)),
        ]

    def knit(self, results: list[QuasiDistr], clbit_idx: int) -> QuasiDistr:
        c, s = self._cs()
        if abs(c) < RZZ_ACCURACY:
            return results[0].split(clbit_idx)[0] * s**2
        if abs(s) < RZZ_ACCURACY:
            return results[0].split(clbit_idx)[0] * c**2
        r0 = results[0].split(clbit_idx)[0]
        r1 = results[1].split(clbit_idx)[0]
        p0, p1 = (results[2] + results[3]).split(clbit_idx)
        n0, n1 = (results[4] + results[5]).split(clbit_idx)
        # same association order as the reference (rounding + truncation per step)
        mixed = ((p0 - p1) - n0) + n1
        return (r0 * c**2) + (r1 * s**2) + mixed * c * s

    def knit_coefficients(self) -> list[float]:
        c, s = self._cs()
        if abs(c) < RZZ_ACCURACY:
            return [s**2]
        if abs(s) < RZZ_ACCURACY:
            return [c**2]
        return [c * c, s * s, c * s, c * s, -c * s, -c * s]

    def knit_one_state(self, results: list[QuasiDistr], state: str) -> float:
        raise NotImplementedError("knit_one_state is not implemented yet for VirtualRZZ")


class VirtualCPhase(VirtualRZZ):
    """CPhase as RZZ plus local RZ (``virtual_gates.py:294-310``).

    Rewrites ``params[0] <- -lambda/2`` in place after the base-class
    self-check, which (through the aliasing at ``:22``) also rewrites the
    original gate's parameter — reproduced deliberately.
    """

    def __init__(self, original_gate: Gate, label: str = ""):
        super().__init__(original_gate, label)
        self._params[0] = -self._params[0] / 2

    def _instantiations(self) -> list[QuantumCircuit]:
        lam = self._params[0]
        pre, post = _inst((("rz", lam / 2),), ()), _inst((), (("rz", lam / 2),))
        return [_wrap(i, pre, post) for i in super()._instantiations()]


VIRTUAL_GATE_TYPES: dict[str, type[VirtualBinaryGate]] = {
    "cx": VirtualCX,
    "cy": VirtualCY,
    "cz": VirtualCZ,
    "rzz": VirtualRZZ,
    "cp": VirtualCPhase,
}
