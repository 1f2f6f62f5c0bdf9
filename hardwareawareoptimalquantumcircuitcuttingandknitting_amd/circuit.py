"""Minimal quantum-circuit IR (registers, instructions, circuits).

The reference hands ``qiskit.QuantumCircuit`` objects across its knit API
(``third_party/qvm/qvm/virtual_circuit.py:21-37``). qiskit is not part of this
build, so this module provides the small subset of that data model the hot path
reads: named quantum/classical registers, bits that remember their register,
``CircuitInstruction(operation, qubits, clbits)`` records, gate methods with the
qiskit names and argument order, ``measure_all`` (barrier + ``meas`` register,
as qiskit does) and ``compose`` / ``copy`` / ``to_instruction`` /
``decompose``.

Any object that exposes the same attributes (``qregs``, ``cregs``, iteration
yielding ``.operation/.qubits/.clbits``; operations with ``.name`` and
``.params``) is accepted by :class:`~.virtual_circuit.VirtualCircuit`, so a real
qiskit circuit can be passed in where qiskit is installed.
"""
from __future__ import annotations

import itertools
from typing import Iterable, Iterator, Sequence

import numpy as np

from . import gates as _g

_reg_counter = itertools.count()


class Bit:
    __slots__ = ("_register", "_index")

    def __init__(self, register: "Register", index: int):
        self._register = register
        self._index = index

    @property
    def register(self) -> "Register":
        return self._register

    @property
    def index(self) -> int:
        return self._index

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self._register.name}, {self._index})"

    def __hash__(self) -> int:
        return hash((id(self._register), self._index))

    def __eq__(self, other) -> bool:
        return (
            type(other) is type(self)
            and other._register is self._register
            and other._index == self._index
        )


class Qubit(Bit):
    __slots__ = ()


class Clbit(Bit):
    __slots__ = ()


class Register(Sequence):
    bit_type = Bit
    prefix = "r"

    def __init__(self, size: int, name: str | None = None):
        if size < 0:
            raise ValueError("register size must be >= 0")
        self.name = name if name is not None else f"{self.prefix}{next(_reg_counter)}"
        self.size = int(size)
        self._bits = [self.bit_type(self, i) for i in range(self.size)]

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, i):
        return self._bits[i]

    def __iter__(self) -> Iterator[Bit]:
        return iter(self._bits)

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.size}, '{self.name}')"

    def __hash__(self) -> int:
        return id(self)

    def __eq__(self, other) -> bool:
        return self is other


class QuantumRegister(Register):
    bit_type = Qubit
    prefix = "q"


class ClassicalRegister(Register):
    bit_type = Clbit
    prefix = "c"


class Operation:
    """A named operation. ``matrix`` is available for unitary gates."""

    def __init__(self, name: str, num_qubits: int, num_clbits: int = 0, params=(), label=None):
        self.name = name
        self.num_qubits = num_qubits
        self.num_clbits = num_clbits
        self.params = list(params)
        self.label = label

    def to_matrix(self) -> np.ndarray:
        return _g.gate_matrix(self.name, self.params)

    def __repr__(self) -> str:
        p = f"({', '.join(f'{x:.6g}' for x in self.params)})" if self.params else ""
        return f"{self.name}{p}"


class Gate(Operation):
    def __init__(self, name: str, num_qubits: int, params=(), label=None):
        super().__init__(name, num_qubits, 0, params, label)


class Measure(Operation):
    def __init__(self):
        super().__init__("measure", 1, 1)


class Barrier(Operation):
    def __init__(self, num_qubits: int, label=None):
        super().__init__("barrier", num_qubits, 0, (), label)


class CompositeInstruction(Operation):
    """An operation defined by a sub-circuit (``QuantumCircuit.to_instruction``)."""

    def __init__(self, definition: "QuantumCircuit", name: str = "circuit"):
        super().__init__(name, definition.num_qubits, definition.num_clbits)
        self.definition = definition


class CircuitInstruction:
    __slots__ = ("operation", "qubits", "clbits")

    def __init__(self, operation: Operation, qubits=(), clbits=()):
        self.operation = operation
        self.qubits = tuple(qubits)
        self.clbits = tuple(clbits)

    def __iter__(self):
        # qiskit's legacy (op, qargs, cargs) unpacking
        return iter((self.operation, list(self.qubits), list(self.clbits)))

    def replace(self, operation=None, qubits=None, clbits=None) -> "CircuitInstruction":
        return CircuitInstruction(
            self.operation if operation is None else operation,
            self.qubits if qubits is None else qubits,
            self.clbits if clbits is None else clbits,
        )

    def __repr__(self) -> str:
        return f"CircuitInstruction({self.operation!r}, {list(self.qubits)}, {list(self.clbits)})"


def _std_gate(name: str, nq: int):
    def method(self, *args):
        params, qargs = args[: len(args) - nq], args[len(args) - nq :]
        return self._append_broadcast(Gate(name, nq, params), qargs)

    method.__name__ = name
    return method


class QuantumCircuit:
    def __init__(self, *regs, name: str | None = None):
        self.name = name
        self.qregs: list[QuantumRegister] = []
        self.cregs: list[ClassicalRegister] = []
        self._qubits: list[Qubit] = []
        self._clbits: list[Clbit] = []
        self._qidx: dict[Qubit, int] = {}
        self._cidx: dict[Clbit, int] = {}
        self._data: list[CircuitInstruction] = []
        ints = [r for r in regs if isinstance(r, (int, np.integer))]
        if ints:
            if len(ints) != len(regs) or len(ints) > 2:
                raise ValueError("QuantumCircuit(nq[, nc]) or QuantumCircuit(*registers)")
            self.add_register(QuantumRegister(int(ints[0]), "q"))
            if len(ints) == 2:
                self.add_register(ClassicalRegister(int(ints[1]), "c"))
        else:
            for r in regs:
                self.add_register(r)

    # ------------------------------------------------------------------ registers
    def add_register(self, reg: Register) -> None:
        if isinstance(reg, QuantumRegister):
            if reg in self.qregs:
                raise ValueError(f"register {reg} already in circuit")
            self.qregs.append(reg)
            for b in reg:
                self._qidx[b] = len(self._qubits)
                self._qubits.append(b)
        elif isinstance(reg, ClassicalRegister):
            if reg in self.cregs:
                raise ValueError(f"register {reg} already in circuit")
            self.cregs.append(reg)
            for b in reg:
                self._cidx[b] = len(self._clbits)
                self._clbits.append(b)
        else:
            raise TypeError(f"not a register: {reg!r}")

    @property
    def qubits(self) -> list[Qubit]:
        return list(self._qubits)

    @property
    def clbits(self) -> list[Clbit]:
        return list(self._clbits)

    @property
    def num_qubits(self) -> int:
        return len(self._qubits)

    @property
    def num_clbits(self) -> int:
        return len(self._clbits)

    def find_qubit(self, q: Qubit) -> int:
        return self._qidx[q]

    def find_clbit(self, c: Clbit) -> int:
        return self._cidx[c]

    # ------------------------------------------------------------------ data
    @property
    def data(self) -> list[CircuitInstruction]:
        return self._data

    def __iter__(self) -> Iterator[CircuitInstruction]:
        return iter(self._data)

    def __len__(self) -> int:
        return len(self._data)

    def __getitem__(self, i):
        return self._data[i]

    def _resolve(self, arg, bits: list, cls) -> list:
        if isinstance(arg, cls):
            return [arg]
        if isinstance(arg, (int, np.integer)):
            return [bits[int(arg)]]
        if isinstance(arg, Register):
            return list(arg)
        if isinstance(arg, Iterable):
            out = []
            for a in arg:
                out.extend(self._resolve(a, bits, cls))
            return out
        raise TypeError(f"cannot resolve bit argument {arg!r}")

    def _check_bits(self, qubits, clbits) -> None:
        for q in qubits:
            if q not in self._qidx:
                raise ValueError(f"qubit {q} not in circuit")
        for c in clbits:
            if c not in self._cidx:
                raise ValueError(f"clbit {c} not in circuit")

    def append(self, operation, qargs=None, cargs=None) -> "QuantumCircuit":
        if isinstance(operation, CircuitInstruction):
            instr = operation
            if qargs is not None or cargs is not None:
                instr = instr.replace(
                    qubits=None if qargs is None else self._resolve(qargs, self._qubits, Qubit),
                    clbits=None if cargs is None else self._resolve(cargs, self._clbits, Clbit),
                )
        else:
            qubits = self._resolve(qargs if qargs is not None else [], self._qubits, Qubit)
            clbits = self._resolve(cargs if cargs is not None else [], self._clbits, Clbit)
            instr = CircuitInstruction(operation, qubits, clbits)
        self._check_bits(instr.qubits, instr.clbits)
        self._data.append(instr)
        return self

    def _append_broadcast(self, op: Operation, qargs) -> "QuantumCircuit":
        lists = [self._resolve(a, self._qubits, Qubit) for a in qargs]
        n = max(len(l) for l in lists)
        for l in lists:
            if len(l) not in (1, n):
                raise ValueError("cannot broadcast qubit arguments")
        for i in range(n):
            qs = [l[0] if len(l) == 1 else l[i] for l in lists]
            self.append(Gate(op.name, op.num_qubits, op.params, op.label), qs)
        return self

    # 1-qubit gates (qiskit names, params first then qubit)
    id = _std_gate("id", 1)
    x = _std_gate("x", 1)
    y = _std_gate("y", 1)
    z = _std_gate("z", 1)
    h = _std_gate("h", 1)
    s = _std_gate("s", 1)
    sdg = _std_gate("sdg", 1)
    t = _std_gate("t", 1)
    tdg = _std_gate("tdg", 1)
    sx = _std_gate("sx", 1)
    sxdg = _std_gate("sxdg", 1)
    rx = _std_gate("rx", 1)
    ry = _std_gate("ry", 1)
    rz = _std_gate("rz", 1)
    p = _std_gate("p", 1)
    u1 = _std_gate("u1", 1)
    u2 = _std_gate("u2", 1)
    u3 = _std_gate("u3", 1)
    u = _std_gate("u", 1)
    r = _std_gate("r", 1)
    # 2-qubit gates
    cx = _std_gate("cx", 2)
    cy = _std_gate("cy", 2)
    cz = _std_gate("cz", 2)
    ch = _std_gate("ch", 2)
    cp = _std_gate("cp", 2)
    crz = _std_gate("crz", 2)
    crx = _std_gate("crx", 2)
    cry = _std_gate("cry", 2)
    rzz = _std_gate("rzz", 2)
    swap = _std_gate("swap", 2)

    def measure(self, qubit, clbit) -> "QuantumCircuit":
        qs = self._resolve(qubit, self._qubits, Qubit)
        cs = self._resolve(clbit, self._clbits, Clbit)
        if len(qs) != len(cs):
            raise ValueError("measure: qubit/clbit count mismatch")
        for q, c in zip(qs, cs):
            self.append(Measure(), [q], [c])
        return self

    def barrier(self, *qargs) -> "QuantumCircuit":
        qs = self._resolve(list(qargs), self._qubits, Qubit) if qargs else list(self._qubits)
        return self.append(Barrier(len(qs)), qs)

    def measure_all(self) -> "QuantumCircuit":
        """qiskit semantics: barrier over all qubits, new ``meas`` register."""
        creg = ClassicalRegister(self.num_qubits, "meas")
        self.add_register(creg)
        self.barrier()
        for i, q in enumerate(self._qubits):
            self.append(Measure(), [q], [creg[i]])
        return self

    # ------------------------------------------------------------------ transforms
    def copy(self) -> "QuantumCircuit":
        new = QuantumCircuit(*self.qregs, *self.cregs, name=self.name)
        new._data = list(self._data)
        return new

    def compose(self, other: "QuantumCircuit", inplace: bool = False) -> "QuantumCircuit":
        """Append ``other`` on the same-index bits (equal-width circuits)."""
        if other.num_qubits > self.num_qubits or other.num_clbits > self.num_clbits:
            raise ValueError("compose: other circuit is wider")
        target = self if inplace else self.copy()
        for instr in other:
            qs = [target._qubits[other.find_qubit(q)] for q in instr.qubits]
            cs = [target._clbits[other.find_clbit(c)] for c in instr.clbits]
            target.append(instr.operation, qs, cs)
        return None if inplace else target

    def to_instruction(self) -> CompositeInstruction:
        return CompositeInstruction(self.copy())

    def decompose(self) -> "QuantumCircuit":
        """Inline one level of composite instructions (gate set is already flat)."""
        new = QuantumCircuit(*self.qregs, *self.cregs, name=self.name)
        for instr in self._data:
            op = instr.operation
            if isinstance(op, CompositeInstruction):
                d = op.definition
                for sub in d:
                    qs = [instr.qubits[d.find_qubit(q)] for q in sub.qubits]
                    cs = [instr.clbits[d.find_clbit(c)] for c in sub.clbits]
                    new.append(sub.operation, qs, cs)
            else:
                new.append(instr)
        return new

    def count_ops(self) -> dict[str, int]:
        out: dict[str, int] = {}
        for instr in self._data:
            out[instr.operation.name] = out.get(instr.operation.name, 0) + 1
        return out

    def __repr__(self) -> str:
        return f"QuantumCircuit({self.num_qubits} qubits, {self.num_clbits} clbits, {len(self._data)} ops)"
