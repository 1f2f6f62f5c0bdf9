"""Virtual circuit: fragments, instance labels, merge and knit.

Behavioural mirror of ``third_party/qvm/qvm/virtual_circuit.py``:

* construction (``:21-37``): collect the virtual gates in circuit order,
  replace each by two :class:`VirtualGateEndpoint` s (``:97-113``) and split
  the circuit into one sub-circuit per quantum register (= fragment,
  ``:115-131``); every fragment circuit keeps all classical registers, so
  clbit indices stay global;
* labels (``:39-48,133-148``): per fragment the Cartesian product over ALL
  virtual gates of ``range(n_inst)`` if the gate touches the fragment, else
  ``(-1,)``; the last gate varies fastest;
* knit (``:50-68``): the reference merges fragment distributions label by
  label (XOR of keys, ``:165-171,216-228``) and contracts one virtual gate at a
  time from last to first (``_chunk`` + ``vgate.knit``); here the same linear
  map is one dense contraction over the label axis.

What changes is where the arithmetic runs. :meth:`VirtualCircuit.knit` accepts
the reference's ``dict[fragment, list[QuasiDistr]]`` and runs the contraction
as one dense fp64 MFMA GEMM on the GPU (``engine.knit_dense``); the ``pool``
argument is accepted for signature compatibility and unused. The per-fragment
backend plug (``set_backend`` / ``get_backend``, ``:87-95``) is kept: the
default backend is :class:`~.backend.MI355XBackend`, the batched HIP sweep.
"""
from __future__ import annotations

import itertools
from typing import Any

from .circuit import Barrier, ClassicalRegister, QuantumCircuit
from .quasi_distr import QuasiDistr
from .virtual_gates import VirtualBinaryGate, VirtualGateEndpoint, VirtualMove

InstanceLabelType = tuple[int, ...]


def _is_vgate(op) -> bool:
    return isinstance(op, (VirtualBinaryGate, VirtualMove))


def _is_barrier(op) -> bool:
    return isinstance(op, Barrier) or getattr(op, "name", None) == "barrier"


class VirtualCircuit:
    def __init__(self, circuit: QuantumCircuit) -> None:
        from .ingest import adopt_with_map

        # a foreign (qiskit) cut circuit is rebuilt in this IR; its registers stay valid keys
        circuit, self._frag_alias = adopt_with_map(circuit)
        self._vgate_instrs = [instr for instr in circuit if _is_vgate(instr.operation)]
        self._circuit = self._replace_vgates_with_endpoints(circuit)
        self._frag_circs = {
            qreg: self._circuit_on_fragment(self._circuit, qreg) for qreg in circuit.qregs
        }
        from .backend import MI355XBackend  # local import: backend imports this module

        default = MI355XBackend()
        self._frag_to_backend = {qreg: default for qreg in self._frag_circs}
        # bumped by every mutation of fragments / backends: run_virtual_circuit's plan cache
        # (run.circuit_fingerprint) recomputes the circuit's fingerprint when it changes
        self._generation = 0
        # the content hash of the cut as built (the plan-cache key): part of building the fragments,
        # so a call of run_virtual_circuit on a fresh VirtualCircuit (the reference builds one per
        # call, Utilities.py:74-79) finds its plan without hashing
        from .run import circuit_fingerprint

        circuit_fingerprint(self)

    def _frag(self, fragment):
        """Translate a caller's (possibly foreign) fragment register to the adopted one."""
        return self._frag_alias.get(fragment, fragment)

    # ------------------------------------------------------------------ labels
    def _touches(self, vg_instr, fragment) -> bool:
        return bool(set(vg_instr.qubits) & set(self._frag(fragment)))

    def get_instance_labels(self, fragment) -> list[InstanceLabelType]:
        if not self._vgate_instrs:
            return [()]
        axes = [
            tuple(range(vg.operation.num_instantiations)) if self._touches(vg, fragment) else (-1,)
            for vg in self._vgate_instrs
        ]
        return list(itertools.product(*axes))

    def _global_inst_labels(self) -> list[InstanceLabelType]:
        axes = [range(vg.operation.num_instantiations) for vg in self._vgate_instrs]
        return list(itertools.product(*axes))

    def _global_to_fragment_inst_label(self, fragment, global_inst_label) -> InstanceLabelType:
        return tuple(
            global_inst_label[i] if self._touches(vg, fragment) else -1
            for i, vg in enumerate(self._vgate_instrs)
        )

    def _fragment_results(self, fragment, results: list[QuasiDistr]) -> list[QuasiDistr]:
        by_label = dict(zip(self.get_instance_labels(fragment), results))
        return [
            by_label[self._global_to_fragment_inst_label(fragment, g)]
            for g in self._global_inst_labels()
        ]

    # ------------------------------------------------------------------ knit
    def knit(self, results: dict, pool: Any = None) -> QuasiDistr:
        """Knit per-instance distributions into the uncut circuit's distribution.

        ``results`` maps fragment -> list of ``QuasiDistr`` in
        ``get_instance_labels(fragment)`` order (``run.py:46-58``). The
        contraction runs on the GPU; the returned ``QuasiDistr`` applies the
        reference's ``ACCURACY`` truncation once, to the final result.
        """
        from . import engine

        dense = engine.knit_quasi_distrs(self, {self._frag(f): d for f, d in results.items()})
        return QuasiDistr.from_dense(dense)

    # ------------------------------------------------------------------ fragments / backends
    @property
    def fragment_circuits(self) -> dict:
        return dict(self._frag_circs)

    @property
    def vgate_instructions(self) -> list:
        return list(self._vgate_instrs)

    @property
    def circuit(self) -> QuantumCircuit:
        """The cut circuit with virtual gates replaced by endpoints."""
        return self._circuit

    def replace_fragment_circuit(self, fragment, circuit: QuantumCircuit) -> None:
        self._frag_circs[self._frag(fragment)] = circuit
        self._generation += 1

    def get_backend(self, fragment):
        fragment = self._frag(fragment)
        if fragment not in self._frag_to_backend:
            raise ValueError("Fragment not found.")
        return self._frag_to_backend[fragment]

    def set_backend(self, fragment, backend) -> None:
        fragment = self._frag(fragment)
        if fragment not in self._frag_to_backend:
            raise ValueError("Fragment not found.")
        self._frag_to_backend[fragment] = backend
        self._generation += 1

    def set_backend_for_all(self, backend) -> None:
        self._frag_to_backend = {qreg: backend for qreg in self._frag_circs}
        self._generation += 1

    # ------------------------------------------------------------------ construction helpers
    @staticmethod
    def _replace_vgates_with_endpoints(circuit: QuantumCircuit) -> QuantumCircuit:
        out = QuantumCircuit(*circuit.qregs, *circuit.cregs)
        vgate_index = 0
        for instr in circuit:
            op = instr.operation
            if _is_vgate(op):
                for side in range(2):
                    out.append(VirtualGateEndpoint(op, vgate_idx=vgate_index, qubit_idx=side),
                               [instr.qubits[side]], [])
                vgate_index += 1
            else:
                out.append(op, list(instr.qubits), list(instr.clbits))
        return out

    @staticmethod
    def _circuit_on_fragment(circuit: QuantumCircuit, fragment) -> QuantumCircuit:
        out = QuantumCircuit(fragment, *circuit.cregs)
        members = set(fragment)
        for instr in circuit.data:
            qs = set(instr.qubits)
            if qs <= members:
                out.append(instr.operation, list(instr.qubits), list(instr.clbits))
            elif _is_barrier(instr.operation):
                continue
            elif qs & members:
                raise ValueError(
                    f"Circuit contains gates that act on multiple fragments. {instr.operation}"
                )
        return out


def generate_instantiations(fragment_circuit: QuantumCircuit, inst_labels: list) -> list:
    """Instance circuits of a fragment (``virtual_circuit.py:183-190``)."""
    return [_instantiate_fragment(fragment_circuit, label) for label in inst_labels]


def _chunk(lst: list, n: int) -> list[list]:
    return [lst[i : i + n] for i in range(0, len(lst), n)]


def _instantiate_fragment(fragment_circuit: QuantumCircuit, inst_label: InstanceLabelType) -> QuantumCircuit:
    """Substitute each endpoint by its side of instantiation ``inst_label[vgate_idx]``.

    Adds the ``vgate_c`` register (one config clbit per virtual gate) and
    decomposes one level, as ``virtual_circuit.py:197-213`` does.
    """
    if len(inst_label) == 0:
        return fragment_circuit.copy()
    config = ClassicalRegister(len(inst_label), "vgate_c")
    out = QuantumCircuit(*fragment_circuit.qregs, *fragment_circuit.cregs, config)
    for instr in fragment_circuit:
        op, qubits, clbits = instr.operation, list(instr.qubits), list(instr.clbits)
        if isinstance(op, VirtualGateEndpoint):
            clbits = [config[op.vgate_idx]]
            op = op.instantiate(inst_label[op.vgate_idx])
        out.append(op, qubits, clbits)
    return out.decompose()
