"""Compile a plain instance circuit (mid-circuit measurements allowed) for the sweep.

Used by :class:`~.backend.MI355XBackend.run` when the simulator plug is called
with explicit instance circuits (``generate_instantiations`` output, or any
circuit), mirroring what ``AerSimulator`` receives at ``run.py:42``. A
measurement followed by further operations on its qubit becomes a
:class:`~.fragment_program.BranchMeasure` slot (two projector branches, no sign
folding); the others are final measurements.
"""
from __future__ import annotations

from types import SimpleNamespace

from .circuit import CircuitInstruction, CompositeInstruction
from .fragment_program import BranchMeasure, build_jobs, compile_fragment


def _inline(circ):
    out = []
    for instr in circ.data:
        op = instr.operation
        if isinstance(op, CompositeInstruction):
            d = op.definition
            for sub in d:
                qs = [instr.qubits[d.find_qubit(q)] for q in sub.qubits]
                cs = [instr.clbits[d.find_clbit(c)] for c in sub.clbits]
                out.append(CircuitInstruction(sub.operation, qs, cs))
        else:
            out.append(instr)
    return out


def compile_instance(circ):
    clidx = {}
    for creg in circ.cregs:
        for b in creg:
            clidx[b] = len(clidx)
    instrs = _inline(circ)
    rewritten, branch_clbits = [], []
    for i, instr in enumerate(instrs):
        op = instr.operation
        if op.name == "measure":
            q = instr.qubits[0]
            later = any(
                q in nxt.qubits and nxt.operation.name not in ("barrier",) for nxt in instrs[i + 1 :]
            )
            if later:
                bm = BranchMeasure(len(branch_clbits), clidx[instr.clbits[0]])
                branch_clbits.append(clidx[instr.clbits[0]])
                rewritten.append(CircuitInstruction(bm, instr.qubits, ()))
                continue
        rewritten.append(instr)
    prog = compile_fragment(SimpleNamespace(data=rewritten), list(circ.qubits), lambda c: clidx[c])
    jobs = build_jobs(prog, [()])
    return prog, jobs, branch_clbits
