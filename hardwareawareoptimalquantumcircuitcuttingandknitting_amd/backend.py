"""BackendV2-shaped simulator plug backed by the HIP sweep.

The reference runs every fragment's instance batch through a duck-typed
backend: ``virt.get_backend(frag).run(instantiations, shots=shots)`` then
``job.result().get_counts()`` (``third_party/qvm/qvm/run.py:42,48-56``).
:class:`MI355XBackend` is the default backend of
:class:`~.virtual_circuit.VirtualCircuit`; :func:`~.run.run_virtual_circuit`
recognises it and drives the batched sweep directly (one program per fragment,
no per-instance circuits). Its ``run()`` also accepts arbitrary instance
circuits (e.g. from ``generate_instantiations``) and returns exact
probabilities shaped like counts (``get_counts`` keyed by bit strings, values
``p * shots``; ``get_probabilities`` for the exact values), so third-party
callers of the plug keep working.
"""
from __future__ import annotations

import numpy as np

from .circuit import QuantumCircuit


class MI355XBackend:
    name = "mi355x_statevector"

    def __init__(self, device: int = 0):
        self.device = device

    def run(self, circuits, shots: int | None = None, **kwargs) -> "ExactJob":
        if isinstance(circuits, QuantumCircuit):
            circuits = [circuits]
        return ExactJob([_simulate_instance(c, self.device) for c in circuits], shots)

    def __repr__(self) -> str:
        return f"MI355XBackend(device={self.device})"


class ExactJob:
    def __init__(self, probs: list, shots: int | None):
        self._result = ExactResult(probs, shots)

    def result(self) -> "ExactResult":
        return self._result


class ExactResult:
    def __init__(self, probs: list, shots: int | None):
        self._probs = probs  # list of (dict[int, float], reg widths)
        self._shots = shots

    def get_probabilities(self, experiment: int | None = None):
        out = [p for p, _ in self._probs]
        return out if experiment is None else out[experiment]

    def get_counts(self, experiment: int | None = None):
        shots = self._shots or 1
        res = []
        for probs, widths in self._probs:
            if not widths:
                raise ValueError("No counts for experiment (circuit has no classical registers)")
            counts = {}
            for key, p in probs.items():
                parts, rest = [], key
                for w in widths:
                    parts.append(format(rest & ((1 << w) - 1), "b").zfill(w))
                    rest >>= w
                counts[" ".join(reversed(parts))] = p * shots
            res.append(counts)
        if experiment is not None:
            return res[experiment]
        return res[0] if len(res) == 1 else res


def _simulate_instance(circ: QuantumCircuit, device: int):
    """Exact outcome distribution of one (mid-circuit-measuring) circuit on the GPU.

    Every measurement that is followed by further operations on its qubit, or
    whose clbit is not a final data clbit, becomes a branch slot; branches are
    swept as separate jobs and emitted under their own outcome bits (no sign
    folding).
    """
    from . import engine
    from .instance_program import compile_instance

    prog, jobs, branch_clbits = compile_instance(circ)
    widths = [len(r) for r in circ.cregs]
    if prog.n == 0:
        return {0: 1.0}, widths
    T = engine.torch()
    ctx = engine.get_context(device)
    dprog = engine.DeviceProgram.upload(prog, device)
    slot_t, sign_t, _ = engine.jobs_to_device(jobs, device)
    pjob, _ = engine.sweep_jobs(ctx, dprog, slot_t, sign_t, jobs.n_jobs)
    p = pjob.cpu().numpy()
    probs: dict = {}
    data_keys = _deposit(prog.clbits)
    for j in range(jobs.n_jobs):
        extra = 0
        for bit_idx, clbit in enumerate(branch_clbits):
            if (jobs.branch_bits[j] >> bit_idx) & 1:
                extra |= 1 << clbit
        for x in np.nonzero(p[j])[0]:
            k = int(data_keys[x]) | extra
            probs[k] = probs.get(k, 0.0) + float(p[j, x])
    return probs, widths


def _deposit(clbits):
    from .knit_plan import deposit_keys

    return deposit_keys(clbits)
