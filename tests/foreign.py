"""A qiskit-shaped circuit model that is NOT this package's IR — TEST INFRASTRUCTURE ONLY.

Used to check cut-spec ingestion (``ingest.adopt``): registers with names, bits as
(register, index) tuples, operations exposing ``name``/``params``/``label`` and, for
virtual gates, the reference's ``v_<gate>`` naming and already-rewritten ``_params``.
"""
from types import SimpleNamespace


class FReg(list):
    def __init__(self, name, size, kind):
        super().__init__([(name, kind, i) for i in range(size)])
        self.name = name

    def __hash__(self):
        return hash((self.name, len(self)))

    def __eq__(self, o):
        return self is o


class FOp:
    def __init__(self, name, params=(), label=None, num_qubits=1, vparams=None):
        self.name, self.params, self.label, self.num_qubits = name, list(params), label, num_qubits
        if vparams is not None:
            self._params = list(vparams)


def to_foreign(circ):
    """Re-express one of this package's circuits in the foreign model."""
    qregs = [FReg(r.name, len(r), "q") for r in circ.qregs]
    cregs = [FReg(r.name, len(r), "c") for r in circ.cregs]
    qmap = {b: qregs[i][j] for i, r in enumerate(circ.qregs) for j, b in enumerate(r)}
    cmap = {b: cregs[i][j] for i, r in enumerate(circ.cregs) for j, b in enumerate(r)}
    data = []
    for ins in circ:
        op = ins.operation
        vp = getattr(op, "_params", None)
        fop = FOp(op.name, [float(p) for p in getattr(op, "params", [])], getattr(op, "label", None),
                  op.num_qubits, vparams=vp if op.name.startswith("v_") else None)
        data.append(SimpleNamespace(operation=fop, qubits=[qmap[q] for q in ins.qubits],
                                    clbits=[cmap[c] for c in ins.clbits]))
    return SimpleNamespace(qregs=qregs, cregs=cregs, data=data)
