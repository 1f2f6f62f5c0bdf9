"""Literal restatement of the qvm knitting pipeline — TEST INFRASTRUCTURE ONLY.

Given a cut circuit (any object with ``qregs``, ``cregs`` and instructions
exposing ``operation`` (``name``, ``params``), ``qubits``, ``clbits``), this
module reproduces ``run_virtual_circuit`` (``run.py:23-71``) with exact
instance distributions in place of Aer's sampled counts:

* endpoints + fragments: ``virtual_circuit.py:21-37,97-131``
* labels: ``virtual_circuit.py:39-48,133-148``
* instance programs: ``virtual_circuit.py:183-213`` + ``virtual_gates.py:134-150``
* drop of fragments whose counts cannot be read: ``run.py:49-58``
* merge + per-gate knit: ``virtual_circuit.py:50-68,150-171,193-194,216-228``
* final projection: ``quasi_distr.py:28-43`` via ``run.py:71``
"""
import itertools

from . import tables
from .quasi import QD
from .statevector import simulate

_VKIND = {"v_cx": "cx", "v_cz": "cz", "v_cy": "cy", "v_rzz": "rzz", "v_cp": "cp", "v_swap": "move"}


class CutView:
    """Index view of a cut circuit."""

    def __init__(self, circ):
        self.circ = circ
        self.qregs = list(circ.qregs)
        self.clbit_index = {}
        for creg in circ.cregs:
            for b in creg:
                self.clbit_index[b] = len(self.clbit_index)
        self.num_clbits = len(self.clbit_index)
        self.vgates = []  # (kind, params, qubit0, qubit1)
        self.ops = []  # ("vend", j, side, qubit) | (name, params, qubits, clbits)
        for instr in circ:
            op = instr.operation
            kind = _VKIND.get(op.name)
            if kind is not None:
                j = len(self.vgates)
                params = [float(x) for x in getattr(op, "_params", getattr(op, "params", []))]
                self.vgates.append((kind, params, instr.qubits[0], instr.qubits[1]))
                self.ops.append(("vend", j, 0, instr.qubits[0]))
                self.ops.append(("vend", j, 1, instr.qubits[1]))
            else:
                self.ops.append((op.name, [float(x) for x in op.params], tuple(instr.qubits),
                                 tuple(self.clbit_index[c] for c in instr.clbits)))

    def n_inst(self, j):
        kind, params, _, _ = self.vgates[j]
        return len(tables.table(kind, params))

    def touches(self, j, frag):
        _, _, a, b = self.vgates[j]
        return a in frag or b in frag

    def fragment_ops(self, frag):
        fs = set(frag)
        out = []
        for op in self.ops:
            if op[0] == "vend":
                if op[3] in fs:
                    out.append(op)
                continue
            qs = set(op[2])
            if qs <= fs:
                out.append(op)
            elif op[0] == "barrier":
                continue
            elif qs & fs:
                raise ValueError("Circuit contains gates that act on multiple fragments.")
        return out

    def labels(self, frag):
        if not self.vgates:
            return [()]
        axes = [range(self.n_inst(j)) if self.touches(j, frag) else (-1,) for j in range(len(self.vgates))]
        return list(itertools.product(*axes))

    def global_labels(self):
        return list(itertools.product(*[range(self.n_inst(j)) for j in range(len(self.vgates))]))

    def instance_ops(self, frag, label):
        local = {q: i for i, q in enumerate(frag)}
        out = []
        for op in self.fragment_ops(frag):
            if op[0] == "vend":
                _, j, side, q = op
                kind, params, _, _ = self.vgates[j]
                for g in tables.table(kind, params)[label[j]][side]:
                    if g == "M":
                        out.append(("measure", (), (local[q],), (self.num_clbits + j,)))
                    else:
                        out.append((g[0], g[1], (local[q],), ()))
            else:
                name, params, qs, cs = op
                out.append((name, params, tuple(local[q] for q in qs), cs))
        return out


def instance_distributions(view: CutView, frag, accuracy=0.0):
    """Exact per-instance distributions (``QD``) of one fragment, in label order.

    Returns ``None`` when some instance measures nothing (the reference's
    ``get_counts`` raises and the fragment is skipped, ``run.py:49-58``).
    """
    res = []
    for label in view.labels(frag):
        ops = view.instance_ops(frag, label)
        if not any(o[0] == "measure" for o in ops):
            return None
        res.append(QD(simulate(ops, len(frag)), accuracy))
    return res


def _merge_row(row):
    """``_merge_distrs`` (``virtual_circuit.py:216-221``): fold ``QuasiDistr.merge`` over a row."""
    acc = row[0]
    for d in row[1:]:
        acc = acc.merge(d)
    return acc


def knit(view: CutView, results: dict, accuracy=0.0, pool=None):
    """``VirtualCircuit.knit`` (``virtual_circuit.py:50-68``) on ``{frag: [QD]}``.

    ``pool`` (a ``multiprocessing.Pool``) runs the merge and every per-gate knit through
    ``pool.map`` / ``pool.starmap`` exactly as the reference does with its ``Pool(8)``
    (``run.py:64-67``, ``virtual_circuit.py:63-66,224-228``); None runs them in-process."""
    glabels = view.global_labels()
    lists = []
    for frag, distrs in results.items():
        by_label = dict(zip(view.labels(frag), distrs))
        lists.append([by_label[tuple(g[j] if view.touches(j, frag) else -1 for j in range(len(g)))]
                      for g in glabels])
    merged = pool.map(_merge_row, list(zip(*lists))) if pool is not None else [_merge_row(r) for r in zip(*lists)]
    if not view.vgates:
        return merged[0]
    clbit = view.num_clbits + len(view.vgates) - 1
    for j in reversed(range(len(view.vgates))):
        kind, params, _, _ = view.vgates[j]
        n = view.n_inst(j)
        chunks = [merged[i:i + n] for i in range(0, len(merged), n)]
        if pool is not None:
            merged = pool.starmap(tables.knit, [(kind, params, c, clbit) for c in chunks])
        else:
            merged = [tables.knit(kind, params, c, clbit) for c in chunks]
        clbit -= 1
    return merged[0]


def run(circ, accuracy=0.0, pool=None, times=None):
    """Exact-instance ``run_virtual_circuit``: returns (knit QD before projection, NPD dict).

    ``times`` (a dict) receives ``run_time`` / ``knit_time`` split as ``run.py:35,60,65-67``."""
    import time

    t0 = time.perf_counter()
    view = CutView(circ)
    results = {}
    for qreg in view.qregs:
        frag = list(qreg)
        if not frag:
            continue
        d = instance_distributions(view, frag, accuracy)
        if d is not None:
            results[tuple(frag)] = d
    t1 = time.perf_counter()
    out = knit(view, results, accuracy, pool)
    if times is not None:
        times["run_time"], times["knit_time"] = t1 - t0, time.perf_counter() - t1
    return out, out.npd()


def circuit_ops(circ):
    """Flatten an uncut circuit into oracle ops over global qubit/clbit indices."""
    qidx = {q: i for i, q in enumerate(circ.qubits)}
    cidx = {}
    for creg in circ.cregs:
        for b in creg:
            cidx[b] = len(cidx)
    return [(ins.operation.name, [float(x) for x in ins.operation.params],
             tuple(qidx[q] for q in ins.qubits), tuple(cidx[c] for c in ins.clbits)) for ins in circ]
