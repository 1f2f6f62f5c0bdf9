"""Fragment compiler: fragment circuit + instance labels -> batched sweep program.

Replaces what the reference does per instance in Python + Aer
(``virtual_circuit.py:183-213`` builds one instance circuit per label and
``run.py:42`` ships them to ``AerSimulator``): here ONE program per fragment is
compiled, and the per-instance differences are reduced to a table of 2x2
"slot" matrices, one per virtual-gate endpoint per job.

Definitions:

* local qubit order: measured data qubits first, ordered by their global
  ``meas`` clbit (so the fragment output index ``x_f`` is the low ``m`` bits of
  the state index and maps to global keys by a bit deposit), then the
  unmeasured qubits (traced out);
* a *slot* is one :class:`VirtualGateEndpoint`; instantiation ``i`` of its side
  is a 1-qubit program ``U_post . [P_m] . U_pre`` with at most one config-bit
  measurement; a measured side yields two *branches* ``m = 0, 1`` with sign
  ``(-1)^m`` (the reference's ``split`` + subtract, ``virtual_gates.py:105-124,
  179-194,262-286``);
* a *job* is one (label, branch combination); its slot matrices fold the fixed
  1-qubit gates adjacent to the endpoint; its output is ``sign * |amp|^2``
  traced over unmeasured qubits; jobs of one label are contiguous and sum to
  the label's signed-folded distribution ``q_f[label]``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import gates as _g
from .circuit import CompositeInstruction
from .virtual_gates import VirtualGateEndpoint, _memoised, planning_memo  # noqa: F401 (planning_memo re-exported)

P0 = np.array([[1, 0], [0, 0]], dtype=np.complex128)
P1 = np.array([[0, 0], [0, 1]], dtype=np.complex128)
I2 = np.eye(2, dtype=np.complex128)


class UnsupportedCircuit(ValueError):
    pass


@dataclass
class HostOp:
    kind: str  # "u1" | "u2" | "slot"
    qubits: tuple
    mat: np.ndarray | None = None
    slot: int = -1


@dataclass
class SlotSpec:
    vgate_idx: int
    side: int
    qubit: int  # local qubit
    endpoint: VirtualGateEndpoint
    pre: np.ndarray = field(default_factory=lambda: I2.copy())
    post: np.ndarray = field(default_factory=lambda: I2.copy())


@dataclass
class FragmentProgram:
    n: int
    m: int
    clbits: list  # global meas clbit for local output bit i, ascending
    ops: list
    slots: list
    qubit_order: list  # fragment Qubit objects in local order

    @property
    def num_slots(self) -> int:
        return len(self.slots)


def _op_matrix(op) -> np.ndarray:
    if hasattr(op, "to_matrix"):
        try:
            return np.asarray(op.to_matrix(), dtype=np.complex128)
        except Exception:  # qiskit ops without a matrix fall back to the table
            pass
    return _g.gate_matrix(op.name, getattr(op, "params", ()))


def _flatten(instructions, qmap_fn):
    """Yield (op, local qubit tuple, clbit tuple) with composites inlined."""
    for instr in instructions:
        op = instr.operation
        if isinstance(op, CompositeInstruction):
            d = op.definition
            inner_q = [qmap_fn(q) for q in instr.qubits]
            sub = [(s.operation, tuple(inner_q[d.find_qubit(q)] for q in s.qubits),
                    tuple(instr.clbits[d.find_clbit(c)] for c in s.clbits)) for s in d]
            for o, qs, cs in sub:
                yield o, qs, cs
        else:
            yield op, tuple(qmap_fn(q) for q in instr.qubits), tuple(instr.clbits)


def compile_fragment(frag_circuit, fragment, clbit_index) -> FragmentProgram:
    """Compile one fragment circuit (endpoints still in place).

    ``clbit_index(clbit) -> int`` maps a classical bit to its global index in
    the ``meas``-first clbit order of the cut circuit.
    """
    frag_qubits = list(fragment)
    n = len(frag_qubits)
    fidx = {q: i for i, q in enumerate(frag_qubits)}

    # -- pass 1: collect raw ops in fragment-qubit indices, find final measurements
    raw = []
    measured_at = {}  # frag qubit -> (position in raw, global clbit)
    for op, qs, cs in _flatten(frag_circuit.data, lambda q: fidx[q]):
        name = getattr(op, "name", "")
        if isinstance(op, (VirtualGateEndpoint, BranchMeasure)):
            raw.append(("slot", qs, op))
        elif name == "measure":
            q = qs[0]
            if q in measured_at:
                raise UnsupportedCircuit("a qubit is measured twice")
            measured_at[q] = (len(raw), clbit_index(cs[0]))
            raw.append(("measure", qs, None))
        elif name in _g.NON_UNITARY_NOOPS or name == "barrier" or getattr(op, "num_qubits", 1) == 0:
            continue
        elif name == "reset":
            raise UnsupportedCircuit("reset is not supported")
        else:
            nq = len(qs)
            if nq not in (1, 2):
                raise UnsupportedCircuit(f"{nq}-qubit gate '{name}' is not supported (decompose first)")
            raw.append(("u1" if nq == 1 else "u2", qs, _op_matrix(op)))
    for q, (pos, _) in measured_at.items():
        for kind, qs, _ in raw[pos + 1 :]:
            if q in qs:
                raise UnsupportedCircuit("operations after a data measurement are not supported")
    clb = [c for _, c in measured_at.values()]
    if len(set(clb)) != len(clb):
        raise UnsupportedCircuit("two qubits measured into one clbit")

    raw = _recover_cz(raw)

    # -- local order: measured (by clbit) then unmeasured (by fragment index)
    meas_sorted = sorted(measured_at.items(), key=lambda kv: kv[1][1])
    order = [q for q, _ in meas_sorted] + [q for q in range(n) if q not in measured_at]
    loc = {q: i for i, q in enumerate(order)}
    m = len(meas_sorted)
    clbits = [c for _, (_, c) in meas_sorted]

    # -- pass 2: fuse 1-qubit runs, build slots
    ops: list[HostOp] = []
    slots: list[SlotSpec] = []
    pending: dict[int, np.ndarray] = {}

    def flush(q):
        mat = pending.pop(q, None)
        if mat is not None and not _g.is_identity_up_to_phase(mat):
            ops.append(HostOp("u1", (q,), mat))

    for kind, qs, payload in raw:
        lq = tuple(loc[q] for q in qs)
        if kind == "measure":
            continue
        if kind == "u1":
            q = lq[0]
            pending[q] = payload @ pending.get(q, I2)
        elif kind == "u2":
            for q in lq:
                flush(q)
            ops.append(HostOp("u2", lq, payload))
        else:  # slot
            q = lq[0]
            flush(q)
            ep = payload
            slots.append(SlotSpec(ep.vgate_idx, ep.qubit_idx, q, ep))
            ops.append(HostOp("slot", lq, None, len(slots) - 1))
    for q in list(pending):
        flush(q)

    # -- pass 3: absorb fixed 1q gates adjacent (per qubit) to a slot into it
    _absorb_into_slots(ops, slots)
    return FragmentProgram(n=n, m=m, clbits=clbits, ops=ops, slots=slots,
                           qubit_order=[frag_qubits[q] for q in order])


_H = _g.gate_matrix("h")
_CZ = _g.gate_matrix("cz")


def _recover_cz(raw: list) -> list:
    """Undo the cutter's ``cz -> h . cx . h`` decomposition (``Cutter.py:84``).

    Pattern on target ``t``: ``h(t)``, ``cx(c, t)``, ``h(t)`` with no other
    operation on ``t`` in between (operations on ``c`` may interleave: they
    commute with ``h(t)``). The diagonal CZ needs no fiber position in the
    sweep kernel and costs one sign flip instead of two dense 2x2 products.
    """
    nxt = {}  # index -> index of the next op on the same qubit (per qubit)
    last = {}
    for i, (kind, qs, _) in enumerate(raw):
        for q in qs:
            if q in last:
                nxt[(last[q], q)] = i
            last[q] = i
    dead = set()
    out = list(raw)
    for j, (kind, qs, mat) in enumerate(raw):
        if kind != "u2" or not np.array_equal(mat, _g.gate_matrix("cx")) or j in dead:
            continue
        c, t = qs
        prev = [i for i in range(j) if (i, t) in nxt and nxt[(i, t)] == j]
        k = nxt.get((j, t))
        if not prev or k is None:
            continue
        i = prev[0]
        if i in dead or k in dead:
            continue
        ki, qi, mi = raw[i]
        kk, qk, mk = raw[k]
        if ki == "u1" and kk == "u1" and np.allclose(mi, _H, atol=1e-15) and np.allclose(mk, _H, atol=1e-15):
            dead.update((i, k))
            out[j] = ("u2", qs, _CZ.copy())
    return [op for i, op in enumerate(out) if i not in dead]


def _absorb_into_slots(ops: list, slots: list) -> None:
    dead = set()
    for i, op in enumerate(ops):
        if op.kind != "slot":
            continue
        q = op.qubits[0]
        s = slots[op.slot]
        # previous op on q
        for j in range(i - 1, -1, -1):
            if j in dead or q not in ops[j].qubits:
                continue
            if ops[j].kind == "u1":
                s.pre = s.pre @ ops[j].mat  # applied before the slot
                dead.add(j)
            break
        for j in range(i + 1, len(ops)):
            if j in dead or q not in ops[j].qubits:
                continue
            if ops[j].kind == "u1":
                s.post = ops[j].mat @ s.post  # applied after the slot
                dead.add(j)
            break
    ops[:] = [op for i, op in enumerate(ops) if i not in dead]


# ---------------------------------------------------------------------------- jobs
class BranchMeasure:
    """Mid-circuit measurement of a plain instance circuit (no sign folding).

    ``vgate_idx`` is the branch index (bit of ``JobTable.branch_bits``),
    ``clbit`` the global clbit the outcome is written to.
    """

    name = "branch_measure"
    num_qubits = 1

    def __init__(self, branch_idx: int, clbit: int):
        self.vgate_idx = branch_idx
        self.qubit_idx = 0
        self.clbit = clbit


def side_program(endpoint, inst_id: int):
    """``endpoint.side_circuit(inst_id)``, memoised inside :func:`planning_memo`."""
    return _memoised("side", endpoint, inst_id, lambda: endpoint.side_circuit(inst_id))


def side_branches(endpoint, inst_id: int) -> list[tuple[np.ndarray, float]]:
    """Branches ``(matrix, sign)`` of one endpoint side for instantiation ``inst_id``."""
    if isinstance(endpoint, BranchMeasure):
        return [(P0.copy(), 1.0), (P1.copy(), 1.0)]
    got = _memoised("branches", endpoint, inst_id, lambda: _side_branches(endpoint, inst_id))
    return [(m.copy(), sg) for m, sg in got]


def _side_branches(endpoint, inst_id: int) -> list[tuple[np.ndarray, float]]:
    side = side_program(endpoint, inst_id)
    pre, post, measured = I2.copy(), I2.copy(), False
    for instr in side.data:
        name = instr.operation.name
        if name == "measure":
            if measured:
                raise UnsupportedCircuit("two config measurements on one side")
            measured = True
            continue
        if name == "barrier":
            continue
        mat = _op_matrix(instr.operation)
        if measured:
            post = mat @ post
        else:
            pre = mat @ pre
    if not measured:
        return [(post @ pre, 1.0)]
    return [(post @ P0 @ pre, 1.0), (post @ P1 @ pre, -1.0)]


def _side_signature(endpoint, inst_id: int) -> tuple:
    if isinstance(endpoint, BranchMeasure):
        return ("branch",)
    side = side_program(endpoint, inst_id)
    return tuple((ins.operation.name, tuple(round(float(p), 15) for p in getattr(ins.operation, "params", ())))
                 for ins in side.data)


def dedup_labels(prog: FragmentProgram, labels: list) -> tuple[list, np.ndarray]:
    """Merge labels whose instance programs coincide on this fragment.

    Two labels give the same fragment instance when every endpoint of the
    fragment gets the same side program (e.g. VirtualCX instantiations 2 and 3
    are both "measure" on the control side, ``virtual_gates.py:163-168``).
    Returns ``(unique_labels, uidx)`` with ``labels[i]`` simulated as
    ``unique_labels[uidx[i]]``. The reference simulates every label
    (``run.py:36-43``); counts of both are reported.
    """
    sig_cache: dict = {}
    seen: dict = {}
    unique, uidx = [], np.zeros(len(labels), dtype=np.int64)
    for i, label in enumerate(labels):
        key = []
        for s in prog.slots:
            inst = 0 if isinstance(s.endpoint, BranchMeasure) else label[s.vgate_idx]
            ck = (id(s), inst)
            if ck not in sig_cache:
                sig_cache[ck] = _side_signature(s.endpoint, inst)
            key.append(sig_cache[ck])
        key = tuple(key)
        if key not in seen:
            seen[key] = len(unique)
            unique.append(label)
        uidx[i] = seen[key]
    return unique, uidx


@dataclass
class BasisReduction:
    """Instances of a fragment expressed in a smaller spanning set of instances.

    Every fragment output is linear in each slot's signed channel, and a cut's side programs
    are linearly dependent as channels (VirtualCX/CZ control side: ``rho + Z rho Z == S rho S^+
    + S^+ rho S``, so the ``z`` program is ``s + sdg - id``). ``q[unique row] = expand @
    q[basis row]`` exactly; the fragment then sweeps ``labels`` only.
    """

    labels: list  # one representative label per basis instance (slot programs in product order)
    expand: np.ndarray  # [n_unique, n_basis] real


# vec(rho) of one qubit, row-major (index 2a + b for |a><b|): |0><0| and the diagonal
_VEC_ZERO = np.diag([1.0, 0.0, 0.0, 0.0])
_VEC_DIAG = np.diag([1.0, 0.0, 0.0, 1.0])


def _superop(mat: np.ndarray) -> np.ndarray:
    """``vec(M rho M^+) = kron(M, conj(M)) vec(rho)`` (row-major vec)."""
    return np.kron(mat, mat.conj())


def _z_commuting(op: HostOp, q: int, prog: FragmentProgram, insts_of: dict) -> bool:
    """Whether ``op`` maps |a><b| on qubit ``q`` into |a><b|-blocks (commutes with Z_q): a gate
    diagonal on q, or a slot whose every branch matrix (with its absorbed gates) is diagonal."""
    if op.kind != "slot":
        from .sweep_plan import _diag_qubits

        return q in _diag_qubits(op)
    s = prog.slots[op.slot]
    for inst in insts_of[op.slot]:
        for mat, _ in side_branches(s.endpoint, inst):
            full = s.post @ mat @ s.pre
            if full[0, 1] != 0 or full[1, 0] != 0:
                return False
    return True


def slot_relevance(prog: FragmentProgram, unique_labels: list) -> list:
    """Per slot, the projectors ``(P_in, P_out)`` on its qubit's vec(rho) with
    ``q_f(..., Phi_s, ...) == q_f(..., P_out Phi_s P_in, ...)`` exactly, for every instantiation
    of every slot (light-cone argument on the compiled op list):

    * input: every op on the qubit before the slot commutes with Z there, so the qubit is still
      |0><0| (``P_in = |0><0|``);
    * output: every op on the qubit after the slot commutes with Z there (diagonal gates, CZ/CX
      controls, diagonal slot branches), so coherences of the qubit never reach the final
      Z-basis outcomes or the partial trace (``P_out`` = the diagonal).

    Otherwise the identity. Both projections keep |a><b| blocks, so they compose across slots
    on one qubit."""
    insts_of = {}
    for k, s in enumerate(prog.slots):
        if isinstance(s.endpoint, BranchMeasure):
            insts_of[k] = [0]
        else:
            insts_of[k] = list(dict.fromkeys(int(lab[s.vgate_idx]) for lab in unique_labels))
    where = {op.slot: i for i, op in enumerate(prog.ops) if op.kind == "slot"}
    out = []
    for k, s in enumerate(prog.slots):
        t, q = where[k], s.qubit
        before = all(_z_commuting(op, q, prog, insts_of) for op in prog.ops[:t] if q in op.qubits)
        after = all(_z_commuting(op, q, prog, insts_of) for op in prog.ops[t + 1:] if q in op.qubits)
        out.append((_VEC_ZERO if before else np.eye(4), _VEC_DIAG if after else np.eye(4)))
    return out


def _slot_channel(s: SlotSpec, inst_id: int, rel) -> np.ndarray:
    """Real 32-vector of the slot's projected channel ``P_out Post Phi_inst Pre P_in``."""
    phi = np.zeros((4, 4), dtype=np.complex128)
    for mat, sign in side_branches(s.endpoint, inst_id):
        phi += sign * _superop(mat)
    phi = rel[1] @ _superop(s.post) @ phi @ _superop(s.pre) @ rel[0]
    return np.concatenate([phi.real.ravel(), phi.imag.ravel()])


def basis_reduce(prog: FragmentProgram, unique_labels: list, tol: float = 1e-12,
                 relevance: bool = True) -> BasisReduction | None:
    """Per slot, keep a maximal linearly independent subset of its side programs (fewest
    branch jobs first) and write every other program as a combination of it. Returns None
    when that does not reduce the fragment's branch-job count.

    ``relevance``: compare the slot channels after the exact light-cone projections of
    :func:`slot_relevance` (programs that differ only in what the fragment's outcomes cannot
    see become equal, and the basis shrinks)."""
    if not prog.slots or not unique_labels:
        return None
    rels = slot_relevance(prog, unique_labels) if relevance else [(np.eye(4), np.eye(4))] * len(prog.slots)
    per_slot = []  # (representative inst ids of the basis, coefficient map inst -> row of D)
    for s, rel in zip(prog.slots, rels):
        if isinstance(s.endpoint, BranchMeasure):
            per_slot.append(([0], {0: np.ones(1)}))
            continue
        insts = list(dict.fromkeys(int(lab[s.vgate_idx]) for lab in unique_labels))
        sig = {i: _side_signature(s.endpoint, i) for i in insts}
        reps = list({sig[i]: i for i in reversed(insts)}.values())[::-1]  # first inst per program
        nbr = {i: len(side_branches(s.endpoint, i)) for i in reps}
        phis = {i: _slot_channel(s, i, rel) for i in reps}
        basis: list[int] = []
        for i in sorted(reps, key=lambda i: (nbr[i], reps.index(i))):
            cand = np.stack([phis[b] for b in basis + [i]], axis=1)
            if np.linalg.matrix_rank(cand, tol=tol) > len(basis):
                basis.append(i)
        if not basis:  # every program projects to the zero channel: q_f == 0 for all labels
            basis = [reps[0]]
        basis.sort(key=reps.index)
        Bm = np.stack([phis[b] for b in basis], axis=1)
        coef = {}
        for i in insts:
            c, *_ = np.linalg.lstsq(Bm, phis[i], rcond=None)
            c[np.abs(c) < tol] = 0.0
            if np.abs(Bm @ c - phis[i]).max() > 1e-10:
                raise AssertionError("side program outside the span of the chosen basis")
            coef[i] = c
        per_slot.append((basis, coef))
    nb_cache: dict = {}
    jobs_now = sum(_label_jobs(prog, lab, nb_cache) for lab in unique_labels)
    n_basis = int(np.prod([len(b) for b, _ in per_slot]))
    base = list(unique_labels[0])
    labels = []
    for combo in np.ndindex(*[len(b) for b, _ in per_slot]):  # last slot fastest
        lab = list(base)
        for s, (basis, _), k in zip(prog.slots, per_slot, combo):
            if not isinstance(s.endpoint, BranchMeasure):
                lab[s.vgate_idx] = basis[k]
        labels.append(tuple(lab))
    if sum(_label_jobs(prog, lab, nb_cache) for lab in labels) >= jobs_now:
        return None
    # expand[u] = kron over slots of the label's coefficient rows, as a row-wise Khatri-Rao product
    # (the same products in the same order as a per-label np.kron loop: bit-identical)
    expand = np.ones((len(unique_labels), 1))
    for s, (_, coef) in zip(prog.slots, per_slot):
        if isinstance(s.endpoint, BranchMeasure):
            C = np.broadcast_to(coef[0], (len(unique_labels), len(coef[0])))
        else:
            C = np.stack([coef[int(lab[s.vgate_idx])] for lab in unique_labels])
        expand = (expand[:, :, None] * C[:, None, :]).reshape(len(unique_labels), -1)
    return BasisReduction(labels, np.ascontiguousarray(expand))


def _label_jobs(prog: FragmentProgram, label, cache: dict) -> int:
    n = 1
    for s in prog.slots:
        inst = 0 if isinstance(s.endpoint, BranchMeasure) else int(label[s.vgate_idx])
        if (id(s), inst) not in cache:
            cache[(id(s), inst)] = len(side_branches(s.endpoint, inst))
        n *= cache[(id(s), inst)]
    return n


@dataclass
class JobTable:
    slot_mats: np.ndarray  # [n_jobs, n_slots, 2, 2] complex128
    sign: np.ndarray  # [n_jobs] float64
    label_offsets: np.ndarray  # [n_labels + 1] int64
    branch_bits: np.ndarray  # [n_jobs] int64: config-bit outcomes (bit j = vgate j)

    @property
    def n_jobs(self) -> int:
        return int(self.sign.shape[0])

    def label_jobs(self) -> np.ndarray:
        """Branch jobs per label."""
        return np.diff(self.label_offsets)

    def take(self, rows) -> "JobTable":
        """The jobs of labels ``rows`` (any order), labels renumbered 0..len(rows)-1."""
        rows = np.asarray(rows, dtype=np.int64)
        offs = self.label_offsets
        idx = (np.concatenate([np.arange(offs[r], offs[r + 1]) for r in rows]) if rows.size
               else np.zeros(0, np.int64))
        new_offs = np.concatenate([[0], np.cumsum(offs[rows + 1] - offs[rows])]).astype(np.int64)
        return JobTable(self.slot_mats[idx], self.sign[idx], new_offs, self.branch_bits[idx])


def build_jobs(prog: FragmentProgram, labels: list) -> JobTable:
    """Expand labels into branch jobs (labels in the given order, jobs contiguous)."""
    ns = prog.num_slots
    cache: dict = {}
    mats, signs, offs, bits = [], [], [0], []
    for label in labels:
        per_slot = []
        for s in prog.slots:
            inst = 0 if isinstance(s.endpoint, BranchMeasure) else label[s.vgate_idx]
            key = (id(s), inst)
            if key not in cache:
                cache[key] = [(s.post @ m @ s.pre, sg) for m, sg in side_branches(s.endpoint, inst)]
            per_slot.append(cache[key])
        # Cartesian product over slots, last slot fastest
        combos = [((), 1.0, 0)]
        for si, br in enumerate(per_slot):
            vg = prog.slots[si].vgate_idx
            combos = [
                (c + (m,), sg * s2, b | ((1 << vg) if (len(br) == 2 and k == 1) else 0))
                for c, sg, b in combos
                for k, (m, s2) in enumerate(br)
            ]
        for c, sg, b in combos:
            mats.append(np.stack(c) if ns else np.zeros((0, 2, 2), np.complex128))
            signs.append(sg)
            bits.append(b)
        offs.append(len(signs))
    slot_mats = np.stack(mats) if mats else np.zeros((0, ns, 2, 2), np.complex128)
    return JobTable(slot_mats.reshape(len(signs), ns, 2, 2), np.asarray(signs, np.float64),
                    np.asarray(offs, np.int64), np.asarray(bits, np.int64))
