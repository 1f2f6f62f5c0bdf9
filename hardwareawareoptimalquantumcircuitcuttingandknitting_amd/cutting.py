"""Cut-spec: turn a circuit + chosen cuts into a HwAwareCutter-shaped cut circuit.

The reference's cut circuit (``Cutter.getResultCircs``, ``src/HwAwareCutter/Cutter.py:128-160``)
is the drop-in input of the hot path. Its shape:

* the circuit is the cutter's ``decompose()`` of the input (``Cutter.py:84``), so
  every 2-qubit gate reaching the cut model is a ``cx`` (cz -> h.cx.h on the
  target, cp -> p.cx.p.cx.p, ...);
* a cut 2-qubit gate becomes ``VIRTUAL_GATE_TYPES[name](gate)`` in place
  (``Cutter.py:584-589``);
* a wire cut becomes ``VirtualMove(SwapGate)`` from the cut qubit to a fresh
  qubit of a ``vmove`` register, and every later operation on the cut qubit
  (its final measurement included) is re-targeted to that move qubit
  (``Cutter.py:614-645``);
* qubits are regrouped into one ``frag{i}`` quantum register per partition
  (``dag.py:185-203``), classical registers are unchanged.

The z3 optimiser that CHOOSES the cuts stays out of scope (CPU, ``Cutter.py:383-571``).
:func:`cut_circuit` takes the choice explicitly; :data:`CONFIG_CUTS` records the
choices for the BASELINE configs (derivation: SURVEY.md App. C).
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .circuit import CircuitInstruction, Gate, QuantumCircuit, QuantumRegister
from .generators import factor_int, gen_circ
from .virtual_gates import VIRTUAL_GATE_TYPES, VirtualMove


def _decompose_2q(circ: QuantumCircuit) -> QuantumCircuit:
    """qiskit-0.44 definitions of the 2-qubit gates the benchmarks use (one level)."""
    out = QuantumCircuit(*circ.qregs, *circ.cregs)
    for instr in circ:
        op, qs = instr.operation, list(instr.qubits)
        name = op.name
        if name == "cz":
            out.h(qs[1]); out.cx(qs[0], qs[1]); out.h(qs[1])
        elif name == "cp":
            lam = float(op.params[0])
            out.p(lam / 2, qs[0]); out.cx(qs[0], qs[1]); out.p(-lam / 2, qs[1])
            out.cx(qs[0], qs[1]); out.p(lam / 2, qs[1])
        elif name == "cy":
            out.sdg(qs[1]); out.cx(qs[0], qs[1]); out.s(qs[1])
        elif name == "rzz":
            out.cx(qs[0], qs[1]); out.rz(float(op.params[0]), qs[1]); out.cx(qs[0], qs[1])
        elif name == "swap":
            out.cx(qs[0], qs[1]); out.cx(qs[1], qs[0]); out.cx(qs[0], qs[1])
        else:
            out.append(instr)
    return out


def decompose(circ: QuantumCircuit) -> QuantumCircuit:
    return _decompose_2q(circ)


def two_qubit_gate_indices(circ: QuantumCircuit, a: int, b: int) -> list[int]:
    """Instruction indices of 2-qubit gates between qubits ``a`` and ``b`` (any order)."""
    qa, qb = circ.qubits[a], circ.qubits[b]
    return [i for i, ins in enumerate(circ) if len(ins.qubits) == 2 and set(ins.qubits) == {qa, qb}
            and ins.operation.name != "barrier"]


@dataclass
class CutSpec:
    """Explicit cut choice on a (decomposed) circuit."""

    partitions: list  # list[list[int]]: original qubit indices per fragment
    gate_cuts: list = field(default_factory=list)  # instruction indices (decomposed circuit)
    wire_cuts: list = field(default_factory=list)  # (instr index, qubit, dest fragment): cut before instr


def cut_circuit(circ: QuantumCircuit, spec: CutSpec) -> QuantumCircuit:
    """Build the cut circuit (``frag{i}`` registers, virtual gates, ``vmove`` qubits)."""
    n = circ.num_qubits
    frag_of = {}
    for f, qs in enumerate(spec.partitions):
        for q in qs:
            if q in frag_of:
                raise ValueError(f"qubit {q} in two partitions")
            frag_of[q] = f
    if len(frag_of) != n:
        raise ValueError("partitions must cover every qubit exactly once")
    wire_at: dict = {}
    for idx, q, dest in spec.wire_cuts:
        wire_at.setdefault(idx, []).append((q, dest))
    # fragment members: original qubits (sorted) then move qubits (cut order)
    members = [sorted(qs) for qs in spec.partitions]
    moves = []  # (fragment, move id)
    for k, (_, q, dest) in enumerate(sorted(spec.wire_cuts)):
        moves.append((dest, k))
    regs = []
    slot_of_orig, slot_of_move = {}, {}
    for f, qs in enumerate(members):
        mv = [k for d, k in moves if d == f]
        reg = QuantumRegister(len(qs) + len(mv), f"frag{f}")
        regs.append(reg)
        for i, q in enumerate(qs):
            slot_of_orig[q] = reg[i]
        for j, k in enumerate(mv):
            slot_of_move[k] = reg[len(qs) + j]
    out = QuantumCircuit(*regs, *circ.cregs)
    current = {q: slot_of_orig[q] for q in range(n)}  # original qubit -> its current carrier
    move_counter = 0
    sorted_cuts = sorted(spec.wire_cuts)
    gate_cuts = set(spec.gate_cuts)
    orig_index = {q: i for i, q in enumerate(circ.qubits)}
    for idx, instr in enumerate(circ):
        for q, dest in wire_at.get(idx, []):
            k = sorted_cuts.index(next(c for c in sorted_cuts if c[0] == idx and c[1] == q))
            carrier = slot_of_move[k]
            vm = VirtualMove(Gate("swap", 2, (), label=f"WC {idx}_{q}"))
            out.append(vm, [current[q], carrier])
            current[q] = carrier
            move_counter += 1
        qs = [current[orig_index[q]] for q in instr.qubits]
        op = instr.operation
        if idx in gate_cuts:
            if len(qs) != 2 or op.name not in VIRTUAL_GATE_TYPES:
                raise ValueError(f"instruction {idx} ({op.name}) cannot be gate-cut")
            # label as the cutter names it (Cutter.py:585-589); params copied, not aliased
            vg = VIRTUAL_GATE_TYPES[op.name](Gate(op.name, 2, list(op.params)), f"{op.name} {idx}")
            out.append(vg, qs)
            continue
        out.append(CircuitInstruction(op, qs, instr.clbits))
    return out


# ----------------------------------------------------------------------------- configs
@dataclass
class ConfigCut:
    name: str
    num_qubits: int
    depth: int
    partitions: int
    description: str


def _syc_grid_cuts(circ: QuantumCircuit, rows: int, cols: int, split_col: int) -> tuple[list, list]:
    left = [r * cols + c for r in range(rows) for c in range(cols) if c < split_col]
    right = [r * cols + c for r in range(rows) for c in range(cols) if c >= split_col]
    lset = set(left)
    cuts = []
    for i, ins in enumerate(circ):
        if ins.operation.name == "cx":
            a, b = (circ.find_qubit(q) for q in ins.qubits)
            if (a in lset) != (b in lset):
                cuts.append(i)
    return [left, right], cuts


def config_cut_circuit(name: str, num_qubits: int, depth: int, partitions: int = 2,
                       variant: str = "ref", seed: int | None = None):
    """(uncut decomposed circuit, cut circuit, description) for a BASELINE config.

    ``variant="ref"`` reproduces the cut the reference's z3 model selects
    (SURVEY.md App. C); ``"forced"`` is the forced-cut syc 32 1 variant
    (column split, every crossing CZ cut) used because the reference cut of
    ``syc 32 1`` has no cuts at all.
    """
    from .generators import DEFAULT_SEED

    circ = decompose(gen_circ(name, num_qubits, depth, DEFAULT_SEED if seed is None else seed))
    n = circ.num_qubits
    if name == "bv":
        anc = n - 1
        cx_anc = [i for i, ins in enumerate(circ) if ins.operation.name == "cx"]
        half = (n - 1) // 2
        cut_before = cx_anc[half]  # between cx(q_{half-1}, anc) and cx(q_half, anc)
        left = list(range(half)) + [anc]
        right = list(range(half, n - 1))
        spec = CutSpec([left, right], [], [(cut_before, anc, 1)])
        desc = f"1 wire cut on anc before instruction {cut_before}"
    elif name == "hwe":
        if partitions == 2:
            mid = n // 2
            cut = [i for i in two_qubit_gate_indices(circ, mid - 1, mid)][:1]
            spec = CutSpec([list(range(mid)), list(range(mid, n))], cut)
            desc = f"1 VirtualCX on cx({mid - 1},{mid})"
        else:
            sizes = [n // partitions + (1 if i < n % partitions else 0) for i in range(partitions)]
            bounds = [sum(sizes[:i]) for i in range(partitions + 1)]
            cuts = [two_qubit_gate_indices(circ, b - 1, b)[0] for b in bounds[1:-1]]
            spec = CutSpec([list(range(bounds[i], bounds[i + 1])) for i in range(partitions)], cuts)
            desc = f"{len(cuts)} VirtualCX (chain cut into {partitions})"
    elif name == "syc":
        rows, cols = factor_int(n)
        if depth == 1 and variant == "ref":
            # layer A only: the z3 model needs no cut; pairs are split 7/7, leftovers 2/2
            pairs = [(circ.find_qubit(ins.qubits[0]), circ.find_qubit(ins.qubits[1]))
                     for ins in circ if ins.operation.name == "cx"]
            half = len(pairs) // 2
            f0 = sorted({q for p in pairs[:half] for q in p})
            f1 = sorted({q for p in pairs[half:] for q in p})
            left_over = sorted(set(range(n)) - set(f0) - set(f1))
            f0 += left_over[: len(left_over) // 2]
            f1 += left_over[len(left_over) // 2 :]
            spec = CutSpec([sorted(f0), sorted(f1)], [])
            desc = "0 cuts (14 disjoint CZ pairs split 7/7)"
        else:
            parts, cuts = _syc_grid_cuts(circ, rows, cols, cols // 2)
            spec = CutSpec(parts, cuts)
            desc = f"{len(cuts)} VirtualCX across the column {cols // 2 - 1}|{cols // 2} boundary"
    elif name == "qft":
        parts = [list(range(n))] + [[] for _ in range(partitions - 1)]
        spec = CutSpec(parts, [])
        desc = f"0 cuts (all-to-all; {partitions - 1} empty fragments)"
    else:
        raise ValueError(f"no cut recipe for {name}")
    return circ, cut_circuit(circ, spec), desc


#: BASELINE.json configs -> (name, n, depth, partitions, variant)
BASELINE_CONFIGS = {
    "bv_5_1_p2": ("bv", 5, 1, 2, "ref"),
    "hwe_16_1_p2": ("hwe", 16, 1, 2, "ref"),
    "syc_32_1_p2": ("syc", 32, 1, 2, "ref"),
    "qft_16_1_p3": ("qft", 16, 1, 3, "ref"),
    "syc_32_5_p2": ("syc", 32, 5, 2, "ref"),
    # extra cases (SURVEY.md §8 / BASELINE.md §3)
    "syc_32_1_p2_forced": ("syc", 32, 1, 2, "forced"),
    "hwe_16_1_p3": ("hwe", 16, 1, 3, "ref"),
}
