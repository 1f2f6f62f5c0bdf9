"""Oracle and host API pinned against golden vectors produced by the reference's own code.

Fixtures: tests/golden/*.json (generator: tests/golden/make_golden.py, which imports
third_party/qvm and benchmarks/qcg from the reference with placeholder qiskit modules).
"""
import glob
import json
import math
import os

import numpy as np
import pytest

from oracle import dense, qvm, tables
from oracle.quasi import QD
from oracle.statevector import simulate

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import generators, virtual_gates as pvg
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.circuit import Gate
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr import QuasiDistr
import hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr as pqd

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _norm_ops(ops):
    out = []
    for o in ops:
        if o == "M":
            out.append("M")
        else:
            out.append((o[0], tuple(round(float(x), 12) for x in o[1])))
    return out


TABLE_KEYS = {"cx": ("cx", []), "cz": ("cz", []), "cy": ("cy", []), "rzz_0.7": ("rzz", [0.7]),
              "rzz_pi": ("rzz", [math.pi]), "rzz_0": ("rzz", [0.0]), "cp_0.7": ("cp", [0.7]),
              "move": ("move", [])}


@pytest.mark.parametrize("key", sorted(TABLE_KEYS))
def test_oracle_tables_match_reference(key):
    gold = load("instantiations.json")[key]
    kind, params = TABLE_KEYS[key]
    tparams = gold["params_after_init"] if kind in ("rzz", "cp") else params
    mine = tables.table(kind, tparams)
    assert len(mine) == len(gold["instantiations"])
    for (s0, s1), (g0, g1) in zip(mine, gold["instantiations"]):
        assert _norm_ops([o if o == "M" else [o[0], list(o[1])] for o in s0]) == _norm_ops(g0)
        assert _norm_ops([o if o == "M" else [o[0], list(o[1])] for o in s1]) == _norm_ops(g1)


def _product_gate(kind, params):
    if kind == "move":
        return pvg.VirtualMove(Gate("swap", 2, [], label="WC"))
    cls = pvg.VIRTUAL_GATE_TYPES[kind]
    return cls(Gate(kind, 2, list(params)), "l")


@pytest.mark.parametrize("key", sorted(TABLE_KEYS))
def test_product_tables_match_reference(key):
    gold = load("instantiations.json")[key]
    kind, params = TABLE_KEYS[key]
    g = _product_gate(kind, params)
    assert [float(p) for p in g._params] == pytest.approx(gold["params_after_init"])
    assert g.num_instantiations == len(gold["instantiations"])
    for i, (g0, g1) in enumerate(gold["instantiations"]):
        for side, gs in ((0, g0), (1, g1)):
            ep = pvg.VirtualGateEndpoint(g, 0, side)
            ops = []
            for ins in ep.side_circuit(i).data:
                ops.append("M" if ins.operation.name == "measure" else [ins.operation.name, ins.operation.params])
            assert _norm_ops(ops) == _norm_ops(gs)


def _items(x):
    return [(int(k), float(v)) for k, v in x]


@pytest.mark.parametrize("acc", ["acc_1e-05", "acc_0"])
def test_quasi_distr_oracle_and_product_match_reference(acc):
    gold = load("quasi_distr.json")[acc]
    a_val = 1e-5 if acc == "acc_1e-05" else 0.0
    old = pqd.ACCURACY
    pqd.ACCURACY = a_val
    try:
        for c in gold["cases"]:
            a, b, bm = dict(_items(c["a"])), dict(_items(c["b"])), dict(_items(c["bm"]))
            for mk in (lambda d: QD(d, a_val), QuasiDistr):
                A, B, BM = mk(a), mk(b), mk(bm)
                assert sorted(A.items()) == sorted(_items(c["A"]))
                s0, s1 = A.split(3)
                assert sorted(s0.items()) == sorted(_items(c["split3"][0]))
                assert sorted(s1.items()) == sorted(_items(c["split3"][1]))
                if isinstance(A, QD):
                    merged, add, sub, mul, npd = A.merge(BM), A.add(B), A.sub(B), A.scale(0.37), A.npd()
                else:
                    merged, add, sub, mul, npd = A.merge(BM), A + B, A - B, A * 0.37, A.nearest_probability_distribution()
                    assert sorted((0.37 * A).items()) == sorted(_items(c["rmul"]))
                assert sorted(merged.items()) == sorted(_items(c["merge"]))
                assert sorted(add.items()) == sorted(_items(c["add"]))
                assert sorted(sub.items()) == sorted(_items(c["sub"]))
                assert sorted(mul.items()) == sorted(_items(c["mul"]))
                assert sorted(npd.items()) == sorted(_items(c["npd"]))
        fc = gold["from_counts"]
        assert sorted(QD.from_counts(gold["counts"], a_val).items()) == sorted(_items(fc))
        assert sorted(QuasiDistr.from_counts(gold["counts"]).items()) == sorted(_items(fc))
        assert QuasiDistr.from_counts(gold["counts"]).to_counts(5, 1000) == gold["to_counts"]
    finally:
        pqd.ACCURACY = old


KNIT_FILES = sorted(f for f in glob.glob(os.path.join(GOLD, "knit_*.json")) if "knit_samples_" not in f)


def _case_circuits(case):
    import circuits
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    builders = {
        "cx": lambda: circuits.two_fragment("cx"), "cz": lambda: circuits.two_fragment("cz"),
        "cy": lambda: circuits.two_fragment("cy"), "rzz": lambda: circuits.two_fragment("rzz"),
        "rzz_pi": lambda: circuits.two_fragment("rzz", angle=math.pi),
        "rzz_0": lambda: circuits.two_fragment("rzz", angle=0.0),
        "cp": lambda: circuits.two_fragment("cp"), "cx_3cuts": lambda: circuits.two_fragment("cx", 3, 3, n_cuts=3),
        "move": lambda: circuits.wire_cut(), "move_gate": lambda: circuits.wire_cut(3, 2, extra_gate_cut=True),
        "three": lambda: circuits.three_fragment(), "partial": lambda: circuits.partial_measure(),
        "same_fragment": lambda: circuits.same_fragment_cut(),
    }
    if case in builders:
        return builders[case]()
    name, n, d, p, var = cutting.BASELINE_CONFIGS[case]
    circ, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    return circ, cut


@pytest.mark.parametrize("path", KNIT_FILES, ids=[os.path.basename(p)[5:-5] for p in KNIT_FILES])
def test_oracle_knit_matches_reference_knit(path):
    gold = json.load(open(path))
    circ, cut = _case_circuits(gold["case"])
    view = qvm.CutView(cut)
    frags = [list(r) for r in view.qregs if len(r)]
    for acc_tag, acc in (("0", 0.0), ("1e-05", 1e-5)):
        # the instance distributions the reference was fed are the oracle's own (exact)
        results = {}
        for fi, f in enumerate(frags):
            if str(fi) in gold["inputs"]:
                results[tuple(f)] = [QD(dict(_items(x)), acc) for x in gold["inputs"][str(fi)]]
        out = qvm.knit(view, results, acc)
        ref = dict(_items(gold[f"knit_acc_{acc_tag}"]))
        assert set(out) == set(ref)
        for k in ref:
            assert out[k] == pytest.approx(ref[k], abs=1e-15, rel=1e-12)
        assert sorted(out.npd()) == sorted(dict(_items(gold[f"npd_acc_{acc_tag}"])))
    # the inputs themselves are reproduced by the oracle statevector
    for fi, f in enumerate(frags):
        d = qvm.instance_distributions(view, f, 0.0)
        if d is None:
            assert str(fi) not in gold["inputs"]
            continue
        for mine, ref in zip(d, gold["inputs"][str(fi)]):
            ref = dict(_items(ref))
            assert set(mine) == set(ref)
            for k in ref:
                assert mine[k] == pytest.approx(ref[k], abs=1e-15)


@pytest.mark.parametrize("path", KNIT_FILES, ids=[os.path.basename(p)[5:-5] for p in KNIT_FILES])
def test_known_answer_reference_knit_equals_uncut(path):
    """knit(exact instances) == exact uncut distribution — pins the simulation semantics."""
    gold = json.load(open(path))
    circ, cut = _case_circuits(gold["case"])
    unc = dense.uncut_distribution(circ)
    ref = np.zeros_like(unc)
    for k, v in _items(gold["knit_acc_0"]):
        ref[k] = v
    dn = dense.run_dense(cut)
    assert np.abs(dn - ref).max() <= 1e-13  # dense form == literal reference knit
    err = np.abs(ref - unc).max()
    if gold["case"] == "cp":
        # reference VirtualCPhase rewrites params[0] <- -lambda/2 (virtual_gates.py:297) and then
        # wraps rz(params[0]/2) (:300-304): the knit is NOT the uncut distribution. Mirrored as is.
        assert err > 1e-3
    else:
        assert err <= 1e-12


def test_generators_match_reference():
    gold = load("generators.json")

    def ops_of(c):
        out = []
        for ins in c:
            name = ins.operation.name
            if name in ("barrier", "measure"):
                continue
            out.append((name, [round(float(p), 12) for p in ins.operation.params], [c.find_qubit(q) for q in ins.qubits]))
        return out

    def gold_ops(lst):
        return [(n, [round(float(p), 12) for p in ps], qs) for n, ps, qs, _ in lst]

    assert ops_of(generators.sycamore(32, 1)) == gold_ops(gold["syc_32_1"])
    assert ops_of(generators.sycamore(32, 5)) == gold_ops(gold["syc_32_5"])
    assert ops_of(generators.sycamore(12, 2)) == gold_ops(gold["syc_12_2"])
    assert ops_of(generators.hwea(16, 1)) == gold_ops(gold["hwe_16_1"])
    assert ops_of(generators.bernstein_vazirani(5)) == gold_ops(gold["bv_5"])


class _HostDenseQD:
    """numpy model of truncated.DenseQD (the reference-truncation GPU path): the same operations,
    one rounding each (a +- b, s * a), truncation |v| <= acc -> 0 after every one."""

    def __init__(self, t, nbits, acc):
        self.t, self.nbits, self.acc = t, nbits, acc

    def _tr(self, v):
        return _HostDenseQD(np.where(np.abs(v) > self.acc, v, 0.0), self.nbits, self.acc)

    def zero_like(self):
        return _HostDenseQD(None, None, self.acc)

    def split(self, bit):
        assert bit == self.nbits - 1
        h = self.t.size // 2
        return _HostDenseQD(self.t[:h], self.nbits - 1, self.acc), _HostDenseQD(self.t[h:], self.nbits - 1, self.acc)

    def __add__(self, o):
        return o if self.t is None else self._tr(self.t + o.t)

    def __sub__(self, o):
        return o._tr(-o.t) if self.t is None else self._tr(self.t - o.t)

    def __mul__(self, s):
        return self._tr(self.t * float(s))

    __rmul__ = __mul__


@pytest.mark.parametrize("path", KNIT_FILES, ids=[os.path.basename(p)[5:-5] for p in KNIT_FILES])
def test_dense_truncated_knit_model_matches_reference_knit(path):
    """The algorithm of run_virtual_circuit(truncation="reference") (truncated.knit_label_tree: dense
    vectors over N + V key bits, leaf merges, the package's per-gate knit rules on dense operands,
    depth-first over the label tree) on the reference's own inputs at ACCURACY 1e-5 reproduces the
    reference VirtualCircuit.knit (golden knit_acc_1e-05) key for key within 1e-15."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.truncated import knit_label_tree

    acc = 1e-5
    gold = json.load(open(path))
    _, cut = _case_circuits(gold["case"])
    view = qvm.CutView(cut)
    virt = VirtualCircuit(cut)
    vgates = [i.operation for i in virt.vgate_instructions]
    N, V = view.num_clbits, len(vgates)
    frags = [list(r) for r in view.qregs if len(r)]
    inputs = {fi: [{k: v for k, v in _items(x) if abs(v) > acc} for x in gold["inputs"][str(fi)]]
              for fi in range(len(frags)) if str(fi) in gold["inputs"]}
    touches = {fi: [bool(set(vg.qubits) & set(frags[fi])) for vg in virt.vgate_instructions] for fi in inputs}
    index = {fi: {lab: r for r, lab in enumerate(view.labels(frags[fi]))} for fi in inputs}

    def leaf(label):
        merged = None
        for fi in sorted(inputs):
            flab = tuple(label[j] if touches[fi][j] else -1 for j in range(V))
            d = inputs[fi][index[fi][flab]]
            if merged is None:
                merged = d
            else:
                merged = {k1 ^ k2: v1 * v2 for k1, v1 in merged.items() for k2, v2 in d.items()}
                merged = {k: v for k, v in merged.items() if abs(v) > acc}
        t = np.zeros(1 << (N + V))
        for k, v in merged.items():
            t[k] = v
        return _HostDenseQD(t, N + V, acc)

    out = knit_label_tree(vgates, N, leaf).t
    ref = dict(_items(gold["knit_acc_1e-05"]))
    got = {int(k): float(out[k]) for k in np.flatnonzero(out)}
    assert set(got) == set(ref)
    for k in ref:
        assert got[k] == pytest.approx(ref[k], abs=1e-15, rel=1e-12)
