"""Generate the golden fixtures in tests/golden/ FROM THE REFERENCE'S OWN CODE.

Runs only in the build container (needs /root/reference; qiskit is absent, so
small recording placeholders for the ``qiskit``/``qiskit.circuit``/
``qiskit.providers``/``qiskit_aer`` names are registered before importing
``third_party/qvm/qvm/{quasi_distr,virtual_gates,virtual_circuit}.py`` and the
``benchmarks/qcg`` generators). Nothing from the reference is copied: the
outputs are data (op lists, dictionaries of floats).

Fixtures:
  instantiations.json — every virtual gate's instantiation table, per side
  quasi_distr.json    — QuasiDistr ops on seeded inputs (ACCURACY 1e-5 and 0)
  knit_<case>.json    — reference VirtualCircuit.knit on exact instance
                        distributions (computed by oracle.statevector), ACCURACY 0 and 1e-5
  generators.json     — reference syc/hwe/bv generator op lists (random.seed(1234))
  knit_samples_<cfg>.json — reference VirtualCircuit.knit of the 2^32-output configs (syc 32 1,
                        syc 32 5) on exact instances restricted to 64 seeded outcomes per fragment:
                        4096 exact entries of the full distribution (make_knit_samples)

Usage: python tests/golden/make_golden.py [--samples [config ...] | --knit case ...]
"""
import json
import math
import os
import random
import sys
import types
from types import SimpleNamespace as NS

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


# ------------------------------------------------------------------ placeholder qiskit
class _Reg(list):
    def __init__(self, size, name=None):
        super().__init__([(name or "r", i) for i in range(size)])
        self.name, self.size = name, size


class QuantumRegister(_Reg):
    pass


class ClassicalRegister(_Reg):
    pass


class Instruction:
    def __init__(self, *a, **k):
        pass


class Gate(Instruction):
    def __init__(self, name, num_qubits, params, label=None):
        self.name, self.num_qubits, self.params, self.label = name, num_qubits, list(params), label


class Barrier(Instruction):
    def __init__(self, num_qubits, label=None):
        self.num_qubits, self.label = num_qubits, label


class QiskitError(Exception):
    pass


class QuantumCircuit:
    """Records (name, params, qubit indices, clbit indices)."""

    def __init__(self, *args):
        self.ops = []
        self.qubits, self.clbits = [], []
        ints = [a for a in args if isinstance(a, int)]
        if ints:
            self.qubits = list(range(ints[0]))
            self.clbits = list(range(ints[1])) if len(ints) > 1 else []
        for a in args:
            if isinstance(a, QuantumRegister):
                self.qubits += list(a)
            elif isinstance(a, ClassicalRegister):
                self.clbits += list(a)

    def add_register(self, r):
        (self.clbits if isinstance(r, ClassicalRegister) else self.qubits).extend(list(r))

    def _q(self, q):
        if isinstance(q, (list, QuantumRegister)):
            return [self._q(x)[0] for x in q]
        return [q if isinstance(q, int) else self.qubits.index(q)]

    def _a(self, name, qs, params=(), cl=None):
        self.ops.append((name, [float(p) for p in params], qs, cl))

    def __getattr__(self, name):
        if name in ("h", "x", "z", "s", "sdg"):
            def f(q):
                for i in self._q(q):
                    self._a(name, [i])
            return f
        if name in ("rx", "ry", "rz"):
            return lambda t, q: [self._a(name, [i], [t]) for i in self._q(q)]
        if name == "u":
            return lambda t, p, l, q: self._a("u", self._q(q), [t, p, l])
        if name in ("cx", "cz"):
            return lambda a, b: self._a(name, self._q(a) + self._q(b))
        if name == "barrier":
            return lambda *a: None
        raise AttributeError(name)

    def measure(self, q, c):
        self._a("measure", self._q(q), (), c)

    @property
    def data(self):
        return [NS(qubits=[o[2][0]], clbits=([o[3]] if o[3] is not None else []), operation=o[0]) for o in self.ops]

    def compose(self, other, inplace=False):
        n = QuantumCircuit()
        n.ops, n.qubits, n.clbits = self.ops + other.ops, self.qubits, self.clbits
        return n


def install_placeholders():
    qc = types.ModuleType("qiskit.circuit")
    for k, v in dict(Barrier=Barrier, Gate=Gate, QuantumCircuit=QuantumCircuit, Instruction=Instruction,
                     QuantumRegister=QuantumRegister, ClassicalRegister=ClassicalRegister).items():
        setattr(qc, k, v)
    q = types.ModuleType("qiskit")
    q.circuit, q.QuantumCircuit, q.QuantumRegister = qc, QuantumCircuit, QuantumRegister
    q.ClassicalRegister, q.QiskitError = ClassicalRegister, QiskitError
    prov = types.ModuleType("qiskit.providers")
    prov.BackendV2 = object
    aer = types.ModuleType("qiskit_aer")
    aer.AerSimulator = object
    sys.modules.update({"qiskit": q, "qiskit.circuit": qc, "qiskit.providers": prov, "qiskit_aer": aer})
    sys.path.insert(0, os.path.join(REF, "third_party", "qvm"))
    sys.path.insert(0, os.path.join(REF, "benchmarks"))


def side_ops(inst, side):
    out = []
    for name, params, qs, cl in inst.ops:
        if qs[0] == side:
            out.append("M" if name == "measure" else [name, params])
    return out


# ------------------------------------------------------------------ fixtures
def make_instantiations(vg):
    cases = {
        "cx": vg.VirtualCX(Gate("cx", 2, [])),
        "cz": vg.VirtualCZ(Gate("cz", 2, [])),
        "cy": vg.VirtualCY(Gate("cy", 2, [])),
        "rzz_0.7": vg.VirtualRZZ(Gate("rzz", 2, [0.7]), "l"),
        "rzz_pi": vg.VirtualRZZ(Gate("rzz", 2, [math.pi]), "l"),
        "rzz_0": vg.VirtualRZZ(Gate("rzz", 2, [0.0]), "l"),
        "cp_0.7": vg.VirtualCPhase(Gate("cp", 2, [0.7]), "l"),
        "move": vg.VirtualMove(Gate("swap", 2, [], label="WC")),
    }
    out = {}
    for k, g in cases.items():
        out[k] = {
            "params_after_init": [float(p) for p in g._params],
            "instantiations": [[side_ops(i, 0), side_ops(i, 1)] for i in g._instantiations()],
        }
    return out


def make_quasi(qd):
    rng = random.Random(2024)
    res = {}
    for acc in (1e-5, 0.0):
        qd.ACCURACY = acc
        tag = f"acc_{acc:g}"
        cases = []
        for t in range(6):
            a = {rng.randrange(64): rng.choice([1, -1]) * rng.random() * 10 ** -rng.randrange(0, 7) for _ in range(12)}
            b = {rng.randrange(64): rng.choice([1, -1]) * rng.random() * 10 ** -rng.randrange(0, 7) for _ in range(12)}
            # disjoint supports for merge (as in real knits): b lives in bits 6..8
            bm = {(k % 8) << 6: v for k, v in b.items()}
            A, B, BM = qd.QuasiDistr(a), qd.QuasiDistr(b), qd.QuasiDistr(bm)
            s0, s1 = A.split(3)
            cases.append({
                "a": list(a.items()), "b": list(b.items()), "bm": list(bm.items()),
                "A": list(A.items()), "split3": [list(s0.items()), list(s1.items())],
                "merge": list(A.merge(BM).items()), "add": list((A + B).items()),
                "sub": list((A - B).items()), "mul": list((A * 0.37).items()),
                "rmul": list((0.37 * A).items()), "npd": list(A.nearest_probability_distribution().items()),
            })
        counts = {"01 101": 10, "00 000": 1, "11 111": 989}
        res[tag] = {"cases": cases, "from_counts": list(qd.QuasiDistr.from_counts(counts).items()),
                    "counts": counts, "to_counts": qd.QuasiDistr.from_counts(counts).to_counts(5, 1000)}
    qd.ACCURACY = 1e-5
    return res


class _SerialPool:
    def map(self, f, it):
        return [f(x) for x in it]

    def starmap(self, f, it):
        return [f(*x) for x in it]


def make_knit(qd, vg, vc, cut, name):
    """Reference knit on exact instance distributions of ``cut`` (oracle statevector)."""
    from oracle.qvm import CutView, instance_distributions

    view = CutView(cut)
    frags = [tuple(r) for r in view.qregs if len(r)]
    inputs = {}
    for fi, f in enumerate(frags):
        d = instance_distributions(view, list(f), 0.0)
        if d is not None:
            inputs[fi] = [sorted(x.items()) for x in d]
    # reference virtual-gate objects (fresh, from the original, un-rewritten parameters)
    ref_vgates = []
    for instr in cut:
        op = instr.operation
        kind = {"v_cx": "cx", "v_cz": "cz", "v_cy": "cy", "v_rzz": "rzz", "v_cp": "cp", "v_swap": "move"}.get(op.name)
        if kind is None:
            continue
        orig = [float(p) for p in op.original_gate.params] if hasattr(op, "original_gate") else []
        if kind == "cp":  # the product gate already rewrote its (aliased) params to -lambda/2
            orig = [-2.0 * float(op._params[0])]
        if kind == "move":
            g = vg.VirtualMove(Gate("swap", 2, [], label="WC"))
        elif kind in ("rzz", "cp"):
            g = vg.VIRTUAL_GATE_TYPES[kind](Gate(kind, 2, list(orig)), "l")
        else:
            g = vg.VIRTUAL_GATE_TYPES[kind](Gate(kind, 2, []))
        fa = next(i for i, f in enumerate(frags) if instr.qubits[0] in f)
        fb = next(i for i, f in enumerate(frags) if instr.qubits[1] in f)
        ref_vgates.append(NS(operation=g, qubits=[("F", fa), ("F", fb)]))
    out = {"case": name, "num_clbits": view.num_clbits, "inputs": {str(k): v for k, v in inputs.items()}}
    for acc in (0.0, 1e-5):
        qd.ACCURACY = acc
        v = object.__new__(vc.VirtualCircuit)
        v._vgate_instrs = ref_vgates
        v._circuit = NS(num_clbits=view.num_clbits)
        results = {tuple([("F", fi)]): [qd.QuasiDistr(dict(x)) for x in inputs[fi]] for fi in inputs}
        res = v.knit(results, _SerialPool())
        out[f"knit_acc_{acc:g}"] = sorted(res.items())
        out[f"npd_acc_{acc:g}"] = sorted(res.nearest_probability_distribution().items())
    qd.ACCURACY = 1e-5
    return out


_SAMPLE_JOB = {}


def _restricted_instance(job):
    """One instance of a fragment, exact (oracle branching statevector), restricted to the sampled
    data outcomes: ``{data key | config key: p}`` over the fragment's sampled outcomes only."""
    import numpy as np

    from oracle.statevector import simulate_branches

    fi, label = job
    view, frag, cl, sample_keys = (_SAMPLE_JOB[k][fi] if k != "view" else _SAMPLE_JOB[k]
                                   for k in ("view", "frags", "clbits", "keys"))
    n = len(frag)
    branches, final = simulate_branches(view.instance_ops(list(frag), label), n)
    s = np.arange(1 << n, dtype=np.int64)
    data = np.zeros_like(s)
    for q, c in final.items():
        if c < view.num_clbits:
            data |= ((s >> q) & 1) << c
    hit = np.isin(data, sample_keys)
    out = {}
    for p, key in branches:
        for k, v in zip(data[hit].tolist(), p[hit].tolist()):
            if v != 0.0:
                out[k | key] = out.get(k | key, 0.0) + v
    return sorted(out.items())


def make_knit_samples(qd, vc, config: str, n_samples: int = 64, seed: int = 2026, processes: int = 8):
    """Reference ``VirtualCircuit.knit`` (ACCURACY = 0) of a 2^32-output BASELINE config on exact
    instance distributions restricted to ``n_samples`` seeded data outcomes per fragment.

    The knit is entrywise (``qd:55-60``: merges are outer products with disjoint key supports; the
    per-gate knits, ``vg:105-124,179-194``, combine entries of equal data key), so every output key
    whose fragment parts are all sampled receives exactly its unrestricted value: n_samples^2 exact
    entries of the full 2^32 distribution, from the reference's own knit."""
    from multiprocessing import Pool

    import numpy as np
    from oracle import dense
    from oracle.qvm import CutView

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    name, n, d, p, var = cutting.BASELINE_CONFIGS[config]
    _, cut, desc = cutting.config_cut_circuit(name, n, d, p, var)
    view = CutView(cut)
    frags = [tuple(r) for r in view.qregs if len(r)]
    rng = np.random.default_rng(seed)
    clbits, keys, xs = [], [], []
    from oracle.statevector import simulate_branches

    for f in frags:
        cl = dense.fragment_clbits(view, list(f))
        # 3/4 of the samples from the support of the first label's outcome marginal (shallow circuits
        # such as syc 32 1 put zero probability on most outcomes), the rest uniform
        branches, final = simulate_branches(view.instance_ops(list(f), view.labels(list(f))[0]), len(f))
        s_idx = np.arange(1 << len(f), dtype=np.int64)
        xi = np.zeros_like(s_idx)
        for q, c in final.items():
            if c in cl:
                xi |= ((s_idx >> q) & 1) << cl.index(c)
        marg = np.zeros(1 << len(cl))
        for pb, _ in branches:
            np.add.at(marg, xi, pb)
        support = np.nonzero(marg > 0)[0]
        n_sup = min(len(support), 3 * n_samples // 4)
        x = set(rng.choice(support, n_sup, replace=False).tolist())
        while len(x) < n_samples:
            x.add(int(rng.integers(1 << len(cl))))
        x = np.array(sorted(x), dtype=np.int64)
        k = np.zeros_like(x)
        for i, c in enumerate(cl):
            k |= ((x >> i) & 1) << c
        clbits.append(cl)
        xs.append(x)
        keys.append(k)
    _SAMPLE_JOB.update(view=view, frags=frags, clbits=clbits, keys=keys)
    jobs = [(fi, label) for fi, f in enumerate(frags) for label in view.labels(list(f))]
    pool = Pool(processes)
    try:
        rows = pool.map(_restricted_instance, jobs, chunksize=8)
    finally:
        pool.close()
        pool.join()
    inputs = {fi: [] for fi in range(len(frags))}
    for (fi, _), r in zip(jobs, rows):
        inputs[fi].append(r)
    ref_vgates = []
    for instr in cut:
        op = instr.operation
        if not op.name.startswith("v_"):
            continue
        if op.name != "v_cx":
            raise ValueError(f"{config}: unexpected virtual gate {op.name}")
        fa = next(i for i, f in enumerate(frags) if instr.qubits[0] in f)
        fb = next(i for i, f in enumerate(frags) if instr.qubits[1] in f)
        ref_vgates.append(NS(operation=_REF_VG.VirtualCX(Gate("cx", 2, [])), qubits=[("F", fa), ("F", fb)]))
    qd.ACCURACY = 0.0
    v = object.__new__(vc.VirtualCircuit)
    v._vgate_instrs = ref_vgates
    v._circuit = NS(num_clbits=view.num_clbits)
    results = {tuple([("F", fi)]): [qd.QuasiDistr(dict(x)) for x in inputs[fi]] for fi in inputs}
    res = v.knit(results, _SerialPool())
    qd.ACCURACY = 1e-5
    N = view.num_clbits
    out_keys = (keys[0][:, None] | keys[1][None, :]).reshape(-1) if len(keys) == 2 else keys[0]
    vals = [float(res.get(int(k), 0.0)) for k in out_keys]
    allowed = set(out_keys.tolist())
    extra = [k for k in res if k >> N or int(k) not in allowed]
    if extra:
        raise AssertionError(f"{config}: reference knit produced {len(extra)} keys outside the sampled set")
    return {"case": config, "cut": desc, "num_clbits": N, "seed": seed, "n_samples": n_samples,
            "fragment_clbits": clbits, "samples": [x.tolist() for x in xs],
            "keys": [int(k) for k in out_keys], "values": vals,
            "instances": len(jobs), "accuracy": 0.0}


_REF_VG = None


def make_generators():
    import importlib

    qg = importlib.import_module("qcg.Supremacy.Qgrid_Sycamore")
    hw = importlib.import_module("qcg.QAOA.hw_efficient_ansatz")
    bvm = importlib.import_module("qcg.BernsteinVazirani.bernstein_vazirani")
    out = {}
    for n, d, (r, c) in ((32, 1, (4, 8)), (32, 5, (4, 8)), (12, 2, (4, 3))):
        random.seed(1234)
        g = qg.Qgrid(r, c, d, order=None, singlegates=True, barriers=False, measure=False, regname="q")
        circ = g.gen_circuit()
        out[f"syc_{n}_{d}"] = circ.ops
    h = hw.HWEA(16, 1, parameters="optimal", barriers=False, measure=False, regname="q")
    out["hwe_16_1"] = h.gen_circuit().ops
    b = bvm.BV(secret="1111", barriers=False, measure=False, regname="q")
    out["bv_5"] = b.gen_circuit().ops
    return out


def main_samples():
    """knit_samples_<config>.json only (2^32-output configs; minutes of CPU on 8 processes)."""
    global _REF_VG
    install_placeholders()
    import qvm.quasi_distr as qd
    import qvm.virtual_circuit as vc
    import qvm.virtual_gates as vg

    _REF_VG = vg
    for config in sys.argv[2:] or ("syc_32_1_p2", "syc_32_5_p2"):
        obj = make_knit_samples(qd, vc, config)
        with open(os.path.join(HERE, f"knit_samples_{config}.json"), "w") as f:
            json.dump(obj, f, separators=(",", ":"))
        print("wrote", config, "instances", obj["instances"], "nonzero", sum(v != 0 for v in obj["values"]))


def main():
    install_placeholders()
    import contextlib
    import io

    import qvm.quasi_distr as qd
    import qvm.virtual_circuit as vc
    import qvm.virtual_gates as vg

    import circuits
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    def dump(name, obj):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, separators=(",", ":"))

    dump("instantiations.json", make_instantiations(vg))
    dump("quasi_distr.json", make_quasi(qd))
    cases = {
        "cx": circuits.two_fragment("cx"), "cz": circuits.two_fragment("cz"),
        "cy": circuits.two_fragment("cy"), "rzz": circuits.two_fragment("rzz"),
        "rzz_pi": circuits.two_fragment("rzz", angle=math.pi), "rzz_0": circuits.two_fragment("rzz", angle=0.0),
        "cp": circuits.two_fragment("cp"), "cx_3cuts": circuits.two_fragment("cx", 3, 3, n_cuts=3),
        "move": circuits.wire_cut(), "move_gate": circuits.wire_cut(3, 2, extra_gate_cut=True),
        "three": circuits.three_fragment(), "partial": circuits.partial_measure(),
        "same_fragment": circuits.same_fragment_cut(),
    }
    only = sys.argv[2:] if len(sys.argv) > 2 and sys.argv[1] == "--knit" else None
    if only:  # regenerate just these knit fixtures
        for k in only:
            dump(f"knit_{k}.json", make_knit(qd, vg, vc, cases[k][1], k))
        print("wrote", only)
        return
    for key in ("bv_5_1_p2", "hwe_16_1_p2", "hwe_16_1_p3"):
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        circ, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
        cases[key] = (circ, cut)
    for k, (_, cut) in cases.items():
        dump(f"knit_{k}.json", make_knit(qd, vg, vc, cut, k))
    with contextlib.redirect_stdout(io.StringIO()):
        gens = make_generators()
    dump("generators.json", gens)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--samples":
        main_samples()
    else:
        main()
