"""Fixture of every swept basis row of the syc 32 5 fragments (oracle statevector, build container).

The bench plan sweeps a spanning set of instances per fragment (engine.prepare_fragments(basis=True),
the light-cone basis reduction): 64 + 256 = 320 rows of 2^16 signed-folded outcome probabilities
(q_f). Each row is simulated here by the oracle's branching statevector
(oracle/statevector.py, pinned to the reference by the knit fixtures) and folded over the config bits
(oracle/dense.fold); the fixture keeps, per row, 24 entries at seeded positions, the row sum, its
squared norm and four projections on seeded Rademacher vectors (size-independent checks of all
2^16 entries; tests/test_gpu.py test_syc_32_5_basis_rows_match_oracle recomputes them from the same
seeds). 320 rows x ~1 s on 8 processes: ~1 minute.

Usage: python tests/golden/make_rows.py
"""
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

SEED = 20260417
N_SAMPLES = 24
N_PROJ = 4
OUT = os.path.join(HERE, "basis_rows_syc_32_5_p2.json")


def probes(width: int):
    """(sample positions [N_SAMPLES], Rademacher projections [N_PROJ, width]) from SEED."""
    rng = np.random.default_rng(SEED)
    pos = np.sort(rng.choice(width, N_SAMPLES, replace=False))
    proj = rng.integers(0, 2, size=(N_PROJ, width)).astype(np.float64) * 2.0 - 1.0
    return pos, proj


def row_summary(row: np.ndarray, pos, proj) -> dict:
    return {"samples": [float(x) for x in row[pos]], "sum": float(row.sum()), "sumsq": float(row @ row),
            "proj": [float(x) for x in proj @ row]}


_W = {}


def _init():
    """Each worker builds the cut itself (pickled circuits would carry copies of the registers, and
    the IR's bits compare by register identity)."""
    from oracle import qvm

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    _, cut = cutting.config_cut_circuit("syc", 32, 5, 2)[:2]
    view = qvm.CutView(cut)
    _W["view"], _W["frags"] = view, [list(r) for r in view.qregs if len(r)]


def _row(job):
    from oracle import dense
    from oracle.statevector import simulate

    fi, label, clbits = job
    view, frag = _W["view"], _W["frags"][fi]
    d = simulate(view.instance_ops(frag, label), len(frag))
    return dense.fold(d, view.num_clbits, clbits)


def main():
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine

    _, cut = cutting.config_cut_circuit("syc", 32, 5, 2)[:2]
    virt = VirtualCircuit(cut)
    frags = engine.prepare_fragments(virt, 0, upload=False, basis=True)
    out = {"case": "syc_32_5_p2", "seed": SEED, "n_samples": N_SAMPLES, "n_proj": N_PROJ, "fragments": []}
    with Pool(8, initializer=_init) as pool:
        for fi, fs in enumerate(frags):
            width = 1 << fs.prog.m
            pos, proj = probes(width)
            jobs = [(fi, tuple(lab), list(fs.prog.clbits)) for lab in fs.basis_labels]
            rows = pool.map(_row, jobs)
            out["fragments"].append({
                "qubits": len(fs.fragment), "clbits": list(fs.prog.clbits),
                "basis_labels": [list(lab) for lab in fs.basis_labels],
                "positions": [int(p) for p in pos],
                "rows": [row_summary(r, pos, proj) for r in rows],
            })
            print(f"fragment of {len(fs.fragment)} qubits: {len(rows)} basis rows", flush=True)
        pool.close()
        pool.join()
    with open(OUT, "w") as f:
        json.dump(out, f)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
