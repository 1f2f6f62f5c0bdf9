"""Shot sampling restated — TEST INFRASTRUCTURE ONLY.

The reference samples every instance circuit ``shots`` times on its backend
(``run.py:42`` ``backend.run(instantiations, shots=shots)``), reads the counts
(``run.py:54-56``) and turns them into frequencies with ``QuasiDistr.from_counts``
(``quasi_distr.py:12-20``: ``count / shots``, entries not above ``ACCURACY``
dropped). Aer's random stream is not reproducible outside Aer, so the product
(``csrc/qknit_sample.hip``) draws from the exact instance distributions with a
counter-based SplitMix64 stream; this module restates that stream and the
inverse-CDF draw in numpy, so the GPU's counts can be compared draw for draw.

Outcome order of an instance (the CDF order): config-bit branches first (the
instance's measured virtual gates ascending, the last one fastest, outcome 0
first), then the fragment's data outcome ``x`` (clbits compressed as in
:func:`oracle.dense.fold`). Label ``l`` of fragment ``f`` (``view.labels``
order) uses stream ``(fragment_seed(seed, f), l)``.
"""
import numpy as np

from .dense import fragment_clbits
from .statevector import simulate

MASK = (1 << 64) - 1
_GOLDEN = 0x9E3779B97F4A7C15
_DRAW = 0xD1B54A32D192ED03
_FRAG = 0x632BE59BD9B4E019


def fragment_seed(seed: int, index: int) -> int:
    """Stream seed of the index-th non-empty fragment (qregs order)."""
    return (int(seed) + index * _FRAG) & MASK


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(seed: int, label: int, shots: int) -> np.ndarray:
    """``u(seed, label, s)`` for ``s < shots``: uniform doubles in [0, 1) (53-bit)."""
    s = np.arange(1, shots + 1, dtype=np.uint64)
    base = (int(seed) + _GOLDEN * (label + 1)) & MASK
    with np.errstate(over="ignore"):
        z = np.uint64(base) + np.uint64(_DRAW) * s
    return (splitmix64(z) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def instance_outcomes(view, frag, label):
    """Exact distribution of one instance in CDF order: ``(p [rows * W], row_signs [rows])``."""
    ops = view.instance_ops(frag, label)
    N = view.num_clbits
    measured = sorted({cs[0] - N for (name, _, _, cs) in ops if name == "measure" and cs and cs[0] >= N})
    cl = fragment_clbits(view, frag)
    pos = {c: i for i, c in enumerate(cl)}
    W = 1 << len(cl)
    rows = 1 << len(measured)
    p = np.zeros(rows * W)
    for key, v in simulate(ops, len(frag)).items():
        data, cfg = key & ((1 << N) - 1), key >> N
        r = 0
        for j in measured:
            r = 2 * r + ((cfg >> j) & 1)
        x = 0
        for c in range(N):
            if data >> c & 1:
                x |= 1 << pos[c]
        p[r * W + x] += v
    signs = np.array([(-1.0) ** bin(r).count("1") for r in range(rows)])
    return p, signs


def sample_counts(p: np.ndarray, seed: int, label: int, shots: int) -> np.ndarray:
    """Counts per outcome of ``shots`` inverse-CDF draws (first index with cdf > u * total)."""
    cdf = np.cumsum(np.abs(p))
    target = uniforms(seed, label, shots) * cdf[-1]
    idx = np.minimum(np.searchsorted(cdf, target, side="right"), p.size - 1)
    return np.bincount(idx, minlength=p.size).astype(np.int64)


def fold_counts(counts: np.ndarray, signs: np.ndarray, shots: int, accuracy: float) -> np.ndarray:
    """``from_counts`` (frequency, ``|v| > ACCURACY``) then the signed config-bit fold."""
    f = counts.reshape(len(signs), -1) / shots
    f = np.where(f > accuracy, f, 0.0)
    return (signs[:, None] * f).sum(axis=0)


def sampled_fragment(view, frag, index: int, shots: int, seed: int, accuracy: float):
    """Per label ``(counts [rows * W], q [W])`` of one fragment, label order."""
    fseed = fragment_seed(seed, index)
    out = []
    for li, label in enumerate(view.labels(frag)):
        p, signs = instance_outcomes(view, frag, label)
        c = sample_counts(p, fseed, li, shots)
        out.append((c, fold_counts(c, signs, shots, accuracy)))
    return out
