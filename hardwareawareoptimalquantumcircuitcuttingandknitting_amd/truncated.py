"""The reference's knit with its per-operation truncation, on the GPU (``truncation="reference"``).

The reference keeps every intermediate result as a ``QuasiDistr`` dict and drops the entries with
``|v| <= ACCURACY`` each time one is built (``quasi_distr.py:7-10``): after ``from_counts``
(``:12-20``), after every fragment merge (``:55-60``, ``virtual_circuit.py:216-228``) and after
every ``+``, ``-`` and scalar ``*`` of a per-gate knit (``virtual_gates.py:105-124,179-194,262-286``),
gate by gate from the last (``virtual_circuit.py:50-68``). The default path of
:func:`run.run_virtual_circuit` contracts exactly and truncates once at the end (a result within
``ACCURACY`` per operation of this one); this module replays the reference's sequence instead:

* instance distributions: every unique instance swept per branch job (``qk_sweep``, signs 1: the
  joint distribution over outcome and config bits the reference's instance circuit measures),
  truncated into ``[label, config, outcome]`` (``qk_qd_from_rows``);
* per global label (``itertools.product`` order, last gate fastest) the fragments merged in
  ``fragment_circuits`` order into a dense vector over ``N + V`` key bits (``qk_qd_merge``; the
  fragments' config bits are disjoint: one side of an instantiation measures at most);
* the label tree knitted depth-first (each chunk's knit depends on that chunk only, so the order of
  chunks does not matter), with the package's own ``VirtualBinaryGate.knit`` running on
  :class:`DenseQD` — the same operations in the same association order, each one rounding and one
  truncation (``qk_qd_axpby``). Splitting at ``clbit_idx = N + j`` takes the top key bit: the
  halves of the vector.

Bounded to ``N + V <= 26`` key bits (a dense vector per live tree node).
"""
from __future__ import annotations

import numpy as np

from . import engine
from . import quasi_distr as _qd
from .fragment_program import BranchMeasure
from .knit_plan import deposit_keys

MAX_KEY_BITS = 26
MAX_MERGE_ITEMS = 1 << 34  # products one merge of a dense vector with a fragment row may form (per label)


class DenseQD:
    """A quasi-distribution over ``2^nbits`` keys as a device vector; every operation truncates at
    ``acc`` like ``QuasiDistr.__init__`` (``quasi_distr.py:7-10``). Implements the operations the
    per-gate knits use: ``split`` at the top key bit, ``+``, ``-``, scalar ``*``."""

    __slots__ = ("t", "nbits", "acc", "ctx")

    def __init__(self, ctx, t, nbits: int, acc: float):
        self.ctx, self.t, self.nbits, self.acc = ctx, t, nbits, acc

    def zero_like(self) -> "DenseQD":
        """The empty ``QuasiDistr({})`` a knit starts its sum from: no vector; ``empty + x`` is ``x``
        and ``empty - x`` is ``-x`` exactly, as the reference's dict operations give."""
        return DenseQD(self.ctx, None, None, self.acc)

    def split(self, bit_index: int):
        if bit_index != self.nbits - 1:
            raise ValueError(f"split at bit {bit_index} of a {self.nbits}-bit key: only the top config bit")
        h = self.t.numel() // 2
        return (DenseQD(self.ctx, self.t[:h], self.nbits - 1, self.acc),
                DenseQD(self.ctx, self.t[h:], self.nbits - 1, self.acc))

    def _axpby(self, alpha: float, other: "DenseQD | None", beta: float) -> "DenseQD":
        b = self if other is None else other
        if b.nbits != self.nbits:
            raise ValueError("key widths differ")
        out = engine.torch().empty_like(self.t)
        ctx = self.ctx
        ctx.check(ctx.lib.qk_qd_axpby(ctx.handle, self.t.numel(), float(alpha), self.t.data_ptr(), float(beta),
                                      b.t.data_ptr(), self.acc, out.data_ptr()), "qk_qd_axpby")
        return DenseQD(ctx, out, self.nbits, self.acc)

    def __add__(self, other: "DenseQD") -> "DenseQD":
        if self.t is None:
            return other
        return self._axpby(1.0, other, 1.0)

    def __sub__(self, other: "DenseQD") -> "DenseQD":
        if self.t is None:
            return other._axpby(-1.0, None, 0.0)
        return self._axpby(1.0, other, -1.0)

    def __mul__(self, other) -> "DenseQD":
        if not isinstance(other, (int, float)):
            raise TypeError(f"Cannot multiply DenseQD by {type(other)}")
        return self._axpby(float(other), None, 0.0)

    def __rmul__(self, other) -> "DenseQD":
        return self.__mul__(other)


def _pext_np(x: np.ndarray, mask: int) -> np.ndarray:
    out = np.zeros_like(x)
    j = 0
    for i in range(64):
        if mask >> i & 1:
            out |= ((x >> i) & 1) << j
            j += 1
    return out


def knit_reference_truncated(virt, device: int = 0, accuracy: float | None = None):
    """The reference's ``virt.knit(results)`` (``virtual_circuit.py:50-68``) on exact instance
    distributions with ``QuasiDistr`` truncation at ``accuracy`` (default ``quasi_distr.ACCURACY``)
    after every operation; returns the dense ``[2^N]`` result on the device (entries the reference's
    dict would not hold are 0)."""
    T = engine.torch()
    acc = _qd.ACCURACY if accuracy is None else float(accuracy)
    ctx = engine.get_context(device)
    dev = T.device("cuda", device)
    N = virt.circuit.num_clbits
    vgates = [instr.operation for instr in virt.vgate_instructions]
    V = len(vgates)
    if N + V > MAX_KEY_BITS:
        raise ValueError(f"truncation='reference' holds dense vectors of 2^(N + V) = 2^{N + V} keys "
                         f"(at most 2^{MAX_KEY_BITS})")
    frags = [fs for fs in engine.prepare_fragments(virt, device, basis=False) if not fs.dropped]
    parts = []  # per fragment: (J [U, 2^c * 2^m] device, keys [2^c * 2^m] device, label -> row)
    for fs in frags:
        if any(isinstance(s.endpoint, BranchMeasure) for s in fs.prog.slots):
            raise ValueError("truncation='reference': fragments with plain mid-circuit measurements")
        jobs = fs.jobs
        touched = [j for j in range(V) if fs.touches[j]]
        tmask = sum(1 << j for j in touched)
        c, m = len(touched), fs.prog.m
        width = 1 << m
        n_rows = len(fs.swept_labels)
        label_of_job = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(jobs.label_offsets))
        cidx = _pext_np(jobs.branch_bits.astype(np.int64), tmask)
        dst = label_of_job * (1 << c) + cidx
        if np.unique(dst).size != dst.size:
            raise ValueError("two branch jobs of one instance with the same config outcome")
        J = T.zeros((max(n_rows, 1) << c) * width, dtype=T.float64, device=dev)
        if jobs.n_jobs:
            slot_t, _, _ = engine.jobs_to_device(jobs, device)
            ones = T.ones(jobs.n_jobs, dtype=T.float64, device=dev)
            pjob, _ = engine.sweep_jobs(ctx, fs.dprog, slot_t, ones, jobs.n_jobs)
            pjob = engine.fold_traced(ctx, pjob, fs.fold).contiguous()
            dst_t = T.from_numpy(dst).to(dev)
            ctx.check(ctx.lib.qk_qd_from_rows(ctx.handle, jobs.n_jobs, width, pjob.data_ptr(), dst_t.data_ptr(), acc,
                                              J.data_ptr()), "qk_qd_from_rows")
        keys = (deposit_keys([N + j for j in touched])[:, None] | deposit_keys(list(fs.prog.clbits))[None, :]).reshape(-1)
        row = {lab: int(r) for lab, r in zip(fs.labels, fs.row_of_label())}
        parts.append((J.view(max(n_rows, 1), -1), T.from_numpy(np.ascontiguousarray(keys)).to(dev), row, fs.touches))
    n_keys = 1 << (N + V)
    # after the first merge the vector is dense over 2^(N + V) keys, and every further merge forms
    # 2^(N + V) x (the next fragment's 2^(c + m)) products per label: refused when that is beyond
    # MAX_MERGE_ITEMS (three fragments near the key-bit limit would run for hours)
    for J, _, _, _ in parts[2:]:
        if n_keys * J.shape[1] > MAX_MERGE_ITEMS:
            raise ValueError(f"truncation='reference': merging a third fragment forms 2^{N + V} x {J.shape[1]} "
                             f"products per label (at most {MAX_MERGE_ITEMS}); use the default truncation")
    one = T.ones(1, dtype=T.float64, device=dev)
    zero_key = T.zeros(1, dtype=T.int64, device=dev)

    def merge(a, ka, b, kb):
        out = T.empty(n_keys, dtype=T.float64, device=dev)
        ctx.check(ctx.lib.qk_qd_merge(ctx.handle, a.numel(), a.data_ptr(), engine._ptr(ka), b.numel(), b.data_ptr(),
                                      engine._ptr(kb), acc, n_keys, out.data_ptr()), "qk_qd_merge")
        return out

    def leaf(label):
        """_merge_distrs (virtual_circuit.py:216-221) of one global label's fragment results."""
        vec = None
        for J, keys, row, touches in parts:
            flab = tuple(label[j] if touches[j] else -1 for j in range(V))
            x = J[row[flab]]
            if vec is None:
                vec, kv = x, keys
            else:
                vec, kv = merge(vec, kv, x, keys), None
        if kv is not None:  # one fragment: its distribution as it stands, on the dense key space
            vec = merge(vec, kv, one, zero_key)
        return DenseQD(ctx, vec, N + V, acc)

    return knit_label_tree(vgates, N, leaf).t


def knit_label_tree(vgates: list, N: int, leaf):
    """The knit loop of ``virtual_circuit.py:50-68`` depth-first: ``leaf(label)`` gives the merged
    result of one global label (a :class:`DenseQD` over ``N + V`` key bits); gate ``j``'s knit
    (``vgates[j].knit``, clbit index ``N + j``) runs on each chunk of ``num_instantiations``
    consecutive labels as soon as the chunk is complete — the reference knits all chunks of the
    last gate first, but each chunk's result depends on that chunk alone."""
    V = len(vgates)

    def subtree(prefix: tuple):
        j = len(prefix)
        if j == V:
            return leaf(prefix)
        chunk = [subtree(prefix + (i,)) for i in range(vgates[j].num_instantiations)]
        return vgates[j].knit(chunk, N + j)

    return subtree(())

