"""Sparse quasi-probability distribution with the reference's truncation rule.

Mirrors ``third_party/qvm/qvm/quasi_distr.py`` (the reference's result type):
a ``dict[int, float]`` keyed by the integer value of the concatenated classical
registers (bit ``i`` = clbit ``i``), whose constructor drops every entry with
``|v| <= ACCURACY`` (``quasi_distr.py:3,7-10``). It is the interchange format of
the reference knit API; the dense GPU path converts to/from it only at the
boundary (:func:`QuasiDistr.from_dense`, :meth:`QuasiDistr.to_dense`).
"""
from __future__ import annotations

from typing import Union

import numpy as np

#: truncation threshold, ``quasi_distr.py:3``
ACCURACY = 1e-5


def _keep(v: float) -> bool:
    return abs(v) > ACCURACY


class QuasiDistr(dict):
    def __init__(self, data: dict) -> None:
        super().__init__((k, v) for k, v in data.items() if _keep(v))

    # ---- conversions ---------------------------------------------------------
    @staticmethod
    def from_counts(counts: dict) -> "QuasiDistr":
        """Counts keyed by space-separated bit strings (``quasi_distr.py:12-20``)."""
        total = sum(counts.values())
        return QuasiDistr({int(k.replace(" ", ""), 2): c / total for k, c in counts.items()})

    def to_counts(self, num_clbits: int, shots: int) -> dict:
        """``quasi_distr.py:22-26``: ``int(|p| * shots)`` per zero-padded key."""
        return {format(k, "b").zfill(num_clbits): int(abs(v * shots)) for k, v in self.items()}

    @staticmethod
    def from_dense(vec, threshold: float | None = None) -> "QuasiDistr":
        """Dense vector (numpy or torch) -> QuasiDistr, keeping ``|v| > ACCURACY``."""
        thr = ACCURACY if threshold is None else threshold
        if hasattr(vec, "detach"):  # torch tensor: threshold where it lives, move only the survivors
            flat = vec.detach().reshape(-1)
            keep = (flat.abs() > thr).nonzero().reshape(-1)
            idx = keep.cpu().numpy()
            vals = flat[keep].cpu().numpy() if idx.size else np.zeros(0)
            out = QuasiDistr({})
            dict.update(out, zip(idx.tolist(), vals.tolist()))
            return out
        vec = np.asarray(vec, dtype=np.float64).ravel()
        idx = np.nonzero(np.abs(vec) > thr)[0]
        out = QuasiDistr({})
        dict.update(out, zip(idx.tolist(), vec[idx].tolist()))
        return out

    def to_dense(self, num_bits: int) -> np.ndarray:
        out = np.zeros(1 << num_bits, dtype=np.float64)
        for k, v in self.items():
            out[k] = v
        return out

    # ---- projection ------------------------------------------------------------
    def nearest_probability_distribution(self) -> dict:
        """Simplex projection of ``quasi_distr.py:28-43``.

        Entries are visited in ascending value order; a running negative mass
        ``beta`` is spread uniformly over the entries not yet visited, and an
        entry whose shifted value is negative is dropped (and its value folded
        into ``beta``).
        """
        ordered = sorted(self.items(), key=lambda kv: kv[1])
        remaining = len(ordered)
        beta = 0.0
        out = {}
        for k, v in ordered:
            shift = beta / remaining
            if v + shift < 0:
                beta += v
                remaining -= 1
            else:
                out[k] = v + shift
        return out

    # ---- algebra ---------------------------------------------------------------
    def split(self, bit_index: int) -> tuple["QuasiDistr", "QuasiDistr"]:
        """Partition on ``bit_index``; the bit is cleared in the second half."""
        mask = 1 << bit_index
        lo = {k: v for k, v in self.items() if not k & mask}
        hi = {k ^ mask: v for k, v in self.items() if k & mask}
        return QuasiDistr(lo), QuasiDistr(hi)

    def merge(self, other: "QuasiDistr") -> "QuasiDistr":
        """Outer product with XOR-combined keys (``quasi_distr.py:55-60``)."""
        # Supports are disjoint in valid use; on a key collision the later
        # (self-major, other-minor) product overwrites, as in the reference.
        out = {k1 ^ k2: v1 * v2 for k1, v1 in self.items() for k2, v2 in other.items()}
        return QuasiDistr(out)

    def _combine(self, other: "QuasiDistr", sign: float) -> "QuasiDistr":
        out = dict(self)
        for k, v in other.items():
            out[k] = out.get(k, 0.0) + sign * v
        return QuasiDistr(out)

    def __add__(self, other: "QuasiDistr") -> "QuasiDistr":
        return self._combine(other, 1.0)

    def __sub__(self, other: "QuasiDistr") -> "QuasiDistr":
        return self._combine(other, -1.0)

    def __mul__(self, other: Union[int, float, "QuasiDistr"]) -> "QuasiDistr":
        if isinstance(other, QuasiDistr):
            return self.merge(other)
        if isinstance(other, (int, float)):
            return QuasiDistr({k: v * other for k, v in self.items()})
        raise TypeError(f"Cannot multiply QuasiDistr by {type(other)}")

    def __rmul__(self, other):
        return self.__mul__(other)
