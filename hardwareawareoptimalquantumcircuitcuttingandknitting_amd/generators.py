"""Benchmark circuit generators (the BASELINE.json configs: syc, hwe, bv, qft).

Re-implementations of the reference's circuit zoo front-end
(``benchmarks/helper_functions.py:206-234`` -> ``generate_circ`` ``:66-127``),
built on this package's circuit IR, with the reference's unseeded ``random``
replaced by a pinned seed. Every generator ends with
``measure_all()`` as ``helper_functions.py:163-185`` does.

* ``syc``  — ``gen_sycamore`` (``qcg/generators.py:46-74``, ``Qgrid_Sycamore.py:149-176``):
  grid ``factor_int(n)`` (``helper_functions.py:16-24``); per layer a random
  1-qubit gate per qubit chosen by ``Qbit.random_gate`` (``Qbit_Sycamore.py:10-19``:
  first draw ``randint(0, 2)`` over X/Y/W, later ``randint(0, 1)`` over the two
  gates other than the previous one), X = rx(pi/2), Y = ry(pi/2), W = z
  (``Qgrid_Sycamore.py:133-147``); then a CZ layer from pattern order ABCDCDAB
  (``:89,159-166``; patterns ``ABCD_layer_generation.py:5-54``).
* ``hwe``  — ``HWEA`` with "optimal" parameters (``hw_efficient_ansatz.py:79-104,118-190``).
* ``bv``   — Bernstein-Vazirani with secret ``1...1`` (``helper_functions.py:26-31``,
  ``bernstein_vazirani.py:61-98``).
* ``qft``  — qiskit ``QFT(n, approximation_degree=0, do_swaps=False).decompose()``
  (``helper_functions.py:83-86``): for ``j = n-1..0``: ``h(j)``, then
  ``cp(pi * 2^(k-j), j, k)`` for ``k = j-1..0``.
"""
from __future__ import annotations

import math
import random

from .circuit import QuantumCircuit, QuantumRegister

DEFAULT_SEED = 1234


def factor_int(n: int) -> tuple[int, int]:
    val = math.ceil(math.sqrt(n))
    while True:
        co = int(n / val)
        if val * co == n:
            return val, co
        val -= 1


def _pattern(rows: int, cols: int, which: str) -> list:
    out = []
    if which in "AB":
        for r in range(rows):
            start = (r % 2) if which == "A" else 1 - (r % 2)
            for c in range(start, cols, 2):
                if c != cols - 1:
                    out.append(((r, c), (r, c + 1)))
    else:
        for c in range(cols):
            start = (c % 2) if which == "C" else 1 - (c % 2)
            for r in range(start, rows, 2):
                if r != rows - 1:
                    out.append(((r, c), (r + 1, c)))
    return out


SYC_ORDER = "ABCDCDAB"
_NEXT_GATE = {"X": ("Y", "W"), "Y": ("X", "W"), "W": ("X", "Y")}


def sycamore(num_qubits: int, depth: int, seed: int | None = DEFAULT_SEED) -> QuantumCircuit:
    rows, cols = factor_int(num_qubits)
    rng = random.Random(seed)
    qr = QuantumRegister(rows * cols, "q")
    qc = QuantumCircuit(qr)
    prev = [[None] * cols for _ in range(rows)]
    for layer in range(depth):
        for r in range(rows):
            for c in range(cols):
                if prev[r][c] is None:
                    g = ("X", "Y", "W")[rng.randint(0, 2)]
                else:
                    g = _NEXT_GATE[prev[r][c]][rng.randint(0, 1)]
                prev[r][c] = g
                q = qr[r * cols + c]
                if g == "X":
                    qc.rx(math.pi / 2, q)
                elif g == "Y":
                    qc.ry(math.pi / 2, q)
                else:
                    qc.z(q)
        for (r0, c0), (r1, c1) in _pattern(rows, cols, SYC_ORDER[layer % len(SYC_ORDER)]):
            qc.cz(qr[r0 * cols + c0], qr[r1 * cols + c1])
    qc.measure_all()
    return qc


def hwea(num_qubits: int, depth: int) -> QuantumCircuit:
    n = num_qubits
    theta = [0.0] * (2 * n * (1 + depth))
    theta[0] = math.pi / 2
    for i in range(2 * n, 2 * n + n // 2):
        theta[i] = math.pi
    qr = QuantumRegister(n, "q")
    qc = QuantumCircuit(qr)
    p = 0
    for i in range(n):
        qc.u(theta[i + p], 0, 0, qr[i])
    p += n
    for i in range(n):
        qc.u(0, 0, theta[i + p], qr[i])
    p += n
    for _ in range(depth):
        for i in range(n - 1):
            qc.cx(qr[i], qr[i + 1])
        for i in range(n):
            qc.u(theta[i + p], 0, 0, qr[i])
        p += n
        for i in range(n):
            qc.u(0, 0, theta[i + p], qr[i])
        p += n
    qc.measure_all()
    return qc


def bernstein_vazirani(num_qubits: int) -> QuantumCircuit:
    secret = "1" * (num_qubits - 1)
    qr = QuantumRegister(num_qubits, "q")
    qc = QuantumCircuit(qr)
    qc.x(qr[num_qubits - 1])
    qc.h(qr)
    for i, bit in enumerate(reversed(secret)):
        if bit == "1":
            qc.cx(qr[i], qr[num_qubits - 1])
    qc.h(qr)
    qc.measure_all()
    return qc


def qft(num_qubits: int) -> QuantumCircuit:
    qr = QuantumRegister(num_qubits, "q")
    qc = QuantumCircuit(qr)
    for j in reversed(range(num_qubits)):
        qc.h(qr[j])
        for k in reversed(range(j)):
            qc.cp(math.pi * 2.0 ** (k - j), qr[j], qr[k])
    qc.measure_all()
    return qc


def gen_circ(name: str, num_qubits: int, depth: int, seed: int | None = DEFAULT_SEED) -> QuantumCircuit:
    """``genCirc`` (``helper_functions.py:206-234``) for the configs this build covers."""
    if name == "syc":
        return sycamore(num_qubits, depth, seed)
    if name == "hwe":
        return hwea(num_qubits, depth)
    if name == "bv":
        return bernstein_vazirani(num_qubits)
    if name == "qft":
        return qft(num_qubits)
    raise RuntimeError(f"circName {name} is not supported")
