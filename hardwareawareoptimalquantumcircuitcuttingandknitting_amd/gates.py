"""Gate library: unitary matrices for the gate names a HwAwareCutter cut circuit contains.

Conventions follow the qiskit 0.44 gate definitions the reference relies on
(reference pins qiskit-terra 0.25.2.1, ``/root/reference/pdm.lock:1047``):

* 1-qubit matrices are 2x2 in the computational basis ``|0>, |1>``.
* 2-qubit matrices act on ``(qubits[0], qubits[1])`` and are indexed
  little-endian: basis index ``b0 + 2*b1`` where ``b0`` is the bit of
  ``qubits[0]`` (so ``cx`` has its control on ``qubits[0]``).

Global phases are irrelevant for the knitted probability distributions and
are not tracked (qiskit's ``decompose()`` changes them freely).
"""
from __future__ import annotations

import cmath
import math

import numpy as np

_S2 = 1.0 / math.sqrt(2.0)


def _u3(theta: float, phi: float, lam: float) -> np.ndarray:
    c, s = math.cos(theta / 2.0), math.sin(theta / 2.0)
    return np.array(
        [[c, -cmath.exp(1j * lam) * s], [cmath.exp(1j * phi) * s, cmath.exp(1j * (phi + lam)) * c]],
        dtype=np.complex128,
    )


def _rx(t: float) -> np.ndarray:
    c, s = math.cos(t / 2.0), math.sin(t / 2.0)
    return np.array([[c, -1j * s], [-1j * s, c]], dtype=np.complex128)


def _ry(t: float) -> np.ndarray:
    c, s = math.cos(t / 2.0), math.sin(t / 2.0)
    return np.array([[c, -s], [s, c]], dtype=np.complex128)


def _rz(t: float) -> np.ndarray:
    return np.array([[cmath.exp(-0.5j * t), 0], [0, cmath.exp(0.5j * t)]], dtype=np.complex128)


def _p(lam: float) -> np.ndarray:
    return np.array([[1, 0], [0, cmath.exp(1j * lam)]], dtype=np.complex128)


def _r(theta: float, phi: float) -> np.ndarray:
    c, s = math.cos(theta / 2.0), math.sin(theta / 2.0)
    return np.array(
        [[c, -1j * cmath.exp(-1j * phi) * s], [-1j * cmath.exp(1j * phi) * s, c]], dtype=np.complex128
    )


def _controlled(u: np.ndarray) -> np.ndarray:
    """Control on qubits[0] (bit b0), target qubits[1]; little-endian 4x4."""
    m = np.eye(4, dtype=np.complex128)
    # indices with b0 = 1: 1 (b1=0), 3 (b1=1)
    m[1, 1], m[1, 3] = u[0, 0], u[0, 1]
    m[3, 1], m[3, 3] = u[1, 0], u[1, 1]
    return m


X = np.array([[0, 1], [1, 0]], dtype=np.complex128)
Y = np.array([[0, -1j], [1j, 0]], dtype=np.complex128)
Z = np.array([[1, 0], [0, -1]], dtype=np.complex128)
H = np.array([[_S2, _S2], [_S2, -_S2]], dtype=np.complex128)
I2 = np.eye(2, dtype=np.complex128)

ONE_QUBIT = {
    "id": lambda: I2.copy(),
    "i": lambda: I2.copy(),
    "x": lambda: X.copy(),
    "y": lambda: Y.copy(),
    "z": lambda: Z.copy(),
    "h": lambda: H.copy(),
    "s": lambda: _p(math.pi / 2),
    "sdg": lambda: _p(-math.pi / 2),
    "t": lambda: _p(math.pi / 4),
    "tdg": lambda: _p(-math.pi / 4),
    "sx": lambda: 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]], dtype=np.complex128),
    "sxdg": lambda: 0.5 * np.array([[1 - 1j, 1 + 1j], [1 + 1j, 1 - 1j]], dtype=np.complex128),
    "rx": _rx,
    "ry": _ry,
    "rz": _rz,
    "p": _p,
    "u1": _p,
    "u2": lambda phi, lam: _u3(math.pi / 2, phi, lam),
    "u3": _u3,
    "u": _u3,
    "r": _r,
}

TWO_QUBIT = {
    "cx": lambda: _controlled(X),
    "cnot": lambda: _controlled(X),
    "cy": lambda: _controlled(Y),
    "cz": lambda: np.diag([1, 1, 1, -1]).astype(np.complex128),
    "ch": lambda: _controlled(H),
    "cp": lambda lam: np.diag([1, 1, 1, cmath.exp(1j * lam)]).astype(np.complex128),
    "cu1": lambda lam: np.diag([1, 1, 1, cmath.exp(1j * lam)]).astype(np.complex128),
    "crz": lambda t: _controlled(_rz(t)),
    "crx": lambda t: _controlled(_rx(t)),
    "cry": lambda t: _controlled(_ry(t)),
    "rzz": lambda t: np.diag(
        [cmath.exp(-0.5j * t), cmath.exp(0.5j * t), cmath.exp(0.5j * t), cmath.exp(-0.5j * t)]
    ).astype(np.complex128),
    "swap": lambda: np.array(
        [[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.complex128
    ),
}

# Gates that carry no quantum action on the statevector.
NON_UNITARY_NOOPS = {"barrier", "delay"}


def gate_matrix(name: str, params=()) -> np.ndarray:
    """Matrix of a named gate; raises ``ValueError`` for unknown names."""
    params = [float(p) for p in params]
    if name in ONE_QUBIT:
        return ONE_QUBIT[name](*params)
    if name in TWO_QUBIT:
        return TWO_QUBIT[name](*params)
    raise ValueError(f"unsupported gate '{name}'")


def num_gate_qubits(name: str) -> int:
    if name in ONE_QUBIT:
        return 1
    if name in TWO_QUBIT:
        return 2
    raise ValueError(f"unsupported gate '{name}'")


def is_diagonal(m: np.ndarray, tol: float = 0.0) -> bool:
    off = m - np.diag(np.diag(m))
    return bool(np.all(np.abs(off) <= tol))


def is_identity_up_to_phase(m: np.ndarray, tol: float = 1e-14) -> bool:
    if not is_diagonal(m, tol):
        return False
    d = np.diag(m)
    return bool(np.all(np.abs(d - d[0]) <= tol))
