"""Gate matrices for the oracle (qiskit 0.44 definitions, little-endian 2-qubit order).

TEST INFRASTRUCTURE ONLY. Independent of the product's gate table so the two
can check each other.
"""
import cmath
import math

import numpy as np


def _u(theta, phi, lam):
    c, s = math.cos(theta / 2), math.sin(theta / 2)
    return np.array([[c, -cmath.exp(1j * lam) * s],
                     [cmath.exp(1j * phi) * s, cmath.exp(1j * (phi + lam)) * c]])


def _ph(lam):
    return np.array([[1, 0], [0, cmath.exp(1j * lam)]])


def _ctrl(u):
    # control = first qubit (bit 0 of the 2-qubit index), target = second
    m = np.eye(4, dtype=complex)
    m[np.ix_([1, 3], [1, 3])] = u
    return m


def matrix(name, params=()):
    p = [float(x) for x in params]
    r2 = 1 / math.sqrt(2)
    one = {
        "id": lambda: np.eye(2), "x": lambda: np.array([[0, 1], [1, 0]]),
        "y": lambda: np.array([[0, -1j], [1j, 0]]), "z": lambda: np.diag([1, -1]),
        "h": lambda: np.array([[r2, r2], [r2, -r2]]), "s": lambda: _ph(math.pi / 2),
        "sdg": lambda: _ph(-math.pi / 2), "t": lambda: _ph(math.pi / 4), "tdg": lambda: _ph(-math.pi / 4),
        "sx": lambda: 0.5 * np.array([[1 + 1j, 1 - 1j], [1 - 1j, 1 + 1j]]),
        "rx": lambda t: np.array([[math.cos(t / 2), -1j * math.sin(t / 2)], [-1j * math.sin(t / 2), math.cos(t / 2)]]),
        "ry": lambda t: np.array([[math.cos(t / 2), -math.sin(t / 2)], [math.sin(t / 2), math.cos(t / 2)]]),
        "rz": lambda t: np.diag([cmath.exp(-0.5j * t), cmath.exp(0.5j * t)]),
        "p": _ph, "u1": _ph, "u2": lambda f, l: _u(math.pi / 2, f, l), "u3": _u, "u": _u,
        "r": lambda t, f: np.array([[math.cos(t / 2), -1j * cmath.exp(-1j * f) * math.sin(t / 2)],
                                    [-1j * cmath.exp(1j * f) * math.sin(t / 2), math.cos(t / 2)]]),
    }
    two = {
        "cx": lambda: _ctrl(np.array([[0, 1], [1, 0]])),
        "cy": lambda: _ctrl(np.array([[0, -1j], [1j, 0]])),
        "cz": lambda: np.diag([1, 1, 1, -1]),
        "cp": lambda l: np.diag([1, 1, 1, cmath.exp(1j * l)]),
        "crz": lambda t: _ctrl(np.diag([cmath.exp(-0.5j * t), cmath.exp(0.5j * t)])),
        "rzz": lambda t: np.diag([cmath.exp(-0.5j * t), cmath.exp(0.5j * t), cmath.exp(0.5j * t), cmath.exp(-0.5j * t)]),
        "swap": lambda: np.eye(4)[[0, 2, 1, 3]],
    }
    if name in one:
        return np.asarray(one[name](*p), dtype=complex)
    if name in two:
        return np.asarray(two[name](*p), dtype=complex)
    raise ValueError(f"oracle: unknown gate {name}")
