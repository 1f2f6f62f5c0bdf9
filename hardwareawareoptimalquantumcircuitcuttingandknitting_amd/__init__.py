"""MI355X-native knitting hot path of HardwareAwareOptimalQuantumCircuitCuttingAndKnitting.

Public surface mirrors the reference's ``qvm`` package (``third_party/qvm/qvm``):

* :class:`VirtualCircuit`, :func:`generate_instantiations`   (``virtual_circuit.py``)
* :func:`run_virtual_circuit`, :class:`RunTimeInfo`           (``run.py``)
* :class:`QuasiDistr`                                          (``quasi_distr.py``)
* virtual gates and ``VIRTUAL_GATE_TYPES``                     (``virtual_gates.py``)

plus the circuit IR (:mod:`.circuit`), the benchmark generators and cut-spec
builder (:mod:`.generators`, :mod:`.cutting`) and the engine (:mod:`.engine`,
C ABI in ``include/qknit.h``).
"""
from .circuit import ClassicalRegister, QuantumCircuit, QuantumRegister
from .quasi_distr import QuasiDistr
from .virtual_gates import (
    RZZ_ACCURACY,
    VIRTUAL_GATE_TYPES,
    VirtualBinaryGate,
    VirtualCPhase,
    VirtualCX,
    VirtualCY,
    VirtualCZ,
    VirtualGateEndpoint,
    VirtualMove,
    VirtualRZZ,
    WireCut,
)
from .virtual_circuit import VirtualCircuit, generate_instantiations
from .run import RunTimeInfo, run_virtual_circuit, run_virtual_circuit_dense

__all__ = [
    "ClassicalRegister", "QuantumCircuit", "QuantumRegister", "QuasiDistr", "RZZ_ACCURACY",
    "VIRTUAL_GATE_TYPES", "VirtualBinaryGate", "VirtualCPhase", "VirtualCX", "VirtualCY",
    "VirtualCZ", "VirtualGateEndpoint", "VirtualMove", "VirtualRZZ", "WireCut", "VirtualCircuit",
    "generate_instantiations", "RunTimeInfo", "run_virtual_circuit", "run_virtual_circuit_dense",
]
