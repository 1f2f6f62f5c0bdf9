"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's knitting hot path
(thangktran/HardwareAwareOptimalQuantumCircuitCuttingAndKnitting,
``third_party/qvm/qvm/{run,virtual_circuit,virtual_gates,quasi_distr}.py``),
used as the checker of the MI355X product path. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product package never does.

* :mod:`oracle.quasi`       — ``QuasiDistr`` restated (dict arithmetic + ``ACCURACY`` truncation)
* :mod:`oracle.tables`      — instantiation tables + knit rules of every virtual gate type
* :mod:`oracle.statevector` — exact branching statevector (numpy), the semantics Aer samples from
* :mod:`oracle.qvm`         — fragments, labels, instance programs and the literal dict knit
* :mod:`oracle.dense`       — dense numpy knit + uncut reference distribution (known answer)

Pinning: the tables, the ``QuasiDistr`` algebra and the knit are
checked against golden vectors produced by the reference's own code
(``tests/golden/make_golden.py`` imports ``third_party/qvm`` with placeholder
qiskit modules in the build container); the simulation semantics (Aer 0.13,
not present) are pinned by the known answer "knit of exact fragment
distributions == exact uncut distribution".
"""
