"""The benchmarks/benchmark.py counterpart (reference ``benchmarks/benchmark.py:22-103``)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
GOLD = os.path.join(ROOT, "tests", "golden")

import benchmark  # noqa: E402


def _gold(name):
    g = json.load(open(os.path.join(GOLD, name)))
    return {int(k): v for k, v in g["npd_acc_1e-05"]}


CASES = [(["-p", "2", "-q", "3", "bv", "5", "1"], "knit_bv_5_1_p2.json", {"S": 8, "A": 8, "nWireCuts": 1, "Q": 3}),
         (["-p", "2", "-q", "8", "hwe", "16", "1"], "knit_hwe_16_1_p2.json", {"S": 6, "A": 0, "nGateCuts": 1, "Q": 8})]


@pytest.mark.parametrize("argv,gold,keys", CASES)
def test_benchmark_cut_and_cpu_baseline(argv, gold, keys, monkeypatch):
    """Cut + model key results (Cutter.py:164-179 semantics) + the reference's CPU algorithm
    (exact instances, literal dict knit in Pool(8)), whose result equals the reference knit's."""
    import bench

    seen = {}
    real = bench.cpu_baseline_qvm
    monkeypatch.setattr(bench, "cpu_baseline_qvm", lambda cut: seen.setdefault("r", real(cut, return_result=True)))
    s = benchmark.run(benchmark.parse(argv + ["--cpu-baseline", "--no-gpu", "--no-save"]))
    assert s["success"]
    for k, v in keys.items():
        assert s["model"][k] == v
    cpu = seen["r"]
    assert cpu["status"] == "ok" and cpu["processes"] == 8
    ref = _gold(gold)
    assert set(cpu["result"]) == set(ref)
    for k in ref:
        assert abs(cpu["result"][k] - ref[k]) <= 1e-9


def test_benchmark_unsat_caps_exit_cleanly():
    """A cut that breaks -q is the reference's unsat case (benchmark.py:53-54): success False."""
    s = benchmark.run(benchmark.parse(["-p", "2", "-q", "8", "syc", "32", "5", "--no-gpu", "--no-save"]))
    assert s["success"] is False and "-q 8" in s["reason"]
    assert s["model"]["nGateCuts"] == 4 and s["model"]["S"] == 1296


def test_benchmark_cpu_baseline_dnf_for_wide_outputs():
    import bench
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    _, cut, _ = cutting.config_cut_circuit("syc", 32, 1, 2)
    r = bench.cpu_baseline_qvm(cut)
    assert r["status"] == "DNF" and "2^32" in r["reason"]


def test_benchmark_cutspec_file(tmp_path):
    spec = {"partitions": [[0, 1, 2, 3, 4, 5, 6, 7], [8, 9, 10, 11, 12, 13, 14, 15]], "gate_cuts": [],
            "wire_cuts": []}
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.generators import gen_circ

    circ = cutting.decompose(gen_circ("hwe", 16, 1))
    spec["gate_cuts"] = cutting.two_qubit_gate_indices(circ, 7, 8)[:1]
    p = tmp_path / "cut.json"
    p.write_text(json.dumps(spec))
    s = benchmark.run(benchmark.parse(["-p", "2", "-q", "8", "hwe", "16", "1", "--cutspec", str(p), "--no-gpu",
                                       "--no-save", "--cut-only"]))
    assert s["success"] and s["model"]["nGateCuts"] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("argv,gold,keys", CASES)
def test_benchmark_gpu_fidelity_and_result(argv, gold, keys, require_gpu):
    """GPU leg: cutVsUncutFidelity (Utilities.py:224) = 1 - O(1e-12), the reference-shaped dict
    (run.py:71) equals the reference knit's golden NPD."""
    s = benchmark.run(benchmark.parse(argv + ["--no-save"]))
    assert s["success"]
    assert abs(s["cutVsUncutFidelity"] - 1.0) <= 1e-12
    ref = _gold(gold)
    assert set(s["result"]) == set(ref)
    for k in ref:
        assert abs(s["result"][k] - ref[k]) <= 1e-9
