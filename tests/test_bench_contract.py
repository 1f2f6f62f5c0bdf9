"""bench.py's output contract (the driver parses its one JSON line): one short run of the headline
workload on the GPU with the optional legs off, checked for the keys and invariants the task's bench
contract names — metric / value / unit, ms_per_step consistent with value, the roofline block of the
write kernel (achieved <= peak, frac = achieved / peak) and the config's workload."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_bench_json_line_contract(require_gpu):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--no-north-star", "--no-npd", "--no-drop-in", "--no-general"]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["config"]["workload"] == "syc 32 5 p=2"
    # value = reference instances per second of whole full knits
    assert abs(d["value"] - d["config"]["instances_ref"] / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["achieved"] <= r["peak"] and abs(r["frac"] - r["achieved"] / r["peak"]) <= 1e-9
    # the write kernel runs inside the step
    assert r["avg_launch_ms"] <= d["ms_per_step"]

