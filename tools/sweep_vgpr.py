#!/usr/bin/env python3
"""Register and LDS budget of the generated sweep kernels (offline: hipcc --genco, no GPU).

For a BASELINE config's plan, generates the per-program and multi-fragment sources exactly as the plan
compiles them (engine.jit_sources) and prints each kernel's VGPR / SGPR / LDS counts from the code
object's metadata — as generated, and with the FINAL pass's branch-job loop replaced by a single job
(what the loop's invariants and running sums cost in registers). QKNIT_SWEEP_LANE_XCHG applies.

    python tools/sweep_vgpr.py [--workload syc_32_5_p2]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def notes(hsaco: str) -> list:
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", hsaco], capture_output=True,
                         text=True, check=True).stdout
    kern = []
    for block in re.split(r"\n\s*- \.agpr_count:", out)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block).group(1)
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", block).group(1))  # noqa: E731
        kern.append({"kernel": name, "vgpr": get("vgpr_count"), "sgpr": get("sgpr_count"),
                     "lds_bytes": get("group_segment_fixed_size"), "vgpr_spill": get("vgpr_spill_count")})
    return kern


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    args = ap.parse_args()
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.build import hipcc

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    res = []
    with tempfile.TemporaryDirectory() as tmp:
        for i, (src, _) in enumerate(engine.jit_sources(VirtualCircuit(cut), basis=True)):
            for variant, text in (("as generated", src),
                                  ("FINAL: one branch job", src.replace(
                                      "for (long long job = j0; job < j1; ++job) {",
                                      "{ const long long job = j0; (void)j1;"))):
                f = os.path.join(tmp, f"s{i}.hip")
                open(f, "w").write(text)
                obj = f + ".hsaco"
                subprocess.run([hipcc(), "--genco", "--no-gpu-bundle-output", *engine.jit_options(text), f, "-o", obj],
                               check=True, capture_output=True)
                for k in notes(obj):
                    res.append({"source": i, "variant": variant, **k})
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
