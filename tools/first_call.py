#!/usr/bin/env python3
"""The drop-in's first call in a fresh process, as the reference's harness makes it
(``Utilities.py:74-89``: ``VirtualCircuit(cutCircuit.copy())`` then one ``run_virtual_circuit`` per run).

Prints one JSON line: import + device init, ``VirtualCircuit``, the first
``run_virtual_circuit(virt, dense=True)`` with its breakdown (``KnitPipeline.first_call_ms``: the plan's
phases, the output buffer, the step) and a few later calls on fresh ``VirtualCircuit`` objects.

    python tools/first_call.py [--workload syc_32_5_p2] [--calls 3] [--dict]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--dict", action="store_true", help="the reference-shaped dict result instead of dense=True")
    args = ap.parse_args()
    t0 = time.perf_counter()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import cached_plan, run_virtual_circuit

    torch.cuda.init()
    engine.get_context(0)
    t_init = time.perf_counter() - t0
    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    kw = {} if args.dict else {"dense": True}
    t = time.perf_counter()
    virt = VirtualCircuit(cut)
    t_virt = time.perf_counter() - t
    t = time.perf_counter()
    out, info = run_virtual_circuit(virt, **kw)
    torch.cuda.synchronize()
    first = time.perf_counter() - t
    pipe = cached_plan(virt, 0)
    del out
    later = []
    for _ in range(args.calls):
        v = VirtualCircuit(cut)
        t = time.perf_counter()
        out, _ = run_virtual_circuit(v, **kw)
        torch.cuda.synchronize()
        later.append((time.perf_counter() - t) * 1e3)
        del out
    print(json.dumps({"workload": args.workload, "api": "dict" if args.dict else "dense=True",
                      "import_and_device_init_ms": round(t_init * 1e3, 1),
                      "virtual_circuit_ms": round(t_virt * 1e3, 2), "first_call_ms": round(first * 1e3, 2),
                      "first_call_breakdown_ms": {k: round(v, 2) for k, v in getattr(pipe, "first_call_ms", {}).items()},
                      "later_calls_ms": [round(x, 2) for x in later], "out_alloc": getattr(pipe, "out_alloc", None),
                      "out_selections": engine.out_selections}), flush=True)


if __name__ == "__main__":
    main()
