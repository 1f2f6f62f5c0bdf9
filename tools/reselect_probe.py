#!/usr/bin/env python3
"""Where a drop-in call that re-selects its output mapping spends its time, in a process shaped like
bench.py's (the bench pipeline's own 34-GB output alive, the NPD leg run, then the drop-in calls).

    python tools/reselect_probe.py [--force]

``--force``: OUT_FAST_GBS = inf, so the first call's un-checked mapping is always replaced."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-bench-pipe", action="store_true", help="skip the bench pipeline (fresh-process shape)")
    args = ap.parse_args()
    import torch

    import bench
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine, quasi_distr
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import clear_plan_cache, run_virtual_circuit

    if args.force:
        engine.OUT_FAST_GBS = float("inf")
    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    torch.cuda.set_stream(torch.cuda.Stream())
    rec = {}
    if not args.no_bench_pipe:
        pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
        for _ in range(3):
            pipe.step()
        torch.cuda.synchronize()
        rec["npd"] = bench.npd_timing(pipe.out, quasi_distr.ACCURACY)
    clear_plan_cache()
    calls = []
    for i in range(4):
        nlog = len(engine.out_selection_log)
        free0 = torch.cuda.mem_get_info()[0]
        t0 = time.perf_counter()
        out, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)
        torch.cuda.synchronize()
        calls.append({"ms": round((time.perf_counter() - t0) * 1e3, 2), "free_GiB_before": round(free0 / 2**30, 1),
                      "selection": engine.out_selection_log[nlog:]})
        del out
    rec["calls"] = calls
    rec["out_selections"] = engine.out_selections
    rec["out_stats"] = engine.out_stats()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
