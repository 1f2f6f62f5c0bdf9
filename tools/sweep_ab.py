#!/usr/bin/env python3
"""A/B of per-program sweep kernel variants (code-generation switches), interleaved rounds in one process,
for the bench plan's sweep (basis-reduced, pruned: 250 branch jobs) and the full direct sweep (2592
jobs). Every variant runs the same arithmetic on the same amplitudes (only data movement and register
allocation differ), so their rows must be bit-identical to the first variant's; printed: ms per sweep
per round, and the equality check.

Variants (environment at code generation): QKNIT_SWEEP_LANE_XCHG (0 LDS only, 1 permlane lane bits 4/5,
2 FINAL passes without LDS), QKNIT_SWEEP_OPAQUE_TID (0/1), QKNIT_SWEEP_WAVES_PER_EU (unset or N).

    python tools/sweep_ab.py [--rounds 4] [--reps 20] [--variants x0o0 x1o0 x1o1 x2o1 x2o1w4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(v: str) -> dict:
    """'x2o1w4' -> {LANE_XCHG: 2, OPAQUE_TID: 1, WAVES_PER_EU: 4}."""
    env = {"QKNIT_SWEEP_LANE_XCHG": v[v.index("x") + 1], "QKNIT_SWEEP_OPAQUE_TID": v[v.index("o") + 1]}
    if "w" in v:
        env["QKNIT_SWEEP_WAVES_PER_EU"] = v[v.index("w") + 1:]
    return env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", nargs="+", default=["x0o0", "x1o0", "x1o1", "x2o1", "x2o1w4"])
    ap.add_argument("--plans", nargs="+", default=["bench", "full"])
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    keys = ("QKNIT_SWEEP_LANE_XCHG", "QKNIT_SWEEP_OPAQUE_TID", "QKNIT_SWEEP_WAVES_PER_EU")
    pipes = {}
    for plan in args.plans:
        for v in args.variants:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(parse(v))
            pipes[(plan, v)] = KnitPipeline(VirtualCircuit(cut), factored=(plan == "bench"))
    for k in keys:
        os.environ.pop(k, None)
    res = {"equal": {}, "ms": {f"{p}/{v}": [] for p, v in pipes}}
    for plan in args.plans:
        ref = [q.clone() for q in pipes[(plan, args.variants[0])].sweep()]
        for v in args.variants[1:]:
            got = pipes[(plan, v)].sweep()
            res["equal"][f"{plan}/{v}"] = all(bool(torch.equal(x, y)) for x, y in zip(ref, got))
    for _ in range(args.rounds):
        for (plan, v), pipe in pipes.items():
            for _ in range(3):
                pipe.sweep()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                pipe.sweep()
            e.record()
            torch.cuda.synchronize()
            res["ms"][f"{plan}/{v}"].append(round(s.elapsed_time(e) / args.reps, 4))
    res["best_ms"] = {k: min(v) for k, v in res["ms"].items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
