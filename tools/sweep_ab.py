#!/usr/bin/env python3
"""A/B of the per-program sweep kernels with and without cross-lane butterflies
(QKNIT_SWEEP_LANE_XCHG, sweep_codegen._plan_layouts), interleaved rounds in one process, for the bench
plan's sweep (basis-reduced, pruned: 250 branch jobs) and the full direct sweep (2592 jobs). The two
variants run the same arithmetic on the same amplitudes (the exchange only moves data between lanes),
so their rows must be bit-identical; printed per round: ms per sweep of each.

    python tools/sweep_ab.py [--rounds 4] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    pipes = {}
    for plan, factored in (("bench", True), ("full", False)):
        for x in ("1", "0"):
            os.environ["QKNIT_SWEEP_LANE_XCHG"] = x
            pipes[(plan, x)] = KnitPipeline(VirtualCircuit(cut), factored=factored)
    os.environ.pop("QKNIT_SWEEP_LANE_XCHG")
    res = {"equal": {}, "ms": {f"{k[0]}/xchg={k[1]}": [] for k in pipes}}
    for plan in ("bench", "full"):
        a = [q.clone() for q in pipes[(plan, "1")].sweep()]
        b = [q.clone() for q in pipes[(plan, "0")].sweep()]
        res["equal"][plan] = all(bool(torch.equal(x, y)) for x, y in zip(a, b))
    for _ in range(args.rounds):
        for key, pipe in pipes.items():
            for _ in range(3):
                pipe.sweep()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                pipe.sweep()
            e.record()
            torch.cuda.synchronize()
            res["ms"][f"{key[0]}/xchg={key[1]}"].append(round(s.elapsed_time(e) / args.reps, 4))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
