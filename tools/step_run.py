#!/usr/bin/env python3
"""Run the bench step (KnitPipeline, syc 32 5 by default) a few times, nothing else: the program a
rocprofv3 pass profiles when only the step's kernels should appear (prep-chain counters,
profiles/r03_prep_pmc.json via tools/prep_pmc.py).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -- python3 tools/step_run.py --steps 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    for _ in range(args.warmup + args.steps):
        pipe.step()
    torch.cuda.synchronize()
    pipe.sync_stats()
    print(f"steps {args.steps}, rank {pipe.last_rank}, fallbacks {pipe.rank_fallbacks}", flush=True)


if __name__ == "__main__":
    main()
