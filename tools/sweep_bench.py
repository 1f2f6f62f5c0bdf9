#!/usr/bin/env python3
"""Time the batched sweep alone for a BASELINE workload, per sweep-chunk size (interleaved rounds).

  python tools/sweep_bench.py [--workload syc_32_5_p2] [--reps 5] [--chunks 0 512 256 128]

Each chunk size is a KnitPipeline (factored, basis-reduced sweep) whose fused fragments run
their passes chunk by chunk through one workspace (engine.label_chunks; 0 = no chunking).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunks", type=int, nargs="*", default=[0, 640, 320, 256, 160, 128, 64])
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    pipes = {c: KnitPipeline(VirtualCircuit(cut), factored=True, chunk_jobs=c) for c in args.chunks}
    ref = [q.clone() for q in pipes[args.chunks[0]].sweep()]
    for c, pipe in pipes.items():
        got = pipe.sweep()
        assert all(torch.equal(a, b) for a, b in zip(got, ref)), f"chunk {c}: sweep differs"
    torch.cuda.synchronize()
    times = {c: [] for c in pipes}
    for rep in range(args.reps):
        for c, pipe in pipes.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            pipe.sweep()
            e.record()
            torch.cuda.synchronize()
            times[c].append(s.elapsed_time(e))
    jobs = pipes[args.chunks[0]].instance_counts()["branch_jobs"]
    for c, t in times.items():
        t = sorted(t)
        print(f"chunk_jobs {c:5d}: sweep median {t[len(t) // 2]:.3f} ms  min {t[0]:.3f} ms  ({jobs} jobs)", flush=True)


if __name__ == "__main__":
    main()
