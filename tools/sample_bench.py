#!/usr/bin/env python3
"""Shot-sampling mode timing (run_virtual_circuit(..., sample=True)) on BASELINE shapes.

  python tools/sample_bench.py [--shots 20000] [--reps 3] [--configs syc_32_5_p2 hwe_16_1_p2]

Per config: the per-fragment sampling (sweep of the unique instances + CDF + draws + fold, HIP
events) and the direct knit over all reference labels, as run_virtual_circuit_dense does it.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shots", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", nargs="*", default=["hwe_16_1_p2", "syc_32_5_p2"])
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import run_virtual_circuit_dense

    for key in args.configs:
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
        virt = VirtualCircuit(cut)
        ctx = engine.get_context(0)
        frags = engine.prepare_fragments(virt, 0)
        for i, fs in enumerate(frags):  # warm-up (module compile, allocator)
            engine.sample_fragment(ctx, fs, args.shots, engine.fragment_seed(1, i), 1e-5)
        torch.cuda.synchronize()
        samp = []
        for rep in range(args.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i, fs in enumerate(frags):
                engine.sample_fragment(ctx, fs, args.shots, engine.fragment_seed(rep, i), 1e-5)
            e.record()
            torch.cuda.synchronize()
            samp.append(s.elapsed_time(e))
        t0 = time.perf_counter()
        out, info = run_virtual_circuit_dense(virt, shots=args.shots, sample=True, seed=7)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        labels = sum(len(fs.labels) for fs in frags)
        print(json.dumps({
            "config": key, "shots": args.shots, "instances_ref": labels, "draws": labels * args.shots,
            "sampling_ms": sorted(samp)[len(samp) // 2],
            "draws_per_s": labels * args.shots / (sorted(samp)[len(samp) // 2] * 1e-3),
            "run_time_s": info.run_time, "knit_time_s": info.knit_time, "wall_s": wall,
            "sum_minus_1": float(out.sum()) - 1.0,
        }), flush=True)
        del out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
