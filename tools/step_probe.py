#!/usr/bin/env python3
"""Per-stage device time of one syc 32 5 pipeline step on the device data-rank path (HIP events).

  python tools/step_probe.py [--steps 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--workload", default="syc_32_5_p2")
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline, _mm_nt

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    be = pipe.be
    T = torch
    stages = {}

    def mark(label, t0):
        e = T.cuda.Event(enable_timing=True)
        e.record()
        stages.setdefault(label, []).append((t0, e))
        return e

    for it in range(args.steps + 2):
        e0 = T.cuda.Event(enable_timing=True)
        e0.record()
        qs = pipe.sweep()
        e1 = mark("sweep", e0)
        mats = pipe.operands(qs)
        if pipe.out is None:
            pipe.out = pipe._alloc_out(mats)
        e2 = mark("operands (transforms)", e1)
        ia, ib = pipe.order[0], pipe.order[-1]
        A, B = mats[ia], mats[ib]
        G = T.stack([_mm_nt(A, A), _mm_nt(B, B)])
        e3 = mark("grams", e2)
        TA, TB, r = be.rank_factors(G[0].contiguous(), G[1].contiguous())
        e4 = mark("qk_rank_factors", e3)
        A2, B2 = (TA @ A).contiguous(), (TB @ B).contiguous()
        e5 = mark("compressed operands", e4)
        k_eff, _ = pipe._accept(A, B, A2, B2, pipe._probes(B.shape[1], B.device), r)
        e6 = mark("probe check", e5)
        cA, cB = pipe.ops.clbits[ia], pipe.ops.clbits[ib]
        be.knit_outer_stream(A2, B2, cA, cB, pipe.N, pipe.out, k_dev=k_eff)
        e7 = mark("blocked knit", e6)
        pipe._contract(mats, skip=k_eff)
        mark("exact contraction (predicated)", e7)
    T.cuda.synchronize()
    pipe.sync_stats()
    print(f"rank {pipe.last_rank} fallbacks {pipe.rank_fallbacks} incompressible {pipe.rank_incompressible}")
    total = 0.0
    for k, v in stages.items():
        ms = sorted(s.elapsed_time(e) for s, e in v[2:])
        med = ms[len(ms) // 2]
        total += med
        print(f"{k:34s} median {med:8.3f} ms")
    print(f"{'sum':34s}        {total:8.3f} ms")


if __name__ == "__main__":
    main()
