#!/usr/bin/env python3
"""Time the knit contraction (qk_gemm_keyed) alone on the syc 32 5 operands.

  python tools/gemm_bench.py [--factored] [--reps 5]
Prints TF/s per launch (HIP events on the launch stream).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--factored", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--synthetic", type=int, nargs=3, metavar=("M", "N", "K"),
                    help="random operands of this shape, output out[i*N + j] (no circuit)")
    ap.add_argument("--deposit", action="store_true",
                    help="synthetic: scatter through syc-like interleaved deposit keys (M = N = 2^16)")
    args = ap.parse_args()
    import torch

    if args.synthetic:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

        M, N, K = args.synthetic
        ctx = engine.get_context(0)
        A = torch.randn(K, M, dtype=torch.float64, device="cuda")
        B = torch.randn(K, N, dtype=torch.float64, device="cuda")
        out = torch.empty(M * N, dtype=torch.float64, device="cuda")
        kw = dict(strideA=N, strideB=1)
        if args.deposit:
            from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys

            bits_b = [r * 8 + c for r in range(4) for c in range(4)]
            bits_a = [r * 8 + 4 + c for r in range(4) for c in range(4)]
            kw = dict(keyA=torch.from_numpy(deposit_keys(bits_a)).cuda(),
                      keyB=torch.from_numpy(deposit_keys(bits_b)).cuda())
        for r in range(args.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            engine.gemm_keyed(ctx, A, B, out=out, **kw)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e)
            print(f"rep {r}: M={M} N={N} K={K} {ms:.3f} ms  {2.0 * M * N * K / ms / 1e9:.2f} TF/s", flush=True)
        return

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    pipe = KnitPipeline(VirtualCircuit(cut), factored=args.factored)
    qs = pipe.sweep()
    mats = pipe.operands(qs)
    pipe.out = pipe._alloc_out(mats)
    M, N, K = pipe.gemm_shape()
    flops = 2.0 * M * N * K
    for r in range(args.reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        pipe._contract(mats)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        print(f"rep {r}: M={M} N={N} K={K} {ms:.3f} ms  {flops / ms / 1e9:.2f} TF/s", flush=True)


if __name__ == "__main__":
    main()
