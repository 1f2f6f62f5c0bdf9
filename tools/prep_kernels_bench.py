#!/usr/bin/env python3
"""Time the data-rank preparation's small kernels alone (syc 32 5 shapes, random operands): compress,
probe errors (V partials + d + accept), rank factors on a rank-2 Gram pair. Compare with their
in-step times in a bench kernel trace (profiles/*bench_kernel_trace.txt) to separate a kernel's own
cost from interference with its neighbours in the step.

    python tools/prep_kernels_bench.py [--n 65536] [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    K, N, R = 64, args.n, 8
    XA, XB = (torch.randn(K, N, dtype=torch.float64, device="cuda", generator=g) for _ in range(2))
    TA, TB = (torch.randn(R, K, dtype=torch.float64, device="cuda", generator=g) for _ in range(2))
    P = torch.randn(16, N, dtype=torch.float64, device="cuda", generator=g)
    U = XB @ P.T
    low = torch.randn(K, 2, dtype=torch.float64, device="cuda", generator=g)
    GA = (low @ low.T).contiguous()
    GB = GA.clone()
    r = torch.full((1,), 2, dtype=torch.int32, device="cuda")

    def timed(name, fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"{name:28s} {s.elapsed_time(e) / args.reps * 1e3:8.1f} us per call", flush=True)

    A2, B2 = engine.compress_operands(ctx, TA, XA, TB, XB)
    timed("compress_operands", lambda: engine.compress_operands(ctx, TA, XA, TB, XB))
    timed("probe_errors (v, d, accept)", lambda: engine.probe_errors(ctx, XA, A2, U, B2, P, r=r, tol=1e-14))
    timed("rank_factors", lambda: engine.rank_factors_device(ctx, GA, GB))
    # the same compress on a non-power-of-two row length (row stride N + 64 doubles): a much lower
    # time per byte would point at HBM channel camping of the 2^19-byte row stride
    XAp, XBp = (torch.randn(K, N + 64, dtype=torch.float64, device="cuda", generator=g) for _ in range(2))
    timed("compress_operands N+64", lambda: engine.compress_operands(ctx, TA, XAp, TB, XBp))
    XAq, XBq = (torch.randn(K, N + 512, dtype=torch.float64, device="cuda", generator=g) for _ in range(2))
    timed("compress_operands N+512", lambda: engine.compress_operands(ctx, TA, XAq, TB, XBq))
    XAh, XBh = (torch.randn(K, N // 2, dtype=torch.float64, device="cuda", generator=g) for _ in range(2))
    timed("compress_operands N/2", lambda: engine.compress_operands(ctx, TA, XAh, TB, XBh))
    z = torch.zeros(1, dtype=torch.float64, device="cuda")
    timed("torch add_ (1 element)", lambda: z.add_(1.0))


if __name__ == "__main__":
    main()


def read_patterns(reps: int = 20):
    """How fast can the [64, 2^16] operand be read at all? Sequential full-buffer reduction, the torch
    (hipBLASLt) T @ X product the compress kernel computes, and a column-sum over the rows."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(64, 65536, dtype=torch.float64, device="cuda", generator=g)
    T = torch.randn(8, 64, dtype=torch.float64, device="cuda", generator=g)
    for name, fn in (("X.sum() (sequential 32 MB)", lambda: X.sum()),
                     ("X.sum(dim=0) (column sums)", lambda: X.sum(dim=0)),
                     ("torch.mm(T, X) [8,64]x[64,2^16]", lambda: torch.mm(T, X))):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        print(f"{name:34s} {us:8.1f} us per call ({32 * 2**20 / us / 1e6:.2f} TB/s)", flush=True)


if __name__ == "__main__" and os.environ.get("QK_READ_PATTERNS"):
    read_patterns()
