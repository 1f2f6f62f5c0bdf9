#!/usr/bin/env python3
"""Time qk_prep_operands alone on syc 32 5's shapes (random operands): K = 64, RA + RB instance rows
(argv: RA RB, default 65 65 — the swept rows after pruning; round 3 used 256 64), 2 x 65536 columns.
Select a tuning build with QKNIT_LIB. Prints mean us per call and MFMA TF/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    RA, RB = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (65, 65)
    K, N = 64, 65536
    WtA, WtB = (torch.randn(R, K, dtype=torch.float64, device="cuda", generator=g) for R in (RA, RB))
    qA, qB = (torch.randn(R, N, dtype=torch.float64, device="cuda", generator=g) for R in (RA, RB))
    P = torch.randn(16, N, dtype=torch.float64, device="cuda", generator=g)
    out = engine.prep_operands(ctx, WtA, qA, WtB, qB, P)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    s.record()
    for _ in range(reps):
        engine.prep_operands(ctx, WtA, qA, WtB, qB, P, out=out)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    flops = 2.0 * K * N * (RA + RB) + 2 * 2.0 * K * K * N + 2.0 * K * 16 * N
    print(json.dumps({"lib": os.environ.get("QKNIT_LIB", "default"), "rows": [RA, RB], "us": us, "TFs": flops / (us * 1e-6) / 1e12}),
          flush=True)


if __name__ == "__main__":
    main()
