#!/usr/bin/env python3
"""A/B of the output-write-bound knit (syc 32 1: 65536 x 65536 outer product, 34 GB written):
qk_gemm_smallk_kernel (K = 1) against the LDS-DMA MFMA kernel on the same operands zero-padded
to K = 16, interleaved in one process (MI355X_MICROARCH.md: compare on one device)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(0)
    M = N = 1 << 16
    g = torch.Generator(device="cuda").manual_seed(0)
    A1 = torch.rand(1, M, dtype=torch.float64, device="cuda", generator=g)
    B1 = torch.rand(1, N, dtype=torch.float64, device="cuda", generator=g)
    A16 = torch.zeros(16, M, dtype=torch.float64, device="cuda")
    B16 = torch.zeros(16, N, dtype=torch.float64, device="cuda")
    A16[0], B16[0] = A1[0], B1[0]
    out = torch.empty(M * N, dtype=torch.float64, device="cuda")
    ways = {"smallk K=1": (A1, B1), "glds K=16 (zero-padded)": (A16, B16)}
    times = {k: [] for k in ways}
    for rep in range(6):
        for k, (A, B) in ways.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            engine.gemm_keyed(ctx, A, B, out=out, strideA=N)
            e.record()
            torch.cuda.synchronize()
            if rep:
                times[k].append(s.elapsed_time(e))
    for k, t in times.items():
        t = sorted(t)
        print(f"{k:26s} median {t[len(t) // 2]:.3f} ms = {8 * M * N / t[len(t) // 2] / 1e9:.2f} TB/s", flush=True)
