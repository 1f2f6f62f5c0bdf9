#!/usr/bin/env python3
"""The syc 32 5 knit contraction shape (65536 x 65536 x 256, fp64, random operands): the LDS-DMA
MFMA kernel (qk_gemm_keyed) against the vendor library GEMM torch dispatches to (rocBLAS /
hipBLASLt dgemm), interleaved in one process, HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(0)
    M = N = 1 << 16
    K = 256
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(K, M, dtype=torch.float64, device="cuda", generator=g)
    B = torch.randn(K, N, dtype=torch.float64, device="cuda", generator=g)
    out = torch.empty(M * N, dtype=torch.float64, device="cuda")
    ways = {
        "qk_gemm_keyed (LDS-DMA MFMA)": lambda: engine.gemm_keyed(ctx, A, B, out=out, strideA=N),
        "torch.mm -> vendor dgemm": lambda: torch.mm(A.t(), B, out=out.view(M, N)),
    }
    times = {k: [] for k in ways}
    for rep in range(4):
        for k, fn in ways.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            if rep:
                times[k].append(s.elapsed_time(e))
    for k, t in times.items():
        t = sorted(t)
        ms = t[len(t) // 2]
        print(f"{k:32s} median {ms:.2f} ms = {2 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)
    ref = torch.mm(A.t()[:512], B[:, :512])
    engine.gemm_keyed(ctx, A, B, out=out, strideA=N)
    print("max |ours - torch| on a 512x512 block:", float((out.view(M, N)[:512, :512] - ref).abs().max()))
