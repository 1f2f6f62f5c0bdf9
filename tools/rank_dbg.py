#!/usr/bin/env python3
"""Phase clocks of qk_rank_factors on the syc 32 5 Grams (QK_RANK_DEBUG variant build:
QKNIT_LIB=tools/variants/lib_rankdbg.so). Prints cholesky / core+Jacobi / rank+factors microseconds
(wall_clock64 at 100 MHz), the Jacobi sweep count and the pivot counts."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, _lib, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    _, cut, _ = cutting.config_cut_circuit("syc", 32, 5, 2)
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    qs = pipe.sweep()
    ia, ib = pipe.order[0], pipe.order[-1]
    mats, G, U = pipe._prep_fused(qs, pipe._probes(qs[ib].shape[1], qs[ib].device))
    lib = _lib.lib()
    out = (ctypes.c_longlong * 8)()
    for _ in range(3):
        pipe.be.rank_factors(G[0], G[1])
        torch.cuda.synchronize()
        lib.qk_rank_debug(out)
        t = [out[i] for i in range(4)]
        print({"gram_load_us": (out[4] - t[0]) / 100, "cholesky_us": (t[1] - t[0]) / 100, "jacobi_us": (t[2] - t[1]) / 100, "factors_us": (t[3] - t[2]) / 100,
               "sweeps": out[5], "ra": out[6], "rb": out[7]}, flush=True)


if __name__ == "__main__":
    main()
