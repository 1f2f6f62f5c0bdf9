#!/usr/bin/env python3
"""Phase clocks of qk_rank_factors on the syc 32 5 Grams (QK_RANK_DEBUG variant build:
QKNIT_LIB=tools/variants/lib_rankdbg.so). Prints the phase times in microseconds
(wall_clock64 at 100 MHz: Gram load, pivoted Cholesky, core, LU, factors) and the pivot counts."""
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
        s0, s1, s2, s3, s4, s5 = (out[i] for i in range(6))  # RK_STAMP(i): 0 start, 4 Grams loaded,
        # 1 Cholesky done, 2 core done, 5 LU done, 3 end (wall_clock64 at 100 MHz)
        print({"gram_load_us": (s4 - s0) / 100, "cholesky_us": (s1 - s4) / 100, "core_us": (s2 - s1) / 100,
               "lu_us": (s5 - s2) / 100, "factors_us": (s3 - s5) / 100, "total_us": (s3 - s0) / 100,
               "ra": out[6], "rb": out[7]}, flush=True)

if __name__ == "__main__":
    main()
