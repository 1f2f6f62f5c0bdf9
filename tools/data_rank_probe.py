#!/usr/bin/env python3
"""Time the pieces of one syc 32 5 knit step with data-rank compression (HIP events + syncs)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref")[1]
pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
for _ in range(2):
    pipe.step()
torch.cuda.synchronize()


def timed(name, f):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    print(f"{name:28s} {1e3 * (time.perf_counter() - t):8.3f} ms", flush=True)
    return r


for rep in range(3):
    qs = timed("sweep", pipe.sweep)
    mats = timed("operands", lambda: pipe.operands(qs))
    low = timed("rank_compress", lambda: pipe._rank_compress(mats))
    timed("contract_lowrank", lambda: pipe._contract_lowrank(low[0]))
    timed("check readback", lambda: float(low[1]))
    timed("full step", pipe.step)
print("rank", pipe.last_rank, "fallbacks", pipe.rank_fallbacks)
