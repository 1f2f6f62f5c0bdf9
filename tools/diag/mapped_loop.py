"""Loop the mapped-output drop-in sequence (take_out -> run_into -> .cpu()) on cx_8x8 and count
wrong results, to chase the one-off 75%-zeros failure of test_mapped_output_buffer_steps_match_oracle."""
import os, sys, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import torch
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, engine, cutting
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline
import circuits
from oracle import dense

mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
if "--big" in sys.argv:  # a 2^32 step first, as the suite's previous test
    _, cut, _ = cutting.config_cut_circuit("syc", 32, 5, 2)
    big = KnitPipeline(VirtualCircuit(cut), factored=True)
    big.step(); torch.cuda.synchronize(); del big
engine.OUT_MAPPED_MIN_BYTES = 0
cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
ref = dense.run_dense(cut)
for _ in range(2):
    pipe.step().cpu()
pipe.sync_stats()
print("kernel", pipe.last_kernel, "covers", pipe.covers_outputs(), "rank", pipe.last_rank, flush=True)
bad_runs = 0
for it in range(60):
    first = pipe.take_out()
    pipe.run_into(first)
    if mode == "sync":
        torch.cuda.synchronize()
    got = first.cpu().numpy()
    bad = np.flatnonzero(np.abs(got - ref) > 1e-12)
    if bad.size:
        bad_runs += 1
        z = np.count_nonzero(got[bad] == 0)
        tiles = np.bincount((bad >> 15) * 2 + ((bad & 255) >> 7), minlength=4)
        pipe.sync_stats()
        print(f"it {it}: {bad.size} wrong [{bad[0]}, {bad[-1]}], zeros {z}, per 128x128 tile {tiles.tolist()}, "
              f"rank {pipe.last_rank}, ptr {first.data_ptr():#x}", flush=True)
    if it % 3 == 0:
        keep = first  # sometimes hold the previous result (a new mapping next time)
    del first
print(f"mode {mode}: {bad_runs} of 60 runs wrong", flush=True)
