#!/usr/bin/env python3
"""Does the output buffer (its allocation, hence its physical pages) change the write time of the
bench step? Times KnitPipeline steps of syc 32 5 into the pipeline's own buffer and into freshly
allocated ones, with HIP events around the write kernel (pipe.events) and wall time per step.

    python tools/out_buffer_probe.py --steps 8
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    torch.cuda.set_stream(torch.cuda.Stream())
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    own = pipe.out

    def run(tag, buf, events=True):
        if buf is not None:
            pipe.out = buf
        pipe.step()
        torch.cuda.synchronize()
        pipe.record_events = events
        pipe.events.clear()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe.step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        w = [s.elapsed_time(e) for s, e in pipe.events]
        rec = {"tag": tag, "wall_ms": round(wall, 4),
               "write_ms": round(sum(w) / len(w), 4) if w else None,
               "write_min_ms": round(min(w), 4) if w else None,
               "ptr": hex(pipe.out.data_ptr())}
        print(json.dumps(rec), flush=True)

    run("own buffer (be.zeros at construction)", None)
    run("own buffer, no events", None, events=False)
    b1 = torch.empty(1 << 32, dtype=torch.float64, device="cuda")
    run("fresh torch.empty #1", b1)
    b2 = torch.empty(1 << 32, dtype=torch.float64, device="cuda")
    run("fresh torch.empty #2", b2)
    run("own buffer again", own)
    del b1
    b3 = torch.zeros(1 << 32, dtype=torch.float64, device="cuda")
    run("fresh torch.zeros #3 (after freeing #1)", b3)
    run("fresh #2 again", b2)


if __name__ == "__main__":
    main()
