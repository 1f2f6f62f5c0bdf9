#!/usr/bin/env python3
"""The bench step's write kernel (qk_knit_outer_blocked_kernel, syc 32 5) timed with HIP events next
to a plain torch fill of the same 2^32-entry buffer, in one process: the write's distance from what a
store-only kernel reaches on this box. Select a tuning build with QKNIT_LIB.

    QKNIT_LIB=tools/variants/lib_X.so python tools/write_bench.py --steps 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--fill", action="store_true", help="also time torch's zero_ on the output buffer")
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    torch.cuda.set_stream(torch.cuda.Stream())
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    for _ in range(2):
        pipe.step()
    torch.cuda.synchronize()
    pipe.record_events = True
    pipe.events.clear()
    for _ in range(args.steps):
        pipe.step()
    torch.cuda.synchronize()
    w = [s.elapsed_time(e) for s, e in pipe.events]
    rec = {"lib": os.path.basename(os.environ.get("QKNIT_LIB", "default")), "write_ms": sum(w) / len(w),
           "write_min_ms": min(w)}
    if args.fill:
        out = pipe.out
        out.zero_()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            out.zero_()
        e.record()
        torch.cuda.synchronize()
        rec["torch_fill_ms"] = s.elapsed_time(e) / 3
    rec["GBs"] = 34.36e9 / (rec["write_ms"] * 1e-3) / 1e9
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
