#!/usr/bin/env python3
"""Write time of the bench knit by task width (QKNIT_OB_TB, read per launch) into several 32-GiB
qk_out_alloc mappings, fast and slow ones alike: does a narrower task — a compact window of
concurrently written addresses instead of ~2048 streams 512 KiB apart — write fast into the slow ones?

    python tools/out_mapping_tb.py [--buffers 5] [--tbs 16 14 12 10 9]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=5)
    ap.add_argument("--tbs", nargs="+", default=["16", "14", "12"],
                    help="task widths, or WGPC:TB pairs (QKNIT_OB_WG_PER_CU as well), optionally /SPREAD "
                         "(QKNIT_OB_SPREAD), e.g. 16/8")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    qs = pipe.sweep()
    p_ = pipe._prep_dev_rank(qs)
    torch.cuda.synchronize()
    A2, B2, k = p_["A2"], p_["B2"], p_["k_eff"]
    cA, cB = pipe.ops.clbits[pipe.order[0]], pipe.ops.clbits[pipe.order[-1]]
    N = pipe.N
    del pipe
    torch.cuda.empty_cache()
    ctx = engine.get_context(0)
    held = []
    for b in range(args.buffers):
        out, owner = engine.out_buffer(ctx, 1 << N)
        held.append((out, owner))
        rec = {"buffer": b}
        for spec in args.tbs:
            head, _, spread = spec.partition("/")
            os.environ["QKNIT_OB_SPREAD"] = spread or "1"
            wgpc, _, tb = head.rpartition(":")
            os.environ["QKNIT_OB_TB"] = tb
            if wgpc:
                os.environ["QKNIT_OB_WG_PER_CU"] = wgpc
            else:
                os.environ.pop("QKNIT_OB_WG_PER_CU", None)
            ts = []
            for _ in range(args.steps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                engine.knit_outer_stream(ctx, A2, B2, cA, cB, N, out, k_dev=k)
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            ms = [a.elapsed_time(b_) for a, b_ in ts[1:]]
            rec[spec] = round(sum(ms) / len(ms), 3)
        os.environ.pop("QKNIT_OB_TB", None)
        os.environ.pop("QKNIT_OB_SPREAD", None)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
