#!/usr/bin/env python3
"""The slice-mode write alone: qk_knit_outer_stream over [r 2^N / P, (r + 1) 2^N / P) of syc 32 5's
compressed operands (taken from a one-GPU step) into a 2^N / P buffer, for P = 1, 2, 4, 8, on all
CUs and on a 160-CU masked stream (the pipelined multi-GPU write), HIP events per launch.

    python tools/slice_write_bench.py [--steps 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--streams", nargs="+", default=["all", "masked160"])
    ap.add_argument("--where", nargs="+", default=["last"],
                    help="last: the last slice into its own mapping; first: the first slice; "
                         "inbig: the first slice into the first part of a full-size mapping")
    ap.add_argument("--env-sets", nargs="+", default=[""],
                    help="A/B settings timed into the same buffer in turn, each 'VAR=v;VAR=v' (read per launch)")
    ap.add_argument("--rounds", type=int, default=1, help="passes over --env-sets per buffer")
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
    ia, ib = pipe.order[0], pipe.order[-1]
    cA, cB = pipe.ops.clbits[ia], pipe.ops.clbits[ib]
    N = pipe.N
    del pipe
    torch.cuda.empty_cache()
    ctx = engine.get_context(0)
    total = torch.cuda.get_device_properties(0).multi_processor_count
    for streams in args.streams:
        if streams == "all":
            s = torch.cuda.Stream()
        else:
            s = engine.cu_masked_stream(0, tuple(range(total - 96)))  # the write CUs of a 96-CU prep split
        with torch.cuda.stream(s):
            ctx.bind_stream()
            big = None
            for P, where in [(P, w) for P in args.worlds for w in args.where]:
                n_out = (1 << N) // P
                if where == "inbig":
                    if big is None:
                        big = engine.out_buffer(ctx, 1 << N)
                    out, owner = big[0][:n_out], None
                else:
                    out, owner = engine.out_buffer(ctx, n_out)
                o_begin = (P - 1) * n_out if where == "last" else 0
                for rnd in range(args.rounds):
                    for es in args.env_sets:
                        saved = {}
                        for kv in filter(None, es.split(";")):
                            kk, vv = kv.split("=", 1)
                            saved[kk] = os.environ.get(kk)
                            os.environ[kk] = vv
                        ts = []
                        for it in range(args.steps + 2):
                            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            a.record()
                            engine.knit_outer_stream(ctx, A2, B2, cA, cB, N, out, o_begin=o_begin, o_count=n_out,
                                                     k_dev=k)
                            b.record()
                            ts.append((a, b))
                        torch.cuda.synchronize()
                        for kk, vv in saved.items():
                            if vv is None:
                                os.environ.pop(kk, None)
                            else:
                                os.environ[kk] = vv
                        ms = [a.elapsed_time(b) for a, b in ts[2:]]
                        avg = sum(ms) / len(ms)
                        q = len(ms) // 4 or 1
                        trend = [round(sum(ms[i:i + q]) / len(ms[i:i + q]), 4) for i in range(0, len(ms), q)][:4]
                        print(json.dumps({"streams": streams, "world": P, "where": where, "env": es, "round": rnd,
                                          "wg_per_cu": os.environ.get("QKNIT_OB_WG_PER_CU", "64"), "write_ms": round(avg, 4),
                                          "GBs": round(8 * n_out / avg / 1e6, 1), "min_ms": round(min(ms), 4),
                                          "quarters_ms": trend}), flush=True)
                del out, owner
        ctx.bind_stream()


if __name__ == "__main__":
    main()
