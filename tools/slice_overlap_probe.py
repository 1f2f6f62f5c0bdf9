#!/usr/bin/env python3
"""Aggregate HBM rate of back-to-back slice writes (syc 32 5's compressed operands, a rank's 2^N / P
outputs, qk_knit_outer_stream_range) into rotating buffers: on one stream (each launch waits for the
last: its ramp and drain are exposed) against 2-3 streams (launches overlap, as the pipelined 8-rank
step's writes do), on every CU and on the 128 write CUs of the 8-rank CU split. Separates a per-launch
cost that overlap hides from a rate limit it does not.

    python tools/slice_overlap_probe.py [--world 8] [--launches 30]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--modes", nargs="+", default=["serial_all", "rot2_all", "rot3_all", "serial_w128", "rot3_w128"],
                    help="..._w128 modes may end in +empty (10 tiny kernels per write on a stream over the other "
                         "128 CUs: kernel boundaries alone) or +chain (the step's real sweep + preparation chain there)")
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
    chain_pipe = pipe  # kept for +chain modes (its sweep and preparation re-run beside the writes)
    del qs
    torch.cuda.empty_cache()
    ctx = engine.get_context(0)
    total = engine.device_cu_count(0)
    n_out = (1 << N) // args.world
    bufs = [engine.out_buffer(ctx, n_out) for _ in range(3)]
    write_cus = tuple(range(total - 128))

    prep_cus = tuple(range(total - 128, total))
    side = engine.cu_masked_stream(0, prep_cus, tag=400)
    tiny = torch.zeros(64, dtype=torch.float64, device="cuda")

    def side_work(kind):
        with torch.cuda.stream(side):
            if kind == "empty":
                for _ in range(10):
                    tiny.add_(1.0)
            elif kind == "chain":
                chain_pipe.be.bind()
                q = chain_pipe.sweep()
                chain_pipe._prep_dev_rank(q)
        ctx.bind_stream()

    def streams(mode):
        mode = mode.split("+")[0]
        nb = 1 if mode.startswith("serial") else int(mode[3])
        if mode.endswith("_all"):
            return [torch.cuda.Stream() for _ in range(nb)]
        return [engine.cu_masked_stream(0, write_cus, tag=200 + t) for t in range(nb)]

    res = {"world": args.world, "n_out": n_out, "GB_per_launch": 8 * n_out / 1e9, "selections": engine.out_selections,
           "modes": {}}
    main_s = torch.cuda.current_stream()
    for rnd in range(args.rounds):
        for mode in args.modes:
            ss = streams(mode)
            for s in ss:
                s.wait_stream(main_s)
            torch.cuda.synchronize()
            for warm in (True, False):
                cnt = 3 if warm else args.launches
                t0 = time.perf_counter()
                extra = mode.split("+")[1] if "+" in mode else None
                for i in range(cnt):
                    if extra:
                        side_work(extra)
                    s = ss[i % len(ss)]
                    with torch.cuda.stream(s):
                        ctx.bind_stream()
                        # the buffer's previous writer is the launch 3 back: on another stream when nb < 3 —
                        # writes of the same values, no ordering needed for a rate measurement
                        engine.knit_outer_stream(ctx, A2, B2, cA, cB, N, bufs[i % 3][0], o_begin=0, o_count=n_out,
                                                 k_dev=k)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            ms = dt / args.launches * 1e3
            res["modes"].setdefault(mode, []).append({"ms_per_launch": round(ms, 4),
                                                      "GBs": round(8 * n_out / (ms * 1e-3) / 1e9, 1)})
    ctx.bind_stream()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
