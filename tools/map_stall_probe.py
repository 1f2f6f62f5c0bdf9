#!/usr/bin/env python3
"""How long a 34-GB qk_out_alloc mapping (and a plain torch allocation) takes to make right after
large frees, after a pause, and with nothing freed — the drop-in's multi-second re-selection calls
(r06i bench: 3157 ms; tools/reselect_probe.py: one candidate's mapping 4360 ms) against the hypothesis
that the device clears released memory before handing it out again.

    python tools/map_stall_probe.py [--gib 32]

Prints one JSON line: per step the host ms of the allocation, the free device memory before it.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=32)
    ap.add_argument("--pause", type=float, default=5.0)
    ap.add_argument("--seq", type=int, default=0,
                    help="instead: make SEQ mappings one after another (all held, each filled), time each, exit "
                         "holding them (run twice back to back: the second process maps right after the first "
                         "one's teardown)")
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(0)
    n = (args.gib << 30) // 8
    steps = []

    def mapped(tag):
        free = torch.cuda.mem_get_info()[0]
        t = time.perf_counter()
        m = engine.MappedOut(ctx, n)
        ms = (time.perf_counter() - t) * 1e3
        x = m.tensor()
        t = time.perf_counter()
        x.fill_(1.0)
        torch.cuda.synchronize()
        steps.append({"step": tag, "kind": "mapped", "alloc_ms": round(ms, 2), "fill_ms": round((time.perf_counter() - t) * 1e3, 2),
                      "free_GiB_before": round(free / 2**30, 1)})
        del x
        return m

    def plain(tag):
        free = torch.cuda.mem_get_info()[0]
        t = time.perf_counter()
        x = torch.empty(n, dtype=torch.float64, device="cuda")
        ms = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        x.fill_(1.0)
        torch.cuda.synchronize()
        steps.append({"step": tag, "kind": "torch", "alloc_ms": round(ms, 2), "fill_ms": round((time.perf_counter() - t) * 1e3, 2),
                      "free_GiB_before": round(free / 2**30, 1)})
        return x

    if args.seq:
        held = [mapped(f"seq {i}") for i in range(args.seq)]
        print(json.dumps({"gib": args.gib, "seq": args.seq, "t_exit": time.time(), "steps": steps}), flush=True)
        del held
        return
    a = mapped("first")
    b = mapped("second, nothing freed")
    del a
    c = mapped("right after freeing one")
    del b, c
    d = mapped("right after freeing two")
    del d
    time.sleep(args.pause)
    e = mapped(f"after {args.pause:.0f} s pause")
    f = mapped("nothing freed since")
    del e, f
    x = plain("torch, right after freeing two mappings")
    del x
    torch.cuda.empty_cache()
    y = plain("torch, right after releasing one")
    del y
    torch.cuda.empty_cache()
    time.sleep(args.pause)
    z = plain(f"torch, after {args.pause:.0f} s pause")
    del z
    torch.cuda.empty_cache()
    print(json.dumps({"gib": args.gib, "steps": steps, "out_stats": engine.out_stats()}), flush=True)


if __name__ == "__main__":
    main()
