#!/usr/bin/env python3
"""Pipelined steps (KnitPipeline._step_overlapped) against plain steps, per preparation CU count.

  python tools/overlap_bench.py [--workload syc_32_5_p2] [--steps 20] [--prep-cus 0 16 32 48 64]

One pipeline; per setting: warm-up, then ``--steps`` steps timed between device syncs (ms per step,
throughput form) and the output of the last step compared with the plain step's (max |diff|).
``--prep-cus 0``: pipelined on a plain side stream (no CU split). Prints one JSON line per setting.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--prep-cus", type=int, nargs="*", default=[32, 48, 64, 0])
    ap.add_argument("--layouts", nargs="*", default=["block"])
    ap.add_argument("--prio", nargs="*", default=[""], help="QKNIT_OVERLAP_PRIO values for --prep-cus 0 ('', write, prep)")
    ap.add_argument("--no-final-plain", action="store_true", help="end with the pipelined runs (timelines)")
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    torch.cuda.set_stream(torch.cuda.Stream())  # pipelined steps need a non-default stream
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    host = {}

    def wrap(name):  # host time spent inside a pipeline phase (a blocking call shows up here)
        fn = getattr(pipe, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            host[name] = host.get(name, 0.0) + time.perf_counter() - t0
            return r

        setattr(pipe, name, w)

    for nm in ("sweep", "_prep_dev_rank", "_launch_dev_rank"):
        wrap(nm)

    def stats():
        ev = lambda L: sum(a.elapsed_time(b) for a, b in L) / max(len(L), 1)  # noqa: E731
        return {"write_ms": ev(pipe.events), "sweep_ms": ev(pipe.sweep_events), "prep_after_sweep_ms": ev(pipe.prep_events)}

    def run(k, timed=False):
        pipe.events.clear()
        pipe.sweep_events.clear()
        pipe.prep_events.clear()
        pipe.record_events = timed
        host.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            pipe.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / k * 1e3
        for nm in list(host):
            host[nm] = host[nm] / k * 1e3
        return ms

    pipe.overlap = False
    run(3)
    plain = run(args.steps)
    ref = pipe.out.clone()
    run(5, timed=True)
    print(json.dumps({"setting": "plain", "ms_per_step": plain, **stats()}), flush=True)
    settings = [(c, lay, pr) for c in args.prep_cus for lay in (args.layouts if c else ["-"])
                for pr in (args.prio if c == 0 else [""])]
    for c, lay, pr in settings:
        os.environ["QKNIT_OVERLAP_PRIO"] = pr
        os.environ["QKNIT_PREP_CUS"] = str(c)
        os.environ["QKNIT_PREP_CU_LAYOUT"] = lay
        pipe._prep_stream = pipe._write_stream = None
        pipe.overlap = True
        pipe.out.fill_(float("nan"))
        run(3)
        ms = run(args.steps)
        host_ms = dict(host)
        diff = float((pipe.out - ref).abs().max())
        run(5, timed=True)
        pipe.sync_stats()
        print(json.dumps({"setting": "pipelined", "prep_cus": c, "layout": lay, "prio": pr, "cus": pipe.overlap_cus, "ms_per_step": ms,
                          "max_abs_diff_vs_plain": diff, "rank_fallbacks": pipe.rank_fallbacks, "host_ms": host_ms, **stats()}),
              flush=True)
    if not args.no_final_plain:
        pipe.overlap = False
        print(json.dumps({"setting": "plain (again)", "ms_per_step": run(args.steps)}), flush=True)


if __name__ == "__main__":
    main()
