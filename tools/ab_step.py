#!/usr/bin/env python3
"""A/B of pipeline step settings in one process, into one output buffer (small deltas need that:
the write's rate depends on the buffer).

    python tools/ab_step.py [--workload syc_32_5_p2] [--steps 20] [--rounds 3] --settings spec_write=0 spec_write=1

A setting is ``attr=value`` on the KnitPipeline (ints / floats parsed) or ``ENV:VAR=value``; settings are
timed in turn, ``--rounds`` times, each as ``--steps`` plain steps between device syncs. Prints one JSON
line per (round, setting) and a summary line with the mean per setting.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _apply(pipe, setting):
    undo = []
    for part in filter(None, setting.split(",")):
        if part.startswith("ENV:"):
            k, v = part[4:].split("=", 1)
            undo.append(("env", k, os.environ.get(k)))
            os.environ[k] = v
        else:
            k, v = part.split("=", 1)
            undo.append(("attr", k, getattr(pipe, k)))
            try:
                v = int(v)
            except ValueError:
                try:
                    v = float(v)
                except ValueError:
                    pass
            setattr(pipe, k, v)
    return undo


def _undo(pipe, undo):
    for kind, k, v in reversed(undo):
        if kind == "env":
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        else:
            setattr(pipe, k, v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--settings", nargs="+", default=["", "spec_write=1"])
    ap.add_argument("--builds", nargs="*", default=[],
                    help="one pipeline per build setting 'NAME=v' (a pipeline-module constant set before the "
                         "pipeline is built, e.g. ROW_JOBS=0); all of them write into the first one's output "
                         "buffer; each build is timed under every --settings entry")
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    torch.cuda.set_stream(torch.cuda.Stream())
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import pipeline as P

    pipes = {}
    for b in (args.builds or [""]):
        saved = {}
        for kv in filter(None, b.split(",")):
            k, v = kv.split("=", 1)
            saved[k] = getattr(P, k)
            setattr(P, k, int(v))
        pipes[b] = KnitPipeline(VirtualCircuit(cut), factored=True)
        for k, v in saved.items():
            setattr(P, k, v)
    pipe = next(iter(pipes.values()))
    for _ in range(3):
        pipe.step()
    for q in pipes.values():
        if q is not pipe:
            q.out = pipe.out  # one buffer for every build (the write's rate depends on the buffer)
            q.step()
    torch.cuda.synchronize()
    ref = pipe.out.clone()
    combos = [(b, s) for b in pipes for s in args.settings]
    acc = {c: [] for c in combos}
    for rnd in range(args.rounds):
        for b, s in combos:
            q = pipes[b]
            undo = _apply(q, s)
            q.step()  # warm the setting (streams, code paths)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                q.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            diff = float((q.out - ref).abs().max())
            _undo(q, undo)
            acc[(b, s)].append(ms)
            print(json.dumps({"round": rnd, "build": b, "setting": s, "ms_per_step": round(ms, 4),
                              "max_abs_diff": diff}), flush=True)
    for q in pipes.values():
        q.sync_stats()
    print(json.dumps({"summary": {f"{b}|{s}": round(sum(v) / len(v), 4) for (b, s), v in acc.items()},
                      "rank_fallbacks": [q.rank_fallbacks for q in pipes.values()]}), flush=True)


if __name__ == "__main__":
    main()
