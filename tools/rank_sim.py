#!/usr/bin/env python3
"""One rank's device work of the multi-GPU bench (slice mode), on one GPU, without RCCL.

The driver runs ``bench.py --gpus 8``; a gpurun box has one GPU. Here rank ``r`` of ``world`` ranks
is built exactly as bench.py builds it (syc 32 5, factored knit, ``slice`` mode: the rank owns the
contiguous outputs ``[r, r + 1) * 2^32 / world``); only ``torch.distributed`` is replaced by local
stand-ins that move the same bytes on the device (all_to_all / all_gather: copies into the same
receive buffers; all_reduce / broadcast: no-ops on the rank's own partial values), so the step
times everything a rank computes — its sweep shard, its operand column blocks, the Grams, the
device factorisation, the probe check, its slice of the write — but not the xGMI transfers. The
bytes each collective would receive are printed beside it, so the predicted N-GPU step is
``ms_per_step_no_xgmi + received bytes / xGMI bandwidth``. The probe tolerance is
lifted (the stand-in all_reduce leaves partial Grams, whose factors need not pass the real check);
the accepted rank is reported. The factorisation runs on the true Grams (from a one-GPU step):
the partial ones would factor to a different rank.

    python tools/rank_sim.py --world 2 4 8 --steps 5 [--xgmi-gbs 50 --coll-lat-us 20] [--overlap]

``--xgmi-gbs B``: every stand-in collective also holds its stream for ``lat + received / (links x B)``
(torch.cuda._sleep, calibrated; ``links`` = world - 1 <= 7: fully connected xGMI, each peer's share
on its own link), a model of the transfer time on the rank's timeline. ``--overlap``: pipelined
steps (KnitPipeline._step_overlapped: step i+1's sweep, preparation and collectives on a CU-masked
stream under step i's write), the default of the multi-GPU bench.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Done:
    def wait(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--xgmi-gbs", type=float, default=0.0, help="modelled per-link xGMI GB/s (0: no delay)")
    ap.add_argument("--coll-lat-us", type=float, default=20.0, help="modelled latency per collective")
    ap.add_argument("--overlap", action="store_true", help="pipelined steps (CU-masked prep stream)")
    ap.add_argument("--prep", default="auto", choices=["auto", "replicated", "sharded"],
                    help="slice-mode preparation (QKNIT_SLICE_PREP): replicated = no collective at all")
    ap.add_argument("--cprofile", action="store_true", help="cProfile the timed steps (top host functions to stderr)")
    ap.add_argument("--no-world-sync", action="store_true",
                    help="between worlds only `del pipe` (no gc.collect / synchronize / empty_cache): the "
                         "sequence of round 5's faulting run (profiles/r05bb_*)")
    ap.add_argument("--host-profile", action="store_true",
                    help="host time per pipeline phase (sweep / preparation / launch), to find blocking calls")
    args = ap.parse_args()
    os.environ["QKNIT_SLICE_PREP"] = args.prep
    import torch
    import torch.distributed as dist

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, variant = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, variant)
    recv = {}
    cyc_per_us = [0.0]
    if args.xgmi_gbs > 0:  # calibrate torch.cuda._sleep (cycles of the shader clock) against events
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000000)
        s_.record()
        torch.cuda._sleep(2000000)
        e_.record()
        torch.cuda.synchronize()
        cyc_per_us[0] = 2000000 / (s_.elapsed_time(e_) * 1e3)

    def note(kind, nbytes):
        recv[kind] = recv.get(kind, 0) + nbytes
        if args.xgmi_gbs > 0:  # the modelled transfer holds the issuing stream
            links = max(1, min(world_now[0] - 1, 7))
            us = args.coll_lat_us + nbytes / (links * args.xgmi_gbs * 1e9) * 1e6
            torch.cuda._sleep(int(us * cyc_per_us[0]))
            model[kind] = model.get(kind, 0.0) + us

    def all_to_all_single(out, inp, group=None, async_op=False):
        out.view(-1).copy_(inp.reshape(-1))
        P = world_now[0]
        note("all_to_all", out.numel() * out.element_size() * (P - 1) // P)
        return _Done() if async_op else None

    def all_reduce(t, op=None, group=None, async_op=False):
        P = world_now[0]
        note("all_reduce", 2 * t.numel() * t.element_size() * (P - 1) // P)
        return _Done() if async_op else None

    def broadcast(t, src=0, group=None, async_op=False):
        note("broadcast", t.numel() * t.element_size())
        return _Done() if async_op else None

    side = []

    class _Pending:
        """An async stand-in collective: ran on a side stream; wait() makes the current stream wait."""

        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        P = world_now[0]
        if not async_op:
            out.view(P, -1).copy_(inp.reshape(1, -1).expand(P, -1))
            note("all_gather", out.numel() * out.element_size() * (P - 1) // P)
            return None
        if not side:
            side.append(torch.cuda.Stream())
        s = side[0]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # the transfer (copy + modelled xGMI time) off the issuing stream
            out.view(P, -1).copy_(inp.reshape(1, -1).expand(P, -1))
            note("all_gather_async", out.numel() * out.element_size() * (P - 1) // P)
            ev = torch.cuda.Event()
            ev.record(s)
        return _Pending(ev)

    dist.all_to_all_single = all_to_all_single
    dist.all_reduce = all_reduce
    dist.broadcast = broadcast
    dist.all_gather_into_tensor = all_gather_into_tensor
    dist.get_global_rank = lambda group, r: r
    world_now = [1]
    model = {}

    # the stand-in all_reduce leaves each rank's partial Grams; factorise the TRUE Grams instead (taken
    # from a one-GPU step) so the simulated rank compresses to the real rank, with the same kernel
    one = KnitPipeline(VirtualCircuit(cut), factored=True)
    mats = one.operands(one.sweep())  # (the replicated preparation factors its own, true, Grams)
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import _mm_nt

    A, B = mats[one.order[0]], mats[one.order[-1]]
    G_true = (_mm_nt(A, A).contiguous(), _mm_nt(B, B).contiguous())
    del one, mats, A, B
    torch.cuda.empty_cache()

    for world in args.world:
        world_now[0] = world
        pipe = KnitPipeline(VirtualCircuit(cut), factored=True, rank=args.rank, world=world, mode="slice")
        if pipe.sharded:  # partial Grams from the stand-in all_reduce: factor the true ones, no check
            real = pipe.be.rank_factors
            pipe.be.rank_factors = lambda GA, GB, real=real: real(*G_true)
            pipe.rank_tol = float("inf")
        if args.overlap:
            torch.cuda.set_stream(torch.cuda.Stream())
            pipe.overlap = pipe.overlap_ok()
        host_phase = {}
        if args.host_profile:
            import functools

            for name in ("sweep", "_prep_slice", "_launch_slice", "_slice_exact_operands", "_prep_fused",
                         "_exchange", "_fold"):
                fn = getattr(pipe, name)

                @functools.wraps(fn)
                def timed(*a, _fn=fn, _name=name, **kw):
                    h = time.perf_counter()
                    try:
                        return _fn(*a, **kw)
                    finally:
                        host_phase[_name] = host_phase.get(_name, 0.0) + time.perf_counter() - h

                setattr(pipe, name, timed)
        for _ in range(args.warmup):
            pipe.step()
        torch.cuda.synchronize()
        recv.clear()
        model.clear()
        host_phase.clear()
        pipe.record_events = True
        t0 = time.perf_counter()
        host = 0.0
        prof = None
        if args.cprofile:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        for _ in range(args.steps):
            h0 = time.perf_counter()
            pipe.step()
            host += time.perf_counter() - h0
        if prof is not None:
            import pstats

            prof.disable()
            pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(60)
        t_loop = time.perf_counter()
        torch.cuda.synchronize()
        drain = time.perf_counter() - t_loop  # how far the host got ahead of the device
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        pipe.sync_stats()
        knit = sum(s.elapsed_time(e) for s, e in pipe.events) / len(pipe.events)
        sweep = sum(s.elapsed_time(e) for s, e in pipe.sweep_events) / max(len(pipe.sweep_events), 1)
        prep = sum(s.elapsed_time(e) for s, e in pipe.prep_events) / max(len(pipe.prep_events), 1)
        M, N, K = pipe.gemm_shape()
        print(json.dumps({"workload": args.workload, "mode": pipe.mode, "prep": pipe.slice_prep,
                          "cost_model_ms": pipe.slice_costs, "out_buffers": pipe.out_buffers,
                          "out_selections": list(engine.out_selections),
                          "out_stats": engine.out_stats(),
                          "world": world, "rank": args.rank,
                          "slice": list(pipe.slice), "ms_per_step_no_xgmi": round(ms, 3), "host_ms_per_step": round(host / args.steps * 1e3, 3), "drain_ms": round(drain * 1e3, 3),
                          "sweep_ms": round(sweep, 3), "prep_ms": round(prep, 3), "knit_ms": round(knit, 3),
                          "knit_GBs": round(8 * M * N / (knit * 1e-3) / 1e9, 1), "accepted_rank": pipe.last_rank,
                          "received_bytes_per_step": {k: v // args.steps for k, v in recv.items()},
                          "xgmi_model": ({"per_link_GBs": args.xgmi_gbs, "latency_us": args.coll_lat_us,
                                          "us_per_step": {k: round(v / args.steps, 1) for k, v in model.items()}}
                                         if args.xgmi_gbs > 0 else None),
                          "overlap": bool(pipe.overlap), "cus": pipe.overlap_cus,
                          "host_phase_ms": {k: round(v / args.steps * 1e3, 3) for k, v in host_phase.items()}}),
              flush=True)
        del pipe
        if args.no_world_sync:
            continue
        import gc

        gc.collect()  # this world's output mappings go now (synchronised), not at a later collection
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
