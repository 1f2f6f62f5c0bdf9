#!/usr/bin/env python3
"""One rank's device work of the multi-GPU bench (gather mode), on one GPU, without RCCL.

The driver runs ``bench.py --gpus 8``; this box has one GPU. Here the pipeline of rank ``r`` of
``world`` ranks is built exactly as bench.py builds it (syc 32 5, factored knit, ``gather``
mode); only the two collectives are replaced by local copies of the same size into the same
receive buffers, so the step times everything a rank computes (its sweep shard, the operand
transforms, its block of output rows) but not the xGMI transfer. The per-rank bytes each
collective moves are printed next to it, so the predicted N-GPU step is
``compute + exchange bytes / xGMI bandwidth``.

    python tools/rank_sim.py --world 2 4 8 --steps 5
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
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, variant = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, variant)

    for world in args.world:
        exch = {}

        def local_exchange(self, i, qpad):
            kind, send, recv = self.xbuf[i]
            if kind == "a2a":
                P, per, bw = send.shape
                send.copy_(qpad[:per].view(per, P, bw).transpose(0, 1))
                recv.view(P, per, bw).copy_(send)
                exch[i] = ("all_to_all", send.numel() * 8 * (P - 1) // P)
            else:
                per = recv.shape[0] // self.world
                recv[:per].copy_(qpad[:per])
                exch[i] = ("all_gather", recv.numel() * 8 * (self.world - 1) // self.world)
            return _Done(), recv

        KnitPipeline._exchange = local_exchange
        pipe = KnitPipeline(VirtualCircuit(cut), factored=True, rank=args.rank, world=world, mode="gather")
        for _ in range(args.warmup):
            pipe.step()
        torch.cuda.synchronize()
        pipe.record_events = True
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        gemm = sum(s.elapsed_time(e) for s, e in pipe.events) / len(pipe.events)
        sweep = sum(s.elapsed_time(e) for s, e in pipe.sweep_events) / len(pipe.sweep_events)
        print(json.dumps({"workload": args.workload, "world": world, "rank": args.rank,
                          "ms_per_step_no_xgmi": round(ms, 3), "sweep_ms": round(sweep, 3),
                          "contraction_ms": round(gemm, 3), "gemm_mnk": list(pipe.gemm_shape()),
                          "exchange_bytes_received": {str(k): v for k, v in exch.items()}}), flush=True)
        del pipe
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
