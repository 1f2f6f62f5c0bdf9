#!/usr/bin/env python3
"""Slice mode through a real one-rank RCCL group, step by step, with progress lines and a stack dump
if it stalls (faulthandler): where a collective of the sharded / replicated step waits.

    python tools/rccl_slice_probe.py --case hwe_p2 --prep sharded --buffers 1 [--plain] [--out DIR]
"""
import argparse
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="hwe_p2")
    ap.add_argument("--prep", default="sharded")
    ap.add_argument("--buffers", type=int, default=1)
    ap.add_argument("--plain", action="store_true", help="no pipelined steps")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out")
    ap.add_argument("--dump-after", type=float, default=45.0)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    tb = open(os.path.join(args.out, f"rccl_probe_{args.case}_{args.prep}_{args.buffers}.tb"), "w")
    faulthandler.dump_traceback_later(args.dump_after, repeat=True, file=tb)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QKNIT_SLICE_PREP=args.prep,
                      QKNIT_OUT_BUFFERS=str(args.buffers))
    t0 = time.time()

    def log(msg):
        print(f"{time.time() - t0:7.2f}s {msg}", flush=True)

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    log("nccl group up")
    import circuits
    from oracle import dense

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = {"hwe_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[1],
           "cx_8x8": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]}[args.case]()
    t = torch.ones(4, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    log(f"plain all_reduce ok {t.tolist()}")
    pipe = KnitPipeline(VirtualCircuit(cut), device=0, rank=0, world=1, mode="slice", factored=True,
                        group=dist.group.WORLD, data_rank=True)
    log(f"planned: prep {pipe.slice_prep}, dev_rank {pipe.dev_rank}")
    ref = dense.run_dense(cut)
    torch.cuda.set_stream(torch.cuda.Stream())
    pipe.overlap = (not args.plain) and pipe.overlap_ok()
    for it in range(args.steps):
        out = pipe.step()
        log(f"step {it} queued")
        torch.cuda.synchronize()
        err = float(abs(out.cpu().numpy() - ref).max())
        log(f"step {it} done, max err {err:.2e}, overlap {pipe.overlap} cus {pipe.overlap_cus}")
    pipe.sync_stats()
    log(f"rank {pipe.last_rank} fallbacks {pipe.rank_fallbacks}")
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()
    log("done")


if __name__ == "__main__":
    main()
