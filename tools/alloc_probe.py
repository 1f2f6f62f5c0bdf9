#!/usr/bin/env python3
"""Does the output buffer's allocation change the write rate? The bench step's write kernel
(syc 32 5, 2^32 fp64) timed with HIP events into: the pipeline's own buffer, fresh torch buffers,
a raw hipMalloc and hipExtMallocWithFlags(hipDeviceMallocContiguous) (when the runtime grants it).

    python tools/alloc_probe.py --steps 6
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_CONTIGUOUS = 0x4


class _Raw:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    torch.cuda.set_stream(torch.cuda.Stream())
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    pipe.step()
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    N = 1 << 32

    def run(tag, buf):
        pipe.out = buf
        pipe.step()
        torch.cuda.synchronize()
        pipe.record_events = True
        pipe.events.clear()
        for _ in range(args.steps):
            pipe.step()
        torch.cuda.synchronize()
        w = [s.elapsed_time(e) for s, e in pipe.events]
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        buf.zero_()
        s0.record()
        for _ in range(3):
            buf.zero_()
        s1.record()
        torch.cuda.synchronize()
        print(json.dumps({"tag": tag, "write_ms": round(sum(w) / len(w), 4), "write_min_ms": round(min(w), 4),
                          "torch_fill_ms": round(s0.elapsed_time(s1) / 3, 4), "ptr": hex(buf.data_ptr())}), flush=True)

    own = pipe.out
    run("pipeline's own buffer (first large allocation)", own)
    t1 = torch.empty(N, dtype=torch.float64, device="cuda")
    run("torch.empty #1", t1)
    t2 = torch.empty(N, dtype=torch.float64, device="cuda")
    run("torch.empty #2", t2)
    t3 = torch.empty(N, dtype=torch.float64, device="cuda")
    run("torch.empty #3", t3)
    t4 = torch.empty(N, dtype=torch.float64, device="cuda")
    run("torch.empty #4", t4)
    del t1, t2, t3, t4
    torch.cuda.empty_cache()
    raw = {}
    for tag, flags in (("hipMalloc", None), ("hipExtMallocWithFlags contiguous", HIP_CONTIGUOUS)):
        ptr = ctypes.c_void_p()
        if flags is None:
            err = hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(8 * N))
        else:
            err = hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(8 * N), ctypes.c_uint(flags))
        if err != 0 or not ptr.value:
            print(json.dumps({"tag": tag, "error": int(err)}), flush=True)
            continue
        raw[tag] = ptr
        run(tag, torch.as_tensor(_Raw(ptr.value, N), device="cuda"))
        pipe.out = own
        torch.cuda.synchronize()
        hip.hipFree(ptr)
    run("pipeline's own buffer again", own)


if __name__ == "__main__":
    main()
