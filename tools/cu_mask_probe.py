#!/usr/bin/env python3
"""CU-masked streams on one MI355X: does a masked stream confine its kernels, and do the sweep
(preparation) and the write-bound knit run concurrently on disjoint CU sets?

  GPU_MAX_HW_QUEUES=8 python tools/cu_mask_probe.py

For each (prep CUs, layout): the syc 32 5 sweep alone on the prep stream, the knit write alone on
the write stream, then both issued together (sweep x4 behind the write) — wall time of the pair vs
the sum / max of the parts. One JSON line per setting.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    pipe.step()
    qs = pipe.sweep()
    prep = pipe._prep_dev_rank(qs)
    torch.cuda.synchronize()
    total = engine.device_cu_count(0)

    def timed(stream, fn, reps=3):
        with torch.cuda.stream(stream):
            pipe.be.bind()
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
        pipe.be.bind()
        return (time.perf_counter() - t0) / reps * 1e3

    write = lambda: pipe._launch_dev_rank(prep)  # noqa: E731
    sweep = lambda: pipe.sweep()  # noqa: E731
    full = torch.cuda.Stream()
    print(json.dumps({"setting": "full chip", "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "sweep_ms": timed(full, sweep), "write_ms": timed(full, write)}), flush=True)
    for c, lay in [(32, "spread"), (32, "block"), (64, "spread"), (32, "xcd")]:
        if lay == "block":
            pc = tuple(range(total - c, total))
        elif lay == "xcd":  # c CUs = the low c / 8 of each 32-CU group
            per = c // 8
            pc = tuple(x * (total // 8) + i for x in range(8) for i in range(per))
        else:
            stride = total // c
            pc = tuple(i for i in range(total) if i % stride == stride - 1)[:c]
        wc = tuple(i for i in range(total) if i not in set(pc))
        S, W = engine.cu_masked_stream(0, pc), engine.cu_masked_stream(0, wc)
        t_s, t_w = timed(S, sweep), timed(W, write)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(W):
            pipe.be.bind()
            write()
        with torch.cuda.stream(S):
            pipe.be.bind()
            for _ in range(4):
                sweep()
        torch.cuda.synchronize()
        both = (time.perf_counter() - t0) * 1e3
        pipe.be.bind()
        print(json.dumps({"prep_cus": c, "layout": lay, "sweep_ms_masked": t_s, "write_ms_masked": t_w,
                          "write_plus_4_sweeps_concurrent_ms": both, "serial_sum_ms": t_w + 4 * t_s,
                          "max_ms": max(t_w, 4 * t_s)}), flush=True)


if __name__ == "__main__":
    main()
