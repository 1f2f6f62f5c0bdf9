#!/usr/bin/env python3
"""Compile a workload's per-program sweep kernels offline (hipcc, gfx950) and count their ISA.

  python tools/sweep_isa.py [--workload syc_32_5_p2] [--keep DIR]

No GPU needed: the multi-fragment source KnitPipeline would hand to hiprtc
(sweep_codegen.generate_multi over the basis-reduced fragments) is compiled with hipcc
--offload-device-only, disassembled with llvm-objdump, and per kernel the f64 VALU
instructions (fma / mul / add), LDS ops, VGPR count and LDS size are printed, so codegen changes
can be compared before a GPU run.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--keep", default=None)
    ap.add_argument("--tile-bits", type=int, default=None, help="default: what prepare_fragments picks")
    ap.add_argument("--final-tile-bits", type=int, default=None, help="default: what prepare_fragments picks")
    ap.add_argument("--flags", nargs="*", default=[], help="extra compiler flags (e.g. -fno-signed-zeros)")
    args = ap.parse_args()
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import sweep_codegen, sweep_plan

    name, n, d, p, var = cutting.BASELINE_CONFIGS[args.workload]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    frags = engine.prepare_fragments(VirtualCircuit(cut), 0, upload=False, basis=True)
    live = [fs for fs in frags if not fs.dropped]
    tb = args.tile_bits or live[0].jit[1]
    ftb = args.final_tile_bits if args.final_tile_bits is not None else live[0].jit[2]
    encs = [sweep_plan.encode(engine._device_program(fs.prog)[0], tile_bits=tb, final_tile_bits=ftb or None)
            for fs in live]
    src, names = sweep_codegen.generate_multi(encs)
    d = args.keep or tempfile.mkdtemp()
    os.makedirs(d, exist_ok=True)
    cpp = os.path.join(d, "sweep.hip")
    asm = os.path.join(d, "sweep.s")
    open(cpp, "w").write(src)
    first = src.split("\n", 1)[0]
    if first.startswith("// qk-options:"):  # the options qk_module_compile passes to hiprtc
        args.flags = first[len("// qk-options:"):].split() + args.flags
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--offload-device-only", "-O3", "-std=c++17",
                    "-S", cpp, "-o", asm, "-Rpass-analysis=kernel-resource-usage", *args.flags], check=True,
                   stderr=open(os.path.join(d, "resource.txt"), "w"))
    dis = open(asm).read()
    cur, counts = None, collections.defaultdict(collections.Counter)
    for line in dis.splitlines():
        m = re.match(r"^(\w+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            continue
        m = re.match(r"^\s+(v_\w+|ds_\w+|s_barrier|global_\w+|buffer_\w+)", line)
        if m and cur:
            counts[cur][m.group(1)] += 1
    res = open(os.path.join(d, "resource.txt")).read()
    for k in names:
        c = counts.get(k, collections.Counter())
        f64 = {x: c[x] for x in ("v_fma_f64", "v_fmac_f64_e32", "v_mul_f64", "v_add_f64") if c[x]}
        lds = sum(v for x, v in c.items() if x.startswith("ds_"))
        vg = re.search(rf"Function Name: {k}\n.*?VGPRs: (\d+)", res, re.S)
        print(f"{k}: f64 {f64} (sum {sum(f64.values())}), ds {lds}, barriers {c['s_barrier']}, "
              f"valu total {sum(v for x, v in c.items() if x.startswith('v_'))}, VGPRs {vg.group(1) if vg else '?'}")
    print(f"source / asm in {d}")


if __name__ == "__main__":
    main()
