"""In-tree build of libqknit.so (hipcc, gfx950). Used by __graft_entry__.build() and tests."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f) for f in ("qknit.hip", "qknit_post.hip", "qknit_jit.hip",
                                                              "qknit_sample.hip", "qknit_rank.hip",
                                                              "qknit_plan.hip", "qknit_prep.hip",
                                                              "qknit_select.hip", "qknit_comm.hip",
                                                              "qknit_mem.hip", "qknit_trunc.hip",
                                                              "qknit_prim.hip")]
DEPS = SRCS + [os.path.join(HERE, "csrc", h) for h in ("internal.h", "sweep_ops.h", "prim.h")]
HEADER = os.path.join(os.path.dirname(HERE), "include", "qknit.h")
OUT = os.path.join(HERE, "libqknit.so")
ARCH = os.environ.get("QKNIT_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_library(force: bool = False, verbose: bool = False, out: str = OUT,
                  defines: tuple = ()) -> str:
    """Build ``out`` (default: the in-tree libqknit.so). ``defines`` are extra ``-D`` macros,
    used only by tools/ to build kernel-tuning variants next to the product library."""
    stale = not os.path.exists(out) or any(
        os.path.getmtime(p) > os.path.getmtime(out) for p in DEPS + [HEADER]
    )
    if not (force or stale):
        return out
    tmp = out + ".tmp"
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
             *[f"-D{d}" for d in defines]]
    # one hipcc per translation unit, in parallel (the device code dominates: ~2 min serial), then link
    objdir = os.path.join(os.path.dirname(out), "build", os.path.basename(out) + ".objs")
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    for src in SRCS:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [hipcc(), *flags, "-c", src, "-o", obj]
        jobs.append((cmd, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    errs = []
    for cmd, obj, proc in jobs:
        _, err = proc.communicate()
        if proc.returncode != 0:
            errs.append(f"{' '.join(cmd)}\n{err}")
        elif verbose and err:
            print(err)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    cmd = [hipcc(), *flags, "-shared", *[obj for _, obj, _ in jobs], "-lhiprtc", "-lrccl", "-o", tmp]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc link failed:\n{' '.join(cmd)}\n{res.stderr}")
    os.replace(tmp, out)
    return out


# BASELINE configs whose per-program kernels are compiled ahead of time (jit cache)
AOT_CONFIGS = ("qft_16_1_p3", "syc_32_5_p2", "syc_32_1_p2", "syc_32_1_p2_forced", "hwe_16_1_p2", "hwe_16_1_p3")


def build_jit_cache(configs=AOT_CONFIGS, verbose: bool = False) -> list:
    """Compile the per-program sweep kernels the BASELINE configs' plans use (engine.jit_sources:
    factored and direct plans) with ``hipcc --genco`` into engine.JIT_CACHE_DIR, so no plan of them
    waits for hiprtc at run time (qft 16's 481 ops: ~7 s). Code objects already there are kept.
    Returns the paths written."""
    import tempfile

    from . import VirtualCircuit, cutting, engine

    todo = {}
    for key in configs:
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
        virt = VirtualCircuit(cut)
        for basis in ({False, True} if virt.vgate_instructions else {False}):
            for src, _ in engine.jit_sources(virt, basis=basis):
                path = engine.jit_cache_path(src)
                if not os.path.exists(path):
                    todo[path] = src
    os.makedirs(engine.JIT_CACHE_DIR, exist_ok=True)
    procs = []
    with tempfile.TemporaryDirectory() as tmp:
        for i, (path, src) in enumerate(todo.items()):
            f = os.path.join(tmp, f"prog{i}.hip")
            with open(f, "w") as fh:
                fh.write(src)
            cmd = [hipcc(), "--genco", "--no-gpu-bundle-output", *engine.jit_options(src), f, "-o", path + ".tmp"]
            procs.append((path, cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        errs = []
        for path, cmd, proc in procs:
            _, err = proc.communicate()
            if proc.returncode != 0:
                errs.append(f"{' '.join(cmd)}\n{err}")
            else:
                os.replace(path + ".tmp", path)
                if verbose:
                    print(f"jit cache: {path}")
        if errs:
            raise RuntimeError("hipcc --genco failed:\n" + "\n".join(errs))
    return list(todo)
