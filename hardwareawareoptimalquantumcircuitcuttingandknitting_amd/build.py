"""In-tree build of libqknit.so (hipcc, gfx950). Used by __graft_entry__.build() and tests."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f) for f in ("qknit.hip", "qknit_post.hip", "qknit_jit.hip",
                                                              "qknit_sample.hip", "qknit_rank.hip",
                                                              "qknit_plan.hip", "qknit_prep.hip",
                                                              "qknit_select.hip", "qknit_comm.hip")]
DEPS = SRCS + [os.path.join(HERE, "csrc", h) for h in ("internal.h", "sweep_ops.h")]
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
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result", *[f"-D{d}" for d in defines], *SRCS, "-lhiprtc", "-lrccl", "-o", tmp]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{res.stderr}")
    if verbose and res.stderr:
        print(res.stderr)
    os.replace(tmp, out)
    return out
