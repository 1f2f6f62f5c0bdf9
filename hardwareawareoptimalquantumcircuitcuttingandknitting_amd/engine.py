"""Device-side orchestration: compiled fragments, batched sweep, dense knit.

Everything numeric here runs in ``libqknit.so`` (HIP, gfx950) through the C ABI
(``include/qknit.h``); torch is used only for device allocations and stream
ordering. There is no CPU compute path: without the library or without a GPU
every entry point raises.

Pipeline of one virtual-circuit run (``run.py:23-71`` in the reference):

1. :func:`sweep_fragment` — per fragment: compile (``fragment_program``),
   schedule (``sweep_plan``), expand labels into branch jobs, ``qk_sweep``
   (exact probabilities of every instantiation), ``qk_reduce_labels`` (signed
   config-bit folding) -> ``q_f [L_f, 2^m_f]``.
2. :func:`knit_dense` — gather/scale fragment rows per global label
   (``qk_gather_rows``, or the factored transform), then ``qk_gemm_keyed``
   (fp64 MFMA) writes the dense distribution at global clbit keys.
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import dataclasses
import hashlib
import logging
import os
import threading
from dataclasses import dataclass, field
from time import perf_counter

import numpy as np

from . import _lib
from .fragment_program import (FragmentProgram, JobTable, basis_reduce, build_jobs, compile_fragment,
                               dedup_labels)
from .knit_plan import LabelSpace, deposit_keys, factor_vgate
from .sweep_plan import K_SLOT, EncodedProgram, encode

_torch = None


def torch():
    global _torch
    if _torch is None:
        import torch as t

        _torch = t
    return _torch


def _ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


# ----------------------------------------------------------------------------- context
# set at interpreter exit (atexit): finalizers that would call into the HIP runtime (unmapping outputs,
# destroying contexts) then leave it to the process exit — a mapping or context still alive in a
# reference cycle the final collection breaks crashed the process there (rank_sim --host-profile)
_OUT_EXITING = [False]


def _out_exiting():
    _OUT_EXITING[0] = True


atexit.register(_out_exiting)


class Context:
    """One ``qk_ctx`` per (thread, device); ops run on torch's current stream."""

    def __init__(self, device: int = 0):
        T = torch()
        if not T.cuda.is_available():
            raise _lib.QknitError("no HIP device available (torch.cuda.is_available() is False)")
        self.device = device
        self.lib = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(None, self.lib.qk_ctx_create(device, ctypes.byref(h)), "qk_ctx_create")
        self.handle = h

    def bind_stream(self) -> None:
        s = torch().cuda.current_stream(self.device).cuda_stream
        if s != getattr(self, "_bound", None):
            self.lib.qk_ctx_set_stream(self.handle, ctypes.c_void_p(s))
            self._bound = s

    def check(self, status: int, what: str) -> None:
        _lib.check(self.handle, status, what)

    def close(self) -> None:
        if self.handle:
            self.lib.qk_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        if _OUT_EXITING is None or _OUT_EXITING[0]:  # interpreter exit (module globals cleared too)
            return
        try:
            self.close()
        except Exception:
            pass


_MASKED_STREAMS: dict = {}


def _destroy_masked_streams():
    """atexit: destroy the CU-masked HIP streams while the runtime is still up."""
    for key, st in list(_MASKED_STREAMS.items()):
        try:
            st.synchronize()
            _lib.lib().qk_stream_destroy(ctypes.c_void_p(st.cuda_stream))
        except Exception:
            pass
        _MASKED_STREAMS.pop(key, None)


def device_cu_count(device: int = 0) -> int:
    """Compute units of the device (what an unmasked stream may use)."""
    lib = _lib.lib()
    n = ctypes.c_int()
    _lib.check(None, lib.qk_stream_cu_count(device, None, ctypes.byref(n)), "qk_stream_cu_count")
    return n.value


def cu_masked_stream(device: int, cus: tuple, tag: int = 0):
    """A torch stream over a HIP stream restricted to the logical CUs ``cus``
    (``qk_stream_create_cu_masked``), created once per (device, CU set, tag) and kept for the process
    (``tag``: another stream over the same CUs)."""
    key = (device, tuple(sorted(cus)), tag)
    with _modules_lock:
        if key not in _MASKED_STREAMS:
            lib = _lib.lib()
            words = (max(key[1]) >> 5) + 1
            mask = (ctypes.c_uint32 * words)()
            for c in key[1]:
                mask[c >> 5] |= 1 << (c & 31)
            h = ctypes.c_void_p()
            _lib.check(None, lib.qk_stream_create_cu_masked(device, mask, words, ctypes.byref(h)),
                       "qk_stream_create_cu_masked")
            if not _MASKED_STREAMS:
                import atexit

                atexit.register(_destroy_masked_streams)
            _MASKED_STREAMS[key] = torch().cuda.ExternalStream(h.value, device=torch().device("cuda", device))
        return _MASKED_STREAMS[key]


_tls = threading.local()


def get_context(device: int = 0) -> Context:
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    if device not in cache:
        cache[device] = Context(device)
    ctx = cache[device]
    ctx.bind_stream()
    return ctx


class _Lease:
    """What a tensor over a MappedOut holds (through ``__cuda_array_interface__``): one per
    :meth:`MappedOut.tensor`, alive exactly as long as that tensor's storage (views included)."""

    def __init__(self, owner):
        self.owner = owner
        self.__cuda_array_interface__ = owner.cai


class MappedOut:
    """Owner of one ``qk_out_alloc`` mapping (1-GiB physical chunks at a 1-GiB-aligned address,
    csrc/qknit_mem.hip): the knit output the write kernels stream into at the same rate whichever
    memory the device hands out (a plain allocation: 4.8 or 5.9 ms per 2^32 fp64, by block). Tensors
    over it (:meth:`tensor`) keep it alive; the mapping is released (device synchronised first) when
    the last of them and this object are gone."""

    def __init__(self, ctx: Context, n: int):
        self.lib, self.device, self.n = ctx.lib, ctx.device, int(n)
        p = ctypes.c_void_p()
        ctx.check(ctx.lib.qk_out_alloc(ctx.handle, 8 * self.n, ctypes.byref(p)), "qk_out_alloc")
        self.ptr = p.value
        self.cai = {"shape": (self.n,), "typestr": "<f8", "data": (self.ptr, False), "version": 2}
        self._leases = []

    def tensor(self):
        """A float64 [n] tensor on the mapping (its storage holds this owner)."""
        import weakref

        T = torch()
        lease = _Lease(self)
        with T.cuda.device(self.device):
            t = T.as_tensor(lease, device=T.device("cuda", self.device))
        if t.data_ptr() != self.ptr:
            raise _lib.QknitError("qk_out_alloc buffer was copied instead of shared")
        self._leases = [w for w in self._leases if w() is not None] + [weakref.ref(lease)]
        return t

    def mapped_bytes(self) -> int:
        """Device bytes the mapping holds (whole physical chunks: at least 8 n)."""
        size = ctypes.c_int64()
        if self.ptr is None or self.lib.qk_out_mapped_bytes(ctypes.c_void_p(self.ptr), ctypes.byref(size)) != 0:
            return 8 * self.n
        return size.value

    def in_use(self) -> bool:
        """Whether a tensor handed out by :meth:`tensor` (or a view of it) is still alive."""
        return any(w() is not None for w in self._leases)

    def __del__(self):
        # at interpreter exit (after atexit: _OUT_EXITING) the HIP runtime may already be torn down — a
        # mapping still alive then (e.g. held by a reference cycle the final collection breaks) is left to
        # the process exit; unmapping it there crashed the process (rank_sim --host-profile)
        if getattr(self, "ptr", None) and _OUT_EXITING is not None and not _OUT_EXITING[0]:
            try:
                self.lib.qk_out_free(None, ctypes.c_void_p(self.ptr))
            except Exception:
                pass
        self.ptr = None


OUT_MAPPED_MIN_BYTES = int(os.environ.get("QKNIT_OUT_MAPPED_MIN_BYTES", str(1 << 30)))  # below: torch allocation
# Large outputs are kept only if they write fast. The knit writes its 2^32 fp64 outputs at 4.8-5.0 ms
# into most mappings and at 5.2-5.9 ms into others — fixed per mapping (stable over seconds), the same
# for every store order tried (task widths 2^12-2^16, compact or spread windows, other grids), for
# 1-GiB-aligned and unaligned addresses, chunks created per buffer or all first (tools/write_probe11-13,
# out_mapping_tb.py). qk_out_write_rate times the knit's store order into a new mapping
# (one 5-ms launch for 34 GB); below OUT_FAST_GBS another mapping is made while the earlier ones are held
# (so their memory cannot come straight back), up to OUT_TRIES, the fastest kept and the others freed.
# Extra tries only with free memory for them (2 GiB spare): a 2^32 output holds at most OUT_TRIES x
# 34 GB for the few milliseconds of the selection.
# From 4 GiB on (round 5; before: full 2^32 outputs only): a rank's slice writes at 5.6-6.3 TB/s by the
# same check, below the threshold, so each slice buffer is the fastest of OUT_TRIES mappings — and the
# pipelined multi-GPU step gains from it on every box measured: 8 ranks 0.776-0.816 vs 0.839-0.870 ms,
# 4 ranks 1.39-1.41 vs 1.64, 2 ranks 2.52-2.53 vs 2.62 (profiles/r05ar_*, r05as_*). A slice buffer is
# held by a pipelined step for the run, so the milliseconds of the selection are a plan-time cost.
OUT_SELECT_MIN_BYTES = int(os.environ.get("QKNIT_OUT_SELECT_MIN_BYTES", str(4 << 30)))
# Early-stop rate: a candidate at least this fast is kept at once (the others are made only while the
# candidates so far are slower). Slice buffers of a 2-8-rank step write at 5.6-6.3 TB/s, below it, so
# for them every one of OUT_TRIES candidates is made and the fastest kept (the early stop acts only on
# full 2^32 outputs). QKNIT_OUT_FAST_GBS=inf does the same for every output: one GPU, same box, three
# alternating rounds 4.948-4.967 vs 4.964-4.982 ms per step (profiles/r05av_*). Round 5 saw one
# memory-access fault reported at a write-rate check with inf in a 2 -> 4-rank rank_sim process
# (r05bb); qk_out_write_rate now drains the device first and says when an error predates its probe,
# and qk_out_stats counts reservations (DESIGN.md §4 for what the reruns found)
OUT_FAST_GBS = float(os.environ.get("QKNIT_OUT_FAST_GBS", "6850"))
OUT_TRIES = int(os.environ.get("QKNIT_OUT_TRIES", "3"))
# A candidate mapping that took longer than this (host ms) ends the selection after its rate check:
# memory a process released moments before (e.g. the previous process on the device) is handed out
# again only after the driver has cleared it, and a mapping that reaches into it blocks for seconds
# (tools/map_stall_probe.py --seq: 3.3 s for one 32-GiB mapping right after a process holding 192 GiB
# exited, 0.6-0.8 ms 30 s later; profiles/r06k_*). The next candidate would wait the same way.
OUT_MAP_SLOW_MS = float(os.environ.get("QKNIT_OUT_MAP_SLOW_MS", "200"))
out_selections: list = []  # per selected output: the candidates' write rates (GB/s), the kept one first
out_selection_log: list = []  # per selected output: host ms of each mapping, each rate check, the frees
_out_select_lock = threading.Lock()  # one selection at a time per process: two threads' candidates never stack


OUT_STATS_FIELDS = ("reserved", "reserve_failed", "map_failed", "live", "live_bytes", "retired", "retired_bytes",
                    "max_bytes", "probe_pre_errors")


def out_stats() -> dict:
    """qk_out_alloc's process counters (``qk_out_stats``): reservations made / failed, live and retired
    mappings and bytes, the largest mapping, write-rate checks that found an earlier error."""
    L = _lib.lib()
    v = (ctypes.c_int64 * len(OUT_STATS_FIELDS))()
    if L.qk_out_stats(v, len(OUT_STATS_FIELDS)) != 0:
        raise _lib.QknitError("qk_out_stats failed")
    return dict(zip(OUT_STATS_FIELDS, (int(x) for x in v)))


_out_fallback_warned = [False]


def _out_rate(ctx: Context, owner) -> float:
    g = ctypes.c_double()
    ctx.check(ctx.lib.qk_out_write_rate(ctx.handle, ctypes.c_void_p(owner.ptr), 8 * owner.n, ctypes.byref(g)),
              "qk_out_write_rate")
    return g.value


def out_buffer(ctx: Context, n: int, select: bool = True):
    """(tensor [n] float64, owner or None): a ``qk_out_alloc`` mapping for outputs of at least
    OUT_MAPPED_MIN_BYTES (from OUT_SELECT_MIN_BYTES on, one that writes fast: see above), torch's
    allocator below that. Contents are undefined. ``select=False``: the first mapping, not timed
    (the drop-in's first call: the call's own write then says whether to replace it,
    KnitPipeline.take_out)."""
    T = torch()
    if 8 * n < OUT_MAPPED_MIN_BYTES:
        return T.empty(n, dtype=T.float64, device=T.device("cuda", ctx.device)), None
    try:
        first = MappedOut(ctx, n)
    except _lib.QknitError as e:
        # no mapping (the address space of never-reused retired ranges is full, or no physical chunk):
        # an ordinary allocation, recorded — and said once, since its write rate is the buffer lottery's
        out_selections.append(["torch allocation: qk_out_alloc failed"])
        if not _out_fallback_warned[0]:
            _out_fallback_warned[0] = True
            import warnings

            warnings.warn(f"qk_out_alloc failed ({e}); large outputs fall back to torch allocations "
                          f"(out_stats: {out_stats()})", RuntimeWarning, stacklevel=2)
        return T.empty(n, dtype=T.float64, device=T.device("cuda", ctx.device)), None
    if 8 * n < max(OUT_SELECT_MIN_BYTES, 1 << 19) or OUT_TRIES <= 1 or not select:
        # (qk_out_write_rate times whole 512-KiB blocks: nothing smaller is selected)
        return first.tensor(), first
    with _out_select_lock:
        owner = first
        first = None
        t = perf_counter()
        tried = [(_out_rate(ctx, owner), owner)]
        log = {"bytes": 8 * n, "rate_ms": [(perf_counter() - t) * 1e3], "map_ms": []}
        while tried[-1][0] < OUT_FAST_GBS and len(tried) < OUT_TRIES:
            free, _ = T.cuda.mem_get_info(ctx.device)
            if free < 8 * n + (2 << 30):
                log["stopped"] = f"free {free / 2**30:.1f} GiB"
                break
            t = perf_counter()
            try:  # memory taken meanwhile (another thread / process): keep the best so far
                cand = MappedOut(ctx, n)
            except _lib.QknitError:
                break
            log["map_ms"].append((perf_counter() - t) * 1e3)
            t = perf_counter()
            tried.append((_out_rate(ctx, cand), cand))
            log["rate_ms"].append((perf_counter() - t) * 1e3)
            if log["map_ms"][-1] > OUT_MAP_SLOW_MS:
                log["stopped"] = f"mapping took {log['map_ms'][-1]:.0f} ms"
                break
        best = max(range(len(tried)), key=lambda i: tried[i][0])
        owner = tried[best][1]
        out_selections.append([round(tried[best][0], 1)] + [round(r, 1) for i, (r, _) in enumerate(tried) if i != best])
        t = perf_counter()
        del tried  # the others are unmapped here (cand: the last candidate's name)
        cand = None
        log["free_ms"] = (perf_counter() - t) * 1e3
        out_selection_log.append(log)
    return owner.tensor(), owner


# ----------------------------------------------------------------------------- fragments
@dataclass
class DeviceProgram:
    host: FragmentProgram
    enc: EncodedProgram
    ops: object  # torch tensors (device) kept alive
    groups: object
    mats: object
    passes: object  # ctypes array (host)
    struct: _lib.QkProgram = field(default=None)
    module: object = None  # qk_module* of the per-program kernels (SPLIT programs), or None

    @staticmethod
    def upload(prog: FragmentProgram, device, jit: bool = True, tile_bits: int | None = None,
               final_tile_bits: int | None = None) -> "DeviceProgram":
        T = torch()
        # per-program kernels take up to 13-bit tiles (128 KiB LDS: fewer passes, less state
        # traffic); smaller ones when the batch is too small to fill the chip (jit_tile_bits); the
        # FINAL pass may run on narrower tiles (final_tile_bits)
        jit = jit and _jit_enabled()
        enc = encode(prog, tile_bits=(tile_bits or JIT_TILE_BITS_MAX) if jit else 12,
                     final_tile_bits=final_tile_bits if jit else None)
        dev = T.device("cuda", device)

        def to_dev(arr, dtype):
            buf = np.ascontiguousarray(arr).view(np.uint8)
            t = T.empty(max(buf.size, 8), dtype=T.uint8, device=dev)
            if buf.size:
                t[: buf.size].copy_(T.from_numpy(buf.copy()))
            return t

        ops = to_dev(enc.ops, None)
        groups = to_dev(enc.groups, None)
        mats = T.from_numpy(enc.mats.copy()).to(dev)
        np_pass = enc.passes
        passes = (_lib.QkPass * len(np_pass))()
        for i, p in enumerate(np_pass):
            passes[i].tile_mask = int(p["tile_mask"])
            passes[i].group_begin = int(p["group_begin"])
            passes[i].group_end = int(p["group_end"])
            passes[i].flags = int(p["flags"])
            passes[i].traced_local = int(p["traced_local"])
        st = _lib.QkProgram(enc.n, enc.n_eff, enc.m, enc.n_slots, int(enc.packed), len(np_pass),
                            ctypes.cast(passes, ctypes.POINTER(_lib.QkPass)),
                            ops.data_ptr(), groups.data_ptr(), mats.data_ptr())
        module = compiled_module(device, enc) if (jit and not enc.packed) else None
        return DeviceProgram(prog, enc, ops, groups, mats, passes, st, module)


JIT_TILE_BITS_MAX = 13
JIT_TILE_BITS_MIN = 10
JIT_MIN_BLOCKS = 128  # FINAL-pass workgroups a sweep should at least offer (256 CUs)


def jit_tile_bits(sizes: list) -> int:
    """Tile width of the per-program kernels of one sweep: ``sizes`` = (qubits, branch jobs) of its
    SPLIT fragments (they share launches, so one width). The widest tile (13 bits: fewest passes)
    whose FINAL pass still offers ``JIT_MIN_BLOCKS`` workgroups, else 10 bits: syc 32 5 (750 jobs)
    keeps 13, the two single-instance fragments of syc 32 1 get 10 (2 x 64 workgroups instead of
    2 x 8). ``QKNIT_JIT_TILE_BITS`` forces a width."""
    env = os.environ.get("QKNIT_JIT_TILE_BITS")
    if env:
        return int(env)
    for tb in range(JIT_TILE_BITS_MAX, JIT_TILE_BITS_MIN - 1, -1):
        if sum(j << max(n - tb, 0) for n, j in sizes) >= JIT_MIN_BLOCKS:
            return tb
    return JIT_TILE_BITS_MIN


JIT_FINAL_TILE_BITS = 10  # FINAL-pass tile width to aim for (narrow_final_tile); 0 = the pass width


def jit_final_tile_bits(progs: list, tile_bits: int) -> int | None:
    """FINAL-pass tile width of one sweep's per-program kernels (one launch per pass round, so one
    width): ``JIT_FINAL_TILE_BITS`` raised to what every FINAL pass needs, None when that is not
    narrower than ``tile_bits``. ``QKNIT_FINAL_TILE_BITS`` overrides the target (0: off)."""
    from .sweep_plan import final_need_bits

    target = int(os.environ.get("QKNIT_FINAL_TILE_BITS", JIT_FINAL_TILE_BITS))
    if not target or not progs:
        return None
    need = max(final_need_bits(p, tile_bits) for p in progs)
    f = max(target, need, JIT_TILE_BITS_MIN)
    return f if f < tile_bits else None


def _jit_enabled() -> bool:
    return os.environ.get("QKNIT_SWEEP_JIT", "1") != "0"


_MODULES: dict = {}
_modules_lock = threading.Lock()


def compiled_module(device: int, enc):
    """Per-program sweep kernels of a SPLIT program (sweep_codegen.generate), compiled once per
    (device, program) with hiprtc. QKNIT_SWEEP_JIT=0 selects the interpreter kernel instead."""
    if os.environ.get("QKNIT_SWEEP_JIT", "1") == "0":
        return None
    from . import sweep_codegen

    return _compile_module(device, *sweep_codegen.generate(enc))


def compiled_multi_module(device: int, encs: list):
    """Multi-fragment sweep kernels (sweep_codegen.generate_multi), compiled once per
    (device, program set) with hiprtc."""
    from . import sweep_codegen

    return _compile_module(device, *sweep_codegen.generate_multi(encs))


# Code objects of per-program kernels compiled ahead of time (build: __graft_entry__.build() compiles
# the BASELINE configs' programs with hipcc --genco) or at run time (written back when the directory is
# writable): <sha1 of source + options>.hsaco. A long program's hiprtc compile costs seconds (qft 16:
# 481 ops, ~7 s); from the cache it is a load.
JIT_CACHE_DIR = os.environ.get("QKNIT_JIT_CACHE", os.path.join(os.path.dirname(os.path.abspath(__file__)), "jit_cache"))
JIT_BASE_OPTIONS = ("--offload-arch=gfx950", "-O3", "-std=c++17")  # qknit_jit.hip's hiprtc options


def jit_options(src: str) -> list:
    """hiprtc / hipcc options of a generated source: the base ones plus its ``// qk-options:`` line."""
    opts = list(JIT_BASE_OPTIONS)
    tag = "// qk-options:"
    if src.startswith(tag):
        opts += src[len(tag):src.index("\n")].split()
    return opts


def jit_cache_path(src: str) -> str:
    h = hashlib.sha1(src.encode())
    h.update(" ".join(jit_options(src)).encode())
    return os.path.join(JIT_CACHE_DIR, h.hexdigest() + ".hsaco")


def _compile_module(device: int, src: str, names: list):
    key = (device, names[0], hashlib.sha1(src.encode()).hexdigest())
    with _modules_lock:
        if key not in _MODULES:
            ctx = get_context(device)
            arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
            h = ctypes.c_void_p()
            path = jit_cache_path(src)
            loaded = False
            if os.path.exists(path):
                # a cached object that does not load (truncated, or built by another ROCm / hipcc) is
                # compiled again and rewritten, not an error
                img = open(path, "rb").read()
                loaded = ctx.lib.qk_module_load(ctx.handle, img, len(img), arr, len(names), ctypes.byref(h)) == 0
                if not loaded:
                    logging.getLogger(__name__).warning("jit cache %s did not load: compiling again", path)
            if not loaded:
                ctx.check(ctx.lib.qk_module_compile(ctx.handle, src.encode(), arr, len(names), ctypes.byref(h)),
                          "qk_module_compile")
                _MODULES[key] = h  # kept (and so freed with the others) even if writing the cache fails
                _write_cache(ctx, h, path)
            _MODULES[key] = h
        return _MODULES[key]


def _write_cache(ctx, module, path: str) -> None:
    """Keep a run-time compiled code object for later processes (best effort)."""
    if os.environ.get("QKNIT_JIT_CACHE_WRITE", "1") == "0":
        return
    try:
        n = ctypes.c_int64()
        ctx.check(ctx.lib.qk_module_code(module, None, ctypes.byref(n)), "qk_module_code")
        buf = ctypes.create_string_buffer(n.value)
        ctx.check(ctx.lib.qk_module_code(module, buf, ctypes.byref(n)), "qk_module_code")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(buf.raw[: n.value])
        os.replace(tmp, path)
    except (OSError, _lib.QknitError):
        pass


def init_prefixes(enc, jobs: JobTable):
    """Shared INIT prefixes of a two-pass SPLIT program (``qk_sweep_compiled_multi_shared``).

    The sparse INIT pass starts every branch job from |0..0> and applies the same ops except the
    slot ops, so its output depends on a job only through the slot matrices of the slots that pass
    reads. Jobs with equal rows there share one INIT tile: syc 32 5 sweeps 50 INIT tiles for its
    750 branch jobs (each fragment has 5 channels on each of its 2 INIT slots). Returns
    ``(reps, prefix_of)`` — one representative job per prefix (first occurrence order) and each
    job's prefix index — or None when sharing saves nothing (not two passes, no repeated prefix)
    or ``QKNIT_SWEEP_SHARE=0``."""
    if os.environ.get("QKNIT_SWEEP_SHARE", "1") == "0" or enc.packed or len(enc.passes) != 2:
        return None
    n = jobs.n_jobs
    if n < 2:
        return None
    ps = enc.passes[0]
    slots = sorted({int(enc.ops[o]["slot"]) for gi in range(int(ps["group_begin"]), int(ps["group_end"]))
                    for o in range(int(enc.groups[gi]["op_begin"]), int(enc.groups[gi]["op_end"]))
                    if int(enc.ops[o]["kind"]) == K_SLOT})
    if slots:
        rows = np.ascontiguousarray(jobs.slot_mats[:, slots]).reshape(n, -1)
        keys = rows.view(np.uint8).reshape(n, -1)  # bitwise equality: the kernels read these exact values
        _, first, inv = np.unique(keys, axis=0, return_index=True, return_inverse=True)
        order = np.argsort(first, kind="stable")  # prefixes in first-occurrence order
        rank = np.empty_like(order)
        rank[order] = np.arange(order.size)
        reps, prefix_of = first[order].astype(np.int64), rank[inv.reshape(-1)].astype(np.int32)
    else:  # INIT reads no slot: one prefix for every job
        reps, prefix_of = np.zeros(1, np.int64), np.zeros(n, np.int32)
    if reps.size == n:
        return None
    return reps, prefix_of


def jobs_to_device(jobs: JobTable, device):
    T = torch()
    dev = T.device("cuda", device)
    # a rank's share of a multi-GPU sweep may hold no jobs at all (more ranks than swept rows)
    slots = (np.ascontiguousarray(jobs.slot_mats).view(np.float64).reshape(jobs.n_jobs, -1) if jobs.n_jobs
             else np.zeros((0, 1)))
    slot_t = T.from_numpy(slots.copy()).to(dev) if slots.size else T.zeros(1, dtype=T.float64, device=dev)
    sign_t = T.from_numpy(jobs.sign.copy()).to(dev)
    off_t = T.from_numpy(jobs.label_offsets.copy()).to(dev)
    return slot_t, sign_t, off_t


def sweep_jobs(ctx: Context, dprog: DeviceProgram, slot_t, sign_t, n_jobs: int, pjob=None,
               workspace=None):
    """``qk_sweep``: per-job signed probabilities ``[n_jobs, 2^m]``."""
    T = torch()
    dev = T.device("cuda", ctx.device)
    width = 1 << dprog.enc.m
    if pjob is None:
        pjob = T.empty((n_jobs, width), dtype=T.float64, device=dev)
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_sweep_workspace_bytes(ctypes.byref(dprog.struct), n_jobs, ctypes.byref(need)),
              "qk_sweep_workspace_bytes")
    if need.value and (workspace is None or workspace.numel() < need.value):
        workspace = T.empty(need.value, dtype=T.uint8, device=dev)
    if dprog.module is not None:
        ctx.check(ctx.lib.qk_sweep_compiled(ctx.handle, dprog.module, ctypes.byref(dprog.struct), n_jobs,
                                            slot_t.data_ptr(), sign_t.data_ptr(), _ptr(workspace),
                                            need.value, pjob.data_ptr()), "qk_sweep_compiled")
    else:
        ctx.check(ctx.lib.qk_sweep(ctx.handle, ctypes.byref(dprog.struct), n_jobs, slot_t.data_ptr(),
                                   sign_t.data_ptr(), _ptr(workspace) if need.value else None,
                                   need.value, pjob.data_ptr()), "qk_sweep")
    return pjob, workspace


def label_chunks(offsets: np.ndarray, max_jobs: int) -> list:
    """Consecutive label ranges of at most ``max_jobs`` branch jobs each (a label is never split;
    one with more jobs is a chunk of its own): ``[(l0, l1, j0, j1), ...]``."""
    n = len(offsets) - 1
    out, l0 = [], 0
    while l0 < n:
        l1 = l0 + 1
        while l1 < n and offsets[l1 + 1] - offsets[l0] <= max_jobs:
            l1 += 1
        out.append((l0, l1, int(offsets[l0]), int(offsets[l1])))
        l0 = l1
    return out


def sweep_labels(ctx: Context, dprog: DeviceProgram, slot_t, sign_t, n_jobs: int, off_t, n_labels: int,
                 q=None, workspace=None, chunks=None):
    """``qk_sweep_compiled_labels``: per-label signed-folded distributions ``[n_labels, 2^m]``
    straight from the sweep (the FINAL pass sums each label's branch jobs; no per-job rows and
    no ``qk_reduce_labels``). Compiled (SPLIT) programs only.

    ``chunks`` (``[(l0, l1, j0, j1, chunk_offsets_device), ...]``, :func:`label_chunks`) runs
    the passes chunk by chunk through one workspace of the largest chunk's size: the states a
    pass writes and the next reads then stay in the 256 MiB Infinity Cache instead of HBM."""
    T = torch()
    if dprog.module is None:
        raise ValueError("sweep_labels needs a compiled (SPLIT) program")
    dev = T.device("cuda", ctx.device)
    width = 1 << dprog.enc.m
    if q is None:
        q = T.empty((n_labels, width), dtype=T.float64, device=dev)
    if chunks is None:
        chunks = [(0, n_labels, 0, n_jobs, off_t)]
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_sweep_workspace_bytes(ctypes.byref(dprog.struct), max(c[3] - c[2] for c in chunks),
                                               ctypes.byref(need)), "qk_sweep_workspace_bytes")
    if workspace is None or workspace.numel() < need.value:
        workspace = T.empty(max(need.value, 1), dtype=T.uint8, device=dev)
    slot_row = slot_t[0].numel() * 8 if (dprog.enc.n_slots and slot_t.dim() == 2) else 0
    for l0, l1, j0, j1, oc in chunks:
        ctx.check(ctx.lib.qk_sweep_compiled_labels(ctx.handle, dprog.module, ctypes.byref(dprog.struct), j1 - j0,
                                                   slot_t.data_ptr() + j0 * slot_row, sign_t.data_ptr() + 8 * j0,
                                                   l1 - l0, oc.data_ptr(), workspace.data_ptr(), need.value,
                                                   q.data_ptr() + 8 * width * l0), "qk_sweep_compiled_labels")
    return q, workspace


def reduce_labels(ctx: Context, pjob, off_t, n_labels: int, q=None):
    T = torch()
    width = pjob.shape[1]
    if q is None:
        q = T.empty((n_labels, width), dtype=T.float64, device=pjob.device)
    ctx.check(ctx.lib.qk_reduce_labels(ctx.handle, n_labels, off_t.data_ptr(), width,
                                       pjob.data_ptr(), q.data_ptr()), "qk_reduce_labels")
    return q


# ----------------------------------------------------------------------------- shot sampling
_SEED_STRIDE = 0x632BE59BD9B4E019  # per-fragment stream offset (mirrored by oracle/sampling.py)
_U64 = (1 << 64) - 1


def fragment_seed(seed: int, index: int) -> int:
    """Sampling stream seed of the index-th non-empty fragment (``fragment_circuits`` order)."""
    return (int(seed) + index * _SEED_STRIDE) & _U64


def sample_fragment(ctx: Context, fs: "FragmentState", shots: int, seed: int, accuracy: float):
    """Shot-sampled per-label distributions ``q_f [len(fs.labels), 2^m]`` on the GPU.

    The reference samples every instance circuit ``shots`` times and keeps frequencies above
    ``ACCURACY`` (``run.py:42,56``, ``quasi_distr.py:12-20``). Here every reference label
    draws its own ``shots`` (labels sharing an instance are not merged, as in the reference)
    from the exact per-branch distribution of its swept instance (``qk_sweep``): per instance
    CDF (``qk_sample_cdf``), inverse-CDF draws over (config branch, outcome) with a
    counter-based stream (``qk_sample_counts``), frequencies truncated at ``accuracy`` and
    sign-folded over the config bits (``qk_fold_counts``). Rows follow ``fs.labels``; knit
    the result with :func:`label_rows` ``(fs)``.
    """
    T = torch()
    dev = T.device("cuda", ctx.device)
    L = len(fs.labels)
    if shots <= 0:
        raise ValueError("shots must be positive")
    if fs.dropped:
        return T.ones((L, 1), dtype=T.float64, device=dev)
    if fs.expand is not None:
        raise ValueError("basis-reduced fragments cannot be sampled (prepare with basis=False)")
    jobs = fs.jobs
    width = 1 << fs.prog.m
    slot_t, sign_t, off_t = jobs_to_device(jobs, ctx.device)
    pjob, _ = sweep_jobs(ctx, fs.dprog, slot_t, sign_t, jobs.n_jobs)
    pjob = fold_traced(ctx, pjob, fs.fold)  # one sign per job: |sum_t sign P| = sum_t P
    cdf = T.empty_like(pjob)
    n_seg = len(jobs.label_offsets) - 1
    ctx.check(ctx.lib.qk_sample_cdf(ctx.handle, n_seg, off_t.data_ptr(), width, pjob.data_ptr(),
                                    cdf.data_ptr()), "qk_sample_cdf")
    seg = np.ascontiguousarray(fs.row_of_label(), dtype=np.int64)
    offs = jobs.label_offsets
    row_off = np.zeros(L + 1, dtype=np.int64)
    np.cumsum((offs[1:] - offs[:-1])[seg], out=row_off[1:])
    rows = np.concatenate([np.arange(offs[s], offs[s + 1]) for s in seg])
    seg_t = T.from_numpy(seg).to(dev)
    row_off_t = T.from_numpy(row_off).to(dev)
    row_sign_t = T.from_numpy(np.ascontiguousarray(jobs.sign[rows])).to(dev)
    counts = T.zeros((int(row_off[-1]), width), dtype=T.int32, device=dev)
    ctx.check(ctx.lib.qk_sample_counts(ctx.handle, L, 0, seg_t.data_ptr(), off_t.data_ptr(), row_off_t.data_ptr(),
                                       width, cdf.data_ptr(), int(shots), int(seed) & _U64, counts.data_ptr()),
              "qk_sample_counts")
    q = T.empty((L, width), dtype=T.float64, device=dev)
    ctx.check(ctx.lib.qk_fold_counts(ctx.handle, L, row_off_t.data_ptr(), width, row_sign_t.data_ptr(),
                                     counts.data_ptr(), int(shots), float(accuracy), q.data_ptr()), "qk_fold_counts")
    return q


def label_rows(fs: "FragmentState") -> "FragmentState":
    """``fs`` with one row per reference label: the layout of sampled and foreign-backend q_f."""
    return dataclasses.replace(fs, uidx=None, unique_labels=None)


# ----------------------------------------------------------------------------- GEMM helpers
def gemm_keyed(ctx: Context, A, B, keyA=None, keyB=None, out=None, strideA: int = 0,
               strideB: int = 1, beta: int = 0, skip=None):
    """out[kA(i) + kB(j)] (=|+=) sum_k A[k, i] * B[k, j] on the GPU (fp64 MFMA).

    ``kA(i) = keyA[i]`` if a key tensor is given, else ``i * strideA`` (same for B). ``skip``
    (device int32 tensor): the launch writes nothing when it holds a positive value.
    """
    K, M = A.shape
    K2, N = B.shape
    # row-major operands; a column range of a wider matrix (X[:, lo:hi]) passes its row stride as lda
    assert K == K2 and A.dtype == B.dtype and (A.stride(1) == 1 or M == 1) and (B.stride(1) == 1 or N == 1)
    lda, ldb = (A.stride(0) if K > 1 else M), (B.stride(0) if K > 1 else N)
    if keyA is not None:
        assert keyA.shape[0] == M and keyA.dtype == torch().int64
    if keyB is not None:
        assert keyB.shape[0] == N and keyB.dtype == torch().int64
    ctx.check(ctx.lib.qk_gemm_keyed_pred(ctx.handle, M, N, K, A.data_ptr(), lda, B.data_ptr(), ldb,
                                         _ptr(keyA), strideA, _ptr(keyB), strideB, out.data_ptr(), beta, _ptr(skip)),
              "qk_gemm_keyed_pred")
    return out


def gemm_outer_paired(ctx: Context, A, B, keyB, keyA=None, out=None, strideA: int = 0):
    """Small-K (K <= 8) keyed outer product ``out[kA(i) + keyB[j]] = sum_k A[k, i] * B[k, j]``,
    output-write bound (``qk_gemm_outer_paired``). ``keyB`` must pair adjacent outputs
    (``keyB[2i+1] == keyB[2i] + 1``, ``keyB[2i]`` even): :func:`paired_keys` says when."""
    K, M = A.shape
    K2, N = B.shape
    assert K == K2 and 1 <= K <= 8 and A.is_contiguous() and B.is_contiguous()
    assert keyB.shape[0] == N and keyB.dtype == torch().int64
    if keyA is not None:
        assert keyA.shape[0] == M and keyA.dtype == torch().int64
    ctx.check(ctx.lib.qk_gemm_outer_paired(ctx.handle, M, N, K, A.data_ptr(), M, B.data_ptr(), N,
                                           _ptr(keyA), strideA, keyB.data_ptr(), out.data_ptr()),
              "qk_gemm_outer_paired")
    return out


def knit_outer_stream(ctx: Context, A, B, clbits_a: list, clbits_b: list, nbits: int, out,
                      o_begin: int = 0, o_count: int | None = None, k_dev=None):
    """Two-fragment small-K knit written in output order (``qk_knit_outer_stream_range``):
    ``out[o - o_begin] = sum_k A[k, pext(o, mask_a)] * B[k, pext(o, mask_b)]`` for
    ``o_begin <= o < o_begin + o_count`` (default: all ``2^nbits``). Needs the fragments' clbits to
    split ``0..nbits-1`` with clbit 0 on the B side (:func:`stream_knit_ok`). ``k_dev`` (device
    int32 tensor): run-time K (0: write nothing)."""
    K, M = A.shape
    K2, N = B.shape
    assert K == K2 and 1 <= K <= 8 and A.is_contiguous() and B.is_contiguous()
    mA, mB = sum(1 << c for c in clbits_a), sum(1 << c for c in clbits_b)
    if o_count is None:
        o_count = (1 << nbits) - o_begin
    assert M == 1 << len(clbits_a) and N == 1 << len(clbits_b) and out.numel() >= o_count
    if k_dev is not None:
        assert k_dev.dtype == torch().int32 and k_dev.device == out.device
    ctx.check(ctx.lib.qk_knit_outer_stream_range(ctx.handle, nbits, K, A.data_ptr(), M, B.data_ptr(), N, mA, mB,
                                                 o_begin, o_count, _ptr(k_dev), out.data_ptr()),
              "qk_knit_outer_stream_range")
    return out


OUTER_STREAM_KERNELS = ("qk_knit_outer_stream_kernel", "qk_knit_outer_blocked_kernel",
                        "qk_knit_outer_blocked_kernel<b_global>", "qk_knit_outer_rows_kernel")


def knit_outer_stream_kernel(K: int, clbits_a: list, clbits_b: list, nbits: int, o_begin: int = 0,
                             o_count: int | None = None) -> str:
    """Name of the kernel :func:`knit_outer_stream` launches for these arguments
    (``qk_knit_outer_stream_kind``): the per-output gather, the blocked kernel with both operands
    staged in LDS, or the blocked kernel reading B from global memory."""
    mA, mB = sum(1 << c for c in clbits_a), sum(1 << c for c in clbits_b)
    if o_count is None:
        o_count = (1 << nbits) - o_begin
    kind, tb = ctypes.c_int(), ctypes.c_int()
    _lib.check(None, _lib.lib().qk_knit_outer_stream_kind(nbits, K, mA, mB, o_begin, o_count, ctypes.byref(kind),
                                                          ctypes.byref(tb)), "qk_knit_outer_stream_kind")
    return OUTER_STREAM_KERNELS[kind.value]


def stream_knit_ok(clbits_a: list, clbits_b: list, nbits: int) -> bool:
    """Whether :func:`knit_outer_stream` applies: the two clbit sets partition ``0..nbits-1``
    (2 <= nbits <= 32), clbit 0 is on the B side, and each list is ascending (the kernels index a
    fragment's outcomes by pext over its clbit mask, which packs bits in ascending order)."""
    a, b = set(clbits_a), set(clbits_b)
    return (2 <= nbits <= 32 and not (a & b) and (a | b) == set(range(nbits)) and 0 in b
            and list(clbits_a) == sorted(a) and list(clbits_b) == sorted(b))


def paired_keys(clbits: list) -> bool:
    """Whether a fragment's output keys (deposit into ascending ``clbits``) pair adjacent
    outputs: true exactly when it holds clbit 0 (then key(2i + 1) = key(2i) + 1, key(2i) even)."""
    return len(clbits) >= 1 and sorted(clbits)[0] == 0


def khatri_rao(ctx: Context, A, B):
    T = torch()
    K, M = A.shape
    _, N = B.shape
    out = T.empty((K, M * N), dtype=T.float64, device=A.device)
    ctx.check(ctx.lib.qk_khatri_rao(ctx.handle, K, M, N, A.data_ptr(), M, B.data_ptr(), N,
                                    out.data_ptr()), "qk_khatri_rao")
    return out


def gather_rows(ctx: Context, src, idx_t, coef_t):
    T = torch()
    R = idx_t.shape[0]
    width = src.shape[1]
    out = T.empty((R, width), dtype=T.float64, device=src.device)
    ctx.check(ctx.lib.qk_gather_rows(ctx.handle, R, width, idx_t.data_ptr(), coef_t.data_ptr(),
                                     src.data_ptr(), out.data_ptr()), "qk_gather_rows")
    return out


# ----------------------------------------------------------------------------- virtual circuits
def clbit_indexer(circuit):
    """Map a clbit of the cut circuit to its global index (cregs in order)."""
    index = {}
    i = 0
    for creg in circuit.cregs:
        for b in creg:
            index[b] = i
            i += 1
    return lambda c: index[c]


@dataclass
class FragmentState:
    fragment: object
    labels: list
    prog: FragmentProgram
    dprog: DeviceProgram | None
    jobs: JobTable | None
    touches: list
    dropped: bool = False  # reference skips fragments whose counts cannot be read (run.py:57-58)
    uidx: np.ndarray | None = None  # label -> row of the deduplicated instance list
    unique_labels: list | None = None
    # basis reduction (factored knit only): the sweep runs `basis_labels`, and unique instance
    # u is `expand[u] @ q_basis` (fragment_program.basis_reduce)
    basis_labels: list | None = None
    expand: np.ndarray | None = None
    # traced qubits beyond what a FINAL tile holds: the device program measures `log2(fold)` of them
    # too (widened outputs) and fold_traced sums them out after the sweep (_device_program)
    fold: int = 1
    # per-program kernels: (compiled, tile bits, FINAL tile bits) as prepare_fragments chose them
    jit: tuple = (False, None, None)

    @property
    def swept_labels(self) -> list:
        if self.basis_labels is not None:
            return self.basis_labels
        return self.unique_labels if self.unique_labels is not None else self.labels

    @property
    def n_rows(self) -> int:
        """Rows of the swept q_f (unique instances, or basis instances)."""
        return len(self.swept_labels)

    def row_of_label(self) -> np.ndarray:
        if self.expand is not None:
            raise ValueError("basis-reduced fragment: labels are combinations of swept rows")
        return self.uidx if self.uidx is not None else np.arange(len(self.labels), dtype=np.int64)


TRACED_MAX = 12 - 5  # traced qubits a SPLIT program's FINAL tile holds (sweep_plan: 12-bit tiles, 5 low bits)


def _device_program(prog: FragmentProgram):
    """``(program the device runs, fold)``. The FINAL pass traces out unmeasured qubits inside its
    tile, so a SPLIT program (n > 12) may trace at most TRACED_MAX of them (sweep_plan.schedule_passes).
    With more, the device program measures the lowest extra ones as well (``m`` widened: they are the
    next state bits above the measured ones) and the output row holds ``fold`` blocks of 2^m values,
    one per extra-bit pattern; :func:`fold_traced` sums them after the sweep (a row reduction)."""
    if prog.n <= 12 or prog.n - prog.m <= TRACED_MAX:
        return prog, 1
    m_w = prog.n - TRACED_MAX
    return dataclasses.replace(prog, m=m_w), 1 << (m_w - prog.m)


_FOLD_OFFS: dict = {}


def fold_traced(ctx: Context, x, fold: int):
    """Rows of a widened sweep output ``[rows, fold * 2^m]`` summed over their ``fold`` blocks ->
    ``[rows, 2^m]`` (qk_reduce_labels over each row's blocks); the identity for ``fold == 1``."""
    if fold <= 1:
        return x
    T = torch()
    rows, w = x.shape
    key = (rows, fold, str(x.device))
    off = _FOLD_OFFS.get(key)
    if off is None:
        off = _FOLD_OFFS[key] = T.arange(rows + 1, dtype=T.int64, device=x.device) * fold
    return reduce_labels(ctx, x.contiguous().view(rows * fold, w // fold), off, rows)


_planning_tls = threading.local()


@contextlib.contextmanager
def host_planning():
    """Context of the host side of planning: endpoint side programs memoised for the plan
    (``fragment_program.planning_memo``) and the BLAS pool held to one thread. The plan's matrices are
    tiny (the two-fragment core is 64 x 256), and a multi-threaded OpenBLAS spends 0.25-0.55 s on that
    one SVD spinning up its pool against 2.5 ms on one thread (measured in the build container)."""
    from .fragment_program import planning_memo

    if getattr(_planning_tls, "depth", 0):  # nested (the pipeline's plan around prepare / operands)
        _planning_tls.depth += 1
        try:
            yield
        finally:
            _planning_tls.depth -= 1
        return
    with contextlib.ExitStack() as st:
        st.enter_context(planning_memo())
        try:
            from threadpoolctl import threadpool_limits

            st.enter_context(threadpool_limits(1, user_api="blas"))  # ~0.5 ms to enter: once per plan
        except ImportError:  # threadpoolctl absent: planning still works, only slower
            pass
        _planning_tls.depth = 1
        try:
            yield
        finally:
            _planning_tls.depth = 0


def prepare_fragments(virt, device: int = 0, upload: bool = True, dedup: bool = True,
                      basis: bool = False, jit: bool | None = None, relevance: bool = True) -> list[FragmentState]:
    with host_planning():
        return _prepare_fragments(virt, device, upload, dedup, basis, jit, relevance)


def _prepare_fragments(virt, device: int, upload: bool, dedup: bool, basis: bool, jit: bool | None,
                       relevance: bool) -> list[FragmentState]:
    """Compile every fragment, dedup its instances and expand them into branch jobs.

    ``basis=True`` (factored knit only) additionally sweeps a spanning set of instances
    (``basis_reduce``, slot channels compared after the exact light-cone projections unless
    ``relevance=False``); the knit transform folds the expansion back in. ``jit``: per-program
    sweep kernels for SPLIT programs — None: only for large sweeps (``_worth_compiling``),
    True: for every SPLIT program of at most 400 ops, False: never (interpreter kernel)."""
    circ = virt.circuit
    cl = clbit_indexer(circ)
    vg = virt.vgate_instructions
    out, want = [], []
    for frag, fcirc in virt.fragment_circuits.items():
        if len(frag) == 0:
            continue
        prog = compile_fragment(fcirc, frag, cl)
        labels = virt.get_instance_labels(frag)
        touches = [bool(set(v.qubits) & set(frag)) for v in vg]
        if dedup:
            unique, uidx = dedup_labels(prog, labels)
        else:
            unique, uidx = list(labels), np.arange(len(labels), dtype=np.int64)
        red = basis_reduce(prog, unique, relevance=relevance) if (basis and dedup) else None
        jobs = build_jobs(prog, red.labels if red is not None else unique)
        # run.py:49-58 drops a fragment whose get_counts() raises, i.e. when some instance of
        # it measures nothing at all (no data measurement and no config measurement).
        dropped = prog.m == 0 and _some_label_unmeasured(prog, labels)
        want.append(_worth_compiling(prog, jobs) if jit is None else (jit and len(prog.ops) <= 400))
        out.append(FragmentState(frag, labels, prog, None, jobs, touches, dropped, uidx, unique,
                                 red.labels if red is not None else None,
                                 red.expand if red is not None else None, _device_program(prog)[1]))
    split = [(fs.prog.n, fs.jobs.n_jobs) for fs, w in zip(out, want) if w and not fs.dropped and fs.prog.n > 12]
    tb = jit_tile_bits(split) if split else JIT_TILE_BITS_MAX
    jit_progs = [_device_program(fs.prog)[0] for fs, w in zip(out, want) if w and not fs.dropped and fs.prog.n > 12]
    ftb = jit_final_tile_bits(jit_progs, tb) if jit_progs else None
    for fs, w in zip(out, want):
        fs.jit = (bool(w and _jit_enabled()), tb, ftb)  # what upload compiles (jit_sources)
        if upload and not fs.dropped:
            fs.dprog = DeviceProgram.upload(_device_program(fs.prog)[0], device, jit=w, tile_bits=tb,
                                            final_tile_bits=ftb)
    return out


JIT_LONG_OPS = 200  # programs this long run op-dispatch bound on the interpreter whatever their batch


def _worth_compiling(prog: FragmentProgram, jobs: JobTable) -> bool:
    """Per-program kernels pay their compile (hiprtc: about 1 s per 70 ops; none when the code object
    is in JIT_CACHE_DIR) on real work: >= 2^22 amplitudes per sweep (at most 400 ops), or a long
    program (>= JIT_LONG_OPS ops: qft 16's 586, one instance, 0.36 ms on the interpreter's 16
    workgroups of serial op dispatch)."""
    return ((jobs.n_jobs << prog.n) >= (1 << 22) and len(prog.ops) <= 400) or len(prog.ops) >= JIT_LONG_OPS


def jit_sources(virt, basis: bool = False, relevance: bool = True) -> list:
    """``[(source, kernel names)]`` of the per-program kernels a plan of ``virt`` compiles (no device:
    the ahead-of-time cache of build()): each compiled fragment's module (upload) and, for 2-4 of
    them on one tile width per pass round, the multi-fragment module (pipeline._plan_multi)."""
    from . import sweep_codegen

    frags = prepare_fragments(virt, upload=False, basis=basis, relevance=relevance)
    encs = []
    for fs in frags:
        want, tb, ftb = fs.jit
        dprog = _device_program(fs.prog)[0]
        if fs.dropped or not want or dprog.n <= 12:
            continue
        encs.append(encode(dprog, tile_bits=tb or JIT_TILE_BITS_MAX, final_tile_bits=ftb))
    out = [sweep_codegen.generate(e) for e in encs]
    rounds = max((len(e.passes) for e in encs), default=0)
    if 2 <= len(encs) <= 4 and all(len({e.pass_tile_bits(r) for e in encs if len(e.passes) > r}) == 1
                                   for r in range(rounds)):
        out.append(sweep_codegen.generate_multi(encs))
    return out


def _some_label_unmeasured(prog: FragmentProgram, labels: list) -> bool:
    from .fragment_program import side_branches

    for label in labels:
        if all(len(side_branches(s.endpoint, label[s.vgate_idx])) == 1 for s in prog.slots):
            return True
    return False


def sweep_fragment(ctx: Context, fs: FragmentState, label_range=None):
    """Signed-folded per-label distributions ``q_f`` of one fragment on the GPU.

    ``label_range=(lo, hi)`` restricts the sweep to fragment labels ``[lo, hi)``
    (multi-GPU sharding); rows are returned for that range only. Rows are the
    swept (deduplicated) instances: ``q[fs.row_of_label()]`` is per label.
    """
    T = torch()
    jobs = fs.jobs
    lo, hi = (0, fs.n_rows) if label_range is None else label_range
    width = 1 << fs.prog.m
    if fs.dropped:
        return T.ones((hi - lo, 1), dtype=T.float64, device=T.device("cuda", ctx.device))
    j0, j1 = int(jobs.label_offsets[lo]), int(jobs.label_offsets[hi])
    sub = JobTable(jobs.slot_mats[j0:j1], jobs.sign[j0:j1], jobs.label_offsets[lo : hi + 1] - j0,
                   jobs.branch_bits[j0:j1])
    slot_t, sign_t, off_t = jobs_to_device(sub, ctx.device)
    if sub.n_jobs != hi - lo and fs.dprog.module is not None:  # branching, compiled: fused FINAL
        return fold_traced(ctx, sweep_labels(ctx, fs.dprog, slot_t, sign_t, sub.n_jobs, off_t, hi - lo)[0], fs.fold)
    pjob, _ = sweep_jobs(ctx, fs.dprog, slot_t, sign_t, sub.n_jobs)
    if sub.n_jobs == hi - lo:  # no branching: jobs are labels
        return fold_traced(ctx, pjob, fs.fold)
    return fold_traced(ctx, reduce_labels(ctx, pjob, off_t, hi - lo), fs.fold)


@dataclass
class KnitOperands:
    """Per-fragment knit operands ``W_f`` (contraction rows) and output clbits."""

    rows: list  # per included fragment: np.int64 [R] row index into q_f
    coefs: list  # per included fragment: np.float64 [R]
    transforms: list  # per fragment: None (gather) or dense [R, L_f] matrix (factored)
    clbits: list  # per included fragment: ascending global clbits of its outcome bits
    num_terms: int
    factored_terms: int = 0  # factored knit: prod r_j before the core compression

    def key_table(self, i: int) -> np.ndarray:
        return deposit_keys(self.clbits[i])


def _affine_stride(clbits: list):
    """Stride if the fragment's clbits are contiguous (key = x << c0), else None."""
    if not clbits:
        return 0
    c0 = clbits[0]
    return (1 << c0) if list(clbits) == list(range(c0, c0 + len(clbits))) else None


def knit_operands(virt, frags: list[FragmentState], factored: bool = False, compress: bool = True) -> KnitOperands:
    with host_planning():
        return _knit_operands(virt, frags, factored, compress)


def _knit_operands(virt, frags: list[FragmentState], factored: bool, compress: bool) -> KnitOperands:
    vg = [v.operation for v in virt.vgate_instructions]
    space = LabelSpace([g.num_instantiations for g in vg], [g.knit_coefficients() for g in vg])
    clbits = [[] if fs.dropped else list(fs.prog.clbits) for fs in frags]
    if not factored or not vg:
        if any(fs.expand is not None for fs in frags):
            raise ValueError("basis-reduced fragments need the factored knit")
        c = space.coefficients()
        rows, coefs = [], []
        for i, fs in enumerate(frags):
            rows.append(fs.row_of_label()[space.fragment_rows(fs.touches)])
            coefs.append(c if i == 0 else np.ones_like(c))
        return KnitOperands(rows, coefs, [None] * len(frags), clbits, space.num_labels)
    # factored: per gate rank factorisation, fragment transform = kron over touching gates
    Ts = []
    for j in range(len(vg)):
        eps = _endpoints(virt, j)
        Ts.append(factor_vgate(eps[0], eps[1], vg[j].knit_coefficients()))
    ranks = [t[0].shape[0] for t in Ts]
    transforms = []
    for fs in frags:
        W = np.ones((1, 1))
        sides = _fragment_sides(virt, fs)
        for j in range(len(vg)):
            if sides[j] is None:
                # gate not touching: its rank index is free on this fragment (ones row per r)
                W = np.kron(W, np.ones((ranks[j], 1)))
            else:
                W = np.kron(W, Ts[j][sides[j]])
        if fs.uidx is not None:  # fold labels sharing an instance: W' = W P
            Wu = np.zeros((W.shape[0], len(fs.unique_labels)))
            np.add.at(Wu.T, fs.uidx, W.T)
            W = Wu
        if fs.expand is not None:  # instances as combinations of the swept basis: W'' = W' E
            W = W @ fs.expand
        transforms.append(W)
    terms = factored_terms = int(np.prod(ranks))
    if compress and len(frags) == 2 and not any(fs.dropped for fs in frags):
        transforms, terms = _compress_core(transforms, terms)
    return KnitOperands([None] * len(frags), [None] * len(frags), transforms, clbits, terms, factored_terms)


def _compress_core(transforms: list, terms: int, tol: float = 1e-10):
    """Two fragments: ``R = A^T B = q_0^T (W_0^T W_1) q_1`` depends on the transforms only
    through the core ``C = W_0^T W_1`` ([swept rows_0, swept rows_1]). With C = U S V^T of rank
    r (the light-cone basis reduction makes it rank-deficient: syc 32 5 has 64 swept rows on
    one side, so r <= 64 < 256 factored terms) the transforms become ``(U_r S_r)^T`` and
    ``V_r^T``: the contraction dimension drops from ``prod r_j`` to r, same R up to rounding."""
    W0, W1 = transforms
    C = W0.T @ W1
    if C.size == 0:
        return transforms, terms
    U, S, Vt = np.linalg.svd(C, full_matrices=False)
    r = int((S > tol * S[0]).sum()) if S.size and S[0] > 0 else 0
    if r == 0 or r >= terms:
        return transforms, terms
    T0, T1 = np.ascontiguousarray((U[:, :r] * S[:r]).T), np.ascontiguousarray(Vt[:r])
    # once per plan: the truncated core against the untruncated product, entry by entry (the per-step
    # probe check compares against operands that already went through this core, so it cannot see
    # this truncation). The dropped part has spectral norm S[r] <= tol S[0], which bounds every entry;
    # anything larger means the SVD went wrong: keep the uncompressed transforms.
    err = float(np.abs(C - T0.T @ T1).max())
    if not err <= 4 * tol * S[0] + 64 * np.finfo(np.float64).eps * float(np.abs(C).max()):
        return transforms, terms
    return [T0, T1], r


def data_rank_factors(GA: np.ndarray, GB: np.ndarray, **kw):
    """Rank factors of a two-fragment knit from its Grams (:func:`data_rank.rank_factors`)."""
    from .data_rank import rank_factors

    return rank_factors(GA, GB, **kw)


def rank_factors_device(ctx: Context, GA, GB, rmax: int = 8, out=None):
    """``qk_rank_factors`` on device Grams: ``(TA, TB, r)`` device tensors ([rmax, K] fp64 twice,
    int32 [1]); no host synchronisation. ``r = 0``: no usable factorisation."""
    from . import data_rank as dr

    T = torch()
    K = GA.shape[0]
    assert GA.shape == (K, K) and GB.shape == (K, K) and GA.is_contiguous() and GB.is_contiguous()
    if out is None:
        out = (T.empty((rmax, K), dtype=T.float64, device=GA.device), T.empty((rmax, K), dtype=T.float64,
                                                                              device=GA.device),
               T.empty(1, dtype=T.int32, device=GA.device))
    TA, TB, r = out
    ctx.check(ctx.lib.qk_rank_factors(ctx.handle, K, GA.data_ptr(), GB.data_ptr(), dr.LAM_TOL, dr.S_TOL, dr.S_ABS,
                                      rmax, TA.data_ptr(), TB.data_ptr(), r.data_ptr()), "qk_rank_factors")
    return TA, TB, r


PREP_COLS = 128  # qk_prep_operands: column counts must be multiples of this
N_PROBES = 16    # probes of the data-rank acceptance check (qk_probe_errors)
_PREP_WORK: dict = {}


def prep_ok(K: int, NA: int, NB: int) -> bool:
    """Whether qk_prep_operands takes these operand shapes (even K <= 64, column counts % 128)."""
    return 2 <= K <= 64 and K % 2 == 0 and NA >= PREP_COLS and NB >= PREP_COLS and NA % PREP_COLS == 0 and NB % PREP_COLS == 0


# QKNIT_POISON_UNUSED=1 (tests): the A2 columns a column-range compression leaves unwritten are set to NaN,
# so a write that read outside its slice's columns shows in the output
POISON_UNUSED = os.environ.get("QKNIT_POISON_UNUSED", "0") == "1"


def prep_operands(ctx: Context, WtA, qA, WtB, qB, probes, out=None):
    """``qk_prep_operands``: ``(XA, XB, G, U)`` — the two light-cone operands ``X = Wt^T q`` ([K, N]
    each), their Grams stacked ``G = [XA XA^T, XB XB^T]`` ([2, K, K]) and ``U = XB probes^T`` ([K, 16]),
    in one pass over the swept rows (plus a fixed-order reduction of per-workgroup partials). ``qA`` /
    ``qB`` may be column windows of wider rows (unit column stride; ldq = their row stride)."""
    T = torch()
    RA, K = WtA.shape
    RB, K2 = WtB.shape
    assert K == K2 and qA.shape[0] == RA and qB.shape[0] == RB and probes.shape[0] == N_PROBES
    NA, NB = qA.shape[1], qB.shape[1]
    assert probes.shape[1] == NB and all(t.is_contiguous() for t in (WtA, WtB, probes))
    assert qA.stride(1) == 1 and qB.stride(1) == 1
    dev = qA.device
    if out is None:
        # G and U share one buffer (views of it, G first): a multi-GPU rank all-reduces them in one call
        gu = T.empty(2 * K * K + K * N_PROBES, dtype=T.float64, device=dev)
        out = (T.empty((K, NA), dtype=T.float64, device=dev), T.empty((K, NB), dtype=T.float64, device=dev),
               gu[:2 * K * K].view(2, K, K), gu[2 * K * K:].view(K, N_PROBES))
    XA, XB, G, U = out
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_prep_workspace_bytes(ctx.handle, NA, NB, ctypes.byref(need)), "qk_prep_workspace_bytes")
    key = (str(dev), T.cuda.current_stream(dev).cuda_stream)
    work = _PREP_WORK.get(key)
    if work is None or work.numel() * 8 < need.value:
        work = _PREP_WORK[key] = T.empty(max(need.value // 8, 1), dtype=T.float64, device=dev)
    ctx.check(ctx.lib.qk_prep_operands(ctx.handle, K, RA, WtA.data_ptr(), qA.data_ptr(), qA.stride(0), NA,
                                       XA.data_ptr(), RB, WtB.data_ptr(), qB.data_ptr(), qB.stride(0), NB,
                                       XB.data_ptr(), probes.data_ptr(), G[0].data_ptr(), G[1].data_ptr(),
                                       U.data_ptr(), work.data_ptr(), work.numel() * 8), "qk_prep_operands")
    return XA, XB, G, U


QPREP_ROWS = 80  # qk_qprep_*: swept rows per side at most
# the q-space preparation where it applies (QKNIT_QPREP=1; default the X path). Measured on syc 32 5 and
# not kept (profiles/r05h_*): its chain took 0.235 ms of kernels against 0.143 for the X
# path (qk_qgram 53 us, qk_qcompress_b 74, qk_qcompress_a 53, qk_qproject 17, + two predicated transforms
# for the exact fallback) and 0.94 vs 0.91 ms per 8-rank pipelined step: the transform it removes (~30 us
# of MFMA) does not pay for the extra launches and the latency-bound VALU compress passes.
QPREP = os.environ.get("QKNIT_QPREP", "0") == "1"
_QPREP_WORK: dict = {}


def qprep_ok(K: int, RA: int, RB: int, NA: int, NB: int) -> bool:
    """Whether the q-space preparation (qk_qprep_grams / qk_qprep_compress_check) takes these shapes:
    K <= 64 terms, at most QPREP_ROWS swept rows per side, column counts multiples of 512."""
    return (QPREP and 1 <= K <= 64 and 1 <= RA <= QPREP_ROWS and 1 <= RB <= QPREP_ROWS and NA >= 512 and NB >= 512
            and NA % 512 == 0 and NB % 512 == 0)


def _qprep_work(ctx: Context, NA: int, NB: int, dev):
    T = torch()
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_qprep_workspace_bytes(ctx.handle, NA, NB, ctypes.byref(need)), "qk_qprep_workspace_bytes")
    key = (str(dev), T.cuda.current_stream(dev).cuda_stream)
    work = _QPREP_WORK.get(key)
    if work is None or work.numel() * 8 < need.value:
        work = _QPREP_WORK[key] = T.empty(max(need.value // 8, 1), dtype=T.float64, device=dev)
    return work


def qprep_grams(ctx: Context, WtA, qA, WtB, qB, probes):
    """``qk_qprep_grams``: ``(G, U)`` — the Grams ``[X_A X_A^T, X_B X_B^T]`` ([2, K, K]) and
    ``U = X_B probes^T`` ([K, 16]) of the light-cone operands ``X = Wt^T q``, without forming X."""
    T = torch()
    RA, K = WtA.shape
    RB, K2 = WtB.shape
    assert K == K2 and qA.shape[0] == RA and qB.shape[0] == RB and probes.shape == (N_PROBES, qB.shape[1])
    assert all(t.is_contiguous() for t in (WtA, qA, WtB, qB, probes))
    NA, NB = qA.shape[1], qB.shape[1]
    dev = qA.device
    gu = T.empty(2 * K * K + K * N_PROBES, dtype=T.float64, device=dev)
    G, U = gu[:2 * K * K].view(2, K, K), gu[2 * K * K:].view(K, N_PROBES)
    work = _qprep_work(ctx, NA, NB, dev)
    ctx.check(ctx.lib.qk_qprep_grams(ctx.handle, K, RA, WtA.data_ptr(), qA.data_ptr(), NA, NA, RB, WtB.data_ptr(),
                                     qB.data_ptr(), NB, NB, probes.data_ptr(), G[0].data_ptr(), G[1].data_ptr(),
                                     U.data_ptr(), work.data_ptr(), work.numel() * 8), "qk_qprep_grams")
    return G, U


def qprep_compress_check(ctx: Context, WtA, qA, WtB, qB, TA, TB, U, probes, r, tol: float, rel_tol: float):
    """``qk_qprep_compress_check``: ``(A2, B2, k, err)`` — the compressed operands ``T Wt^T q`` ([rmax, N])
    and the accepted rank of their probe check (as :func:`probe_errors` with ``r``)."""
    T = torch()
    RA, K = WtA.shape
    RB = WtB.shape[0]
    rmax = TA.shape[0]
    NA, NB = qA.shape[1], qB.shape[1]
    dev = qA.device
    ab = T.empty(rmax * (NA + NB), dtype=T.float64, device=dev)
    A2, B2 = ab[:rmax * NA].view(rmax, NA), ab[rmax * NA:].view(rmax, NB)
    k = T.empty(1, dtype=T.int32, device=dev)
    err = T.empty(1, dtype=T.float64, device=dev)
    work = _qprep_work(ctx, NA, NB, dev)
    ctx.check(ctx.lib.qk_qprep_compress_check(ctx.handle, K, rmax, RA, WtA.data_ptr(), qA.data_ptr(), NA, NA, RB,
                                              WtB.data_ptr(), qB.data_ptr(), NB, NB, TA.data_ptr(), TB.data_ptr(),
                                              U.data_ptr(), probes.data_ptr(), A2.data_ptr(), B2.data_ptr(), None,
                                              r.data_ptr(), tol, rel_tol, k.data_ptr(), err.data_ptr(), work.data_ptr(),
                                              work.numel() * 8), "qk_qprep_compress_check")
    return A2, B2, k, err


def compress_operands(ctx: Context, TA, XA, TB, XB, a_cols: tuple | None = None, a_width: int | None = None):
    """``qk_compress_operands``: ``(TA XA, TB XB)`` ([rmax, N] each) in one launch. ``a_cols = (base, n)``:
    only A2's columns [base, base + n) are computed (the others are left unwritten; qk_compress_operands_ld)
    from XA's columns [base, base + n), or from all of XA when it is that window already ([K, n]; A2 is
    then ``a_width`` wide)."""
    T = torch()
    rmax, K = TA.shape
    assert TB.shape == (rmax, K) and XA.shape[0] == K and XB.shape[0] == K
    assert XA.stride(1) == 1 and XB.is_contiguous() and TA.is_contiguous() and TB.is_contiguous()
    NA = XA.shape[1] if a_width is None else a_width
    NB = XB.shape[1]
    # A2 and B2 share one buffer (A2 first): a multi-GPU rank all-gathers them in one call
    ab = T.empty(rmax * (NA + NB), dtype=T.float64, device=XA.device)
    A2 = ab[:rmax * NA].view(rmax, NA)
    B2 = ab[rmax * NA:].view(rmax, NB)
    if a_cols is None:
        assert XA.is_contiguous() and XA.shape[1] == NA
        ctx.check(ctx.lib.qk_compress_operands(ctx.handle, K, rmax, TA.data_ptr(), XA.data_ptr(), NA, A2.data_ptr(),
                                               TB.data_ptr(), XB.data_ptr(), NB, B2.data_ptr()), "qk_compress_operands")
        return A2, B2
    base, n = a_cols
    assert 0 <= base and n >= 1 and base + n <= NA
    src = XA.data_ptr() if XA.shape[1] == n else XA.data_ptr() + 8 * base
    assert XA.shape[1] in (n, NA)
    if POISON_UNUSED:
        A2.fill_(float("nan"))
    ctx.check(ctx.lib.qk_compress_operands_ld(ctx.handle, K, rmax, TA.data_ptr(), src, n, XA.stride(0),
                                              A2.data_ptr() + 8 * base, NA, TB.data_ptr(), XB.data_ptr(), NB, NB,
                                              B2.data_ptr(), NB), "qk_compress_operands_ld")
    return A2, B2


CV_COLS = 512  # qk_compress_probe_v: columns of B per V partial


def compress_probe_v(ctx: Context, TA, XA, TB, XB, probes, a_cols: tuple | None = None, a_width: int | None = None):
    """``qk_compress_probe_v``: ``(A2, B2, vpart)`` — :func:`compress_operands` (same arithmetic per column,
    ``a_cols`` / ``a_width`` alike) with the probe check's V partials of B2 against ``probes`` formed in
    the same launch ([ceil(NB / 512), 8, 16]); :func:`probe_errors` takes them as ``vpart``."""
    T = torch()
    rmax, K = TA.shape
    assert TB.shape == (rmax, K) and XA.shape[0] == K and XB.shape[0] == K
    assert XA.stride(1) == 1 and XB.is_contiguous() and TA.is_contiguous() and TB.is_contiguous()
    NA = XA.shape[1] if a_width is None else a_width
    NB = XB.shape[1]
    assert probes.is_contiguous() and probes.shape == (N_PROBES, NB)
    ab = T.empty(rmax * (NA + NB), dtype=T.float64, device=XA.device)
    A2 = ab[:rmax * NA].view(rmax, NA)
    B2 = ab[rmax * NA:].view(rmax, NB)
    base, n = (0, NA) if a_cols is None else a_cols
    assert 0 <= base and n >= 1 and base + n <= NA and XA.shape[1] in (n, NA)
    src = XA.data_ptr() if XA.shape[1] == n else XA.data_ptr() + 8 * base
    if a_cols is not None and POISON_UNUSED:
        A2.fill_(float("nan"))
    gv = -(-NB // CV_COLS)
    vpart = T.empty((gv, 8, N_PROBES), dtype=T.float64, device=XA.device)
    ctx.check(ctx.lib.qk_compress_probe_v(ctx.handle, K, rmax, TA.data_ptr(), src, n, XA.stride(0),
                                          A2.data_ptr() + 8 * base, NA, TB.data_ptr(), XB.data_ptr(), NB, NB,
                                          B2.data_ptr(), NB, probes.data_ptr(), NB, vpart.data_ptr(), vpart.numel()),
              "qk_compress_probe_v")
    return A2, B2, vpart


def compress_probe_v_ok(XA, XB, a_cols=None) -> bool:
    """Whether qk_compress_probe_v takes these operands (even widths and strides, 16-B aligned)."""
    n = XA.shape[1] if a_cols is None else a_cols[1]
    base = 0 if a_cols is None or XA.shape[1] == n else a_cols[0]
    return (n % 2 == 0 and XB.shape[1] % 2 == 0 and XA.stride(0) % 2 == 0 and base % 2 == 0
            and (XA.data_ptr() + 8 * base) % 16 == 0 and XB.data_ptr() % 16 == 0)


_PROBE_WORK: dict = {}
def probe_errors(ctx: Context, XA, A2, U, B2, probes, r=None, tol: float = 0.0, a2_cols: tuple | None = None,
                 rel_tol: float = 0.0, tally=None, vpart=None):
    """``qk_probe_errors``: ``e2`` ([32]) = the squared probe errors of the compressed knit ([:16]) and the
    squared reference products ``||R p||^2`` ([16:]) over the columns of ``XA`` ([K, NA]); ``A2`` ([rmax, *])
    holds those columns at ``a2_cols = (offset, count)`` of its rows (default: all). ``U = XB probes^T`` and
    ``B2`` / ``probes`` span all of B's columns. With ``r`` (device int32 [1]) also the accepted rank ``k``
    (error <= max(tol, rel_tol max ||R p||)) and the error: ``(e2, k, err)``, else ``(e2, None, None)``."""
    T = torch()
    K, NA = XA.shape
    rmax = A2.shape[0]
    NB = B2.shape[1]
    assert U.shape == (K, N_PROBES) and probes.shape == (N_PROBES, NB) and B2.shape[0] == rmax
    assert all(t.is_contiguous() for t in (A2, U, B2, probes))
    assert XA.stride(1) == 1 and XA.stride(0) >= NA  # a column range of a wider operand (rows stride(0) apart)
    off = 0 if a2_cols is None else a2_cols[0]
    assert (a2_cols is None and A2.shape[1] == NA) or (a2_cols is not None and a2_cols[1] == NA)
    dev = XA.device
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_probe_workspace_bytes(ctx.handle, NA, ctypes.byref(need)), "qk_probe_workspace_bytes")
    key = (str(dev), T.cuda.current_stream(dev).cuda_stream)
    work = _PROBE_WORK.get(key)
    if work is None or work.numel() * 8 < need.value:
        work = _PROBE_WORK[key] = T.empty(max(need.value // 8, 1), dtype=T.float64, device=dev)
    e2 = T.empty(2 * N_PROBES, dtype=T.float64, device=dev)
    k = T.empty(1, dtype=T.int32, device=dev) if r is not None else None
    err = T.empty(1, dtype=T.float64, device=dev) if r is not None else None
    # tally (device int64[4], with r): the step's data-rank statistics updated by the accept kernel itself
    assert tally is None or (r is not None and tally.dtype == T.int64 and tally.numel() == 4)
    if vpart is not None:  # V partials from qk_compress_probe_v: no pass over B2 and the probes here
        assert vpart.is_contiguous() and vpart.shape[1:] == (8, N_PROBES)
        ctx.check(ctx.lib.qk_probe_errors_vpart(ctx.handle, K, rmax, XA.data_ptr(), XA.stride(0), NA,
                                                A2.data_ptr() + 8 * off, A2.shape[1], U.data_ptr(), vpart.data_ptr(),
                                                vpart.shape[0], e2.data_ptr(), _ptr(r), tol, rel_tol, _ptr(k), _ptr(err),
                                                work.data_ptr(), work.numel() * 8, _ptr(tally)), "qk_probe_errors_vpart")
        return e2, k, err
    ctx.check(ctx.lib.qk_probe_errors_tally(ctx.handle, K, rmax, XA.data_ptr(), XA.stride(0), NA, A2.data_ptr() + 8 * off,
                                            A2.shape[1], U.data_ptr(), B2.data_ptr(), NB, NB, probes.data_ptr(), NB,
                                            e2.data_ptr(), _ptr(r), tol, rel_tol, _ptr(k), _ptr(err), work.data_ptr(),
                                            work.numel() * 8, _ptr(tally)), "qk_probe_errors_tally")
    return e2, k, err


def probe_accept(ctx: Context, e2, r, tol: float, rel_tol: float = 0.0):
    """``qk_probe_accept``: ``(k, err)`` from summed ``e2`` rows ([32]: squared errors, squared references)."""
    T = torch()
    k = T.empty(1, dtype=T.int32, device=e2.device)
    err = T.empty(1, dtype=T.float64, device=e2.device)
    ctx.check(ctx.lib.qk_probe_accept(ctx.handle, e2.data_ptr(), 1, r.data_ptr(), tol, rel_tol, k.data_ptr(),
                                      err.data_ptr()), "qk_probe_accept")
    return k, err


def _endpoints(virt, j):
    out = [None, None]
    for instr in virt.circuit:
        op = instr.operation
        if getattr(op, "vgate_idx", None) == j:
            out[op.qubit_idx] = op
    return out


def factored_ok(virt) -> bool:
    """Whether the factored knit (per-gate rank factors split between two fragments, basis reduction
    on each fragment's slots) applies: every virtual gate joins two different fragments. A gate with
    both endpoints in one fragment (allowed by the reference's label logic, vc:39-48,50-68) takes
    the direct knit over all global labels instead."""
    frag_of = {}
    for frag in virt.fragment_circuits:
        for q in frag:
            frag_of[q] = frag
    for instr in virt.vgate_instructions:
        a, b = instr.qubits[0], instr.qubits[1]
        if frag_of.get(a) is frag_of.get(b):
            return False
    return True


def _fragment_sides(virt, fs: FragmentState):
    sides = [None] * len(virt.vgate_instructions)
    members = set(fs.fragment)
    for instr in virt.circuit:
        op = instr.operation
        if hasattr(op, "vgate_idx") and instr.qubits[0] in members:
            if sides[op.vgate_idx] is not None:
                raise NotImplementedError("both sides of a virtual gate in one fragment")
            sides[op.vgate_idx] = op.qubit_idx
    return sides


def fragment_operands(ctx: Context, ops: KnitOperands, qs: list) -> list:
    """Contraction-ready operands ``[num_terms, 2^m_f]`` per fragment (coefficients folded)."""
    T = torch()
    dev = T.device("cuda", ctx.device)
    mats = []
    for i, q in enumerate(qs):
        q = q.contiguous()
        if ops.transforms[i] is not None:
            W = T.from_numpy(np.ascontiguousarray(ops.transforms[i].T)).to(dev)  # [L_f, R]
            a = T.empty((W.shape[1], q.shape[1]), dtype=T.float64, device=dev)
            gemm_keyed(ctx, W, q, out=a, strideA=q.shape[1])
        else:
            idx_t = T.from_numpy(ops.rows[i]).to(dev)
            coef_t = T.from_numpy(ops.coefs[i]).to(dev)
            a = gather_rows(ctx, q, idx_t, coef_t)
        mats.append(a)
    return mats


def plan_transforms(ops: KnitOperands, frags: list) -> list:
    """Per fragment the dense transform ``W_f`` ([swept rows, terms]) of the contraction:
    ``X_f = W_f^T q_f`` (``qk_knit_plan.transforms``). Factored knits carry it already; the direct
    knit's label gather + coefficients become a 0/coef matrix."""
    out = []
    for i, fs in enumerate(frags):
        if ops.transforms[i] is not None:
            out.append(np.ascontiguousarray(ops.transforms[i].T))
            continue
        W = np.zeros((fs.n_rows if not fs.dropped else 1, ops.num_terms))
        W[ops.rows[i], np.arange(ops.num_terms)] = ops.coefs[i]
        out.append(W)
    return out


def knit_plan_c(ctx: Context, virt, frags: list, qs: list, factored: bool = False, out=None):
    """The whole knit through the plan-level C entry ``qk_knit`` (include/qknit.h): what a
    non-Python host calls with the planner's transforms and masks. Same result as
    :func:`knit_dense` (its exact contraction)."""
    T = torch()
    dev = T.device("cuda", ctx.device)
    ops = knit_operands(virt, frags, factored)
    N = virt.circuit.num_clbits
    Ws = [T.from_numpy(W).to(dev) for W in plan_transforms(ops, frags)]
    nf = len(frags)
    rows = (ctypes.c_int64 * nf)(*[W.shape[0] for W in Ws])
    masks = (ctypes.c_uint64 * nf)(*[sum(1 << c for c in cl) for cl in ops.clbits])
    tp = (ctypes.c_void_p * nf)(*[W.data_ptr() for W in Ws])
    plan = _lib.QkKnitPlan(nf, N, ops.num_terms, ctypes.cast(rows, ctypes.POINTER(ctypes.c_int64)),
                           ctypes.cast(masks, ctypes.POINTER(ctypes.c_uint64)),
                           ctypes.cast(tp, ctypes.POINTER(ctypes.c_void_p)))
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_knit_workspace_bytes(ctypes.byref(plan), ctypes.byref(need)), "qk_knit_workspace_bytes")
    ws = T.empty(max(need.value, 1), dtype=T.uint8, device=dev)
    if out is None:
        out = T.zeros(1 << N, dtype=T.float64, device=dev)
    qc = [q.contiguous() for q in qs]
    qp = (ctypes.c_void_p * nf)(*[q.data_ptr() for q in qc])
    ctx.check(ctx.lib.qk_knit(ctx.handle, ctypes.byref(plan), qp, ws.data_ptr(), ws.numel(), out.data_ptr()), "qk_knit")
    torch().cuda.current_stream(ctx.device).synchronize()  # Ws / ws / qc die with this frame
    return out


def knit_lowrank_c(ctx: Context, pipe, qs: list, out=None, rank_tol: float | None = None,
                   rank_tol_rel: float | None = None):
    """The single-GPU data-rank knit through the one-call C entry ``qk_knit_lowrank`` (what a host
    that is not Python calls) with a pipeline's plan: its device transforms, clbit
    masks, probes and tolerances. Returns ``(out [2^N], accepted rank: device int32 [1])``."""
    from . import data_rank as dr

    T = torch()
    ia, ib = pipe.order[0], pipe.order[-1]
    WA, WB = pipe.transforms[ia], pipe.transforms[ib]
    assert WA is not None and WB is not None, "qk_knit_lowrank needs the factored (transform) knit"
    qa, qb = qs[ia].contiguous(), qs[ib].contiguous()
    probes = pipe._probes(qb.shape[1], qb.device)
    plan = _lib.QkLowrankPlan(pipe.N, WA.shape[1], WA.shape[0], WB.shape[0],
                              sum(1 << c for c in pipe.ops.clbits[ia]), sum(1 << c for c in pipe.ops.clbits[ib]),
                              WA.data_ptr(), WB.data_ptr(), probes.data_ptr(), dr.LAM_TOL, dr.S_TOL, dr.S_ABS,
                              pipe.rank_tol if rank_tol is None else rank_tol,
                              pipe.rank_tol_rel if rank_tol_rel is None else rank_tol_rel)
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_knit_lowrank_workspace_bytes(ctx.handle, ctypes.byref(plan), ctypes.byref(need)),
              "qk_knit_lowrank_workspace_bytes")
    ws = T.empty(max(need.value, 1), dtype=T.uint8, device=qa.device)
    if out is None:
        out = T.empty(1 << pipe.N, dtype=T.float64, device=qa.device)
    rank = T.empty(1, dtype=T.int32, device=qa.device)
    ctx.check(ctx.lib.qk_knit_lowrank(ctx.handle, ctypes.byref(plan), qa.data_ptr(), qb.data_ptr(), ws.data_ptr(),
                                      ws.numel(), out.data_ptr(), rank.data_ptr()), "qk_knit_lowrank")
    torch().cuda.current_stream(ctx.device).synchronize()  # ws dies with this frame
    return out, rank


class Comm:
    """An RCCL communicator owned through the C ABI (``qk_comm_init``): the collectives a host that
    is not Python uses for the multi-GPU knit; tests drive them through ctypes."""

    def __init__(self, ctx: Context, uid: bytes, nranks: int, rank: int):
        self.ctx = ctx
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        ctx.check(ctx.lib.qk_comm_init(ctx.handle, buf, nranks, rank, ctypes.byref(h)), "qk_comm_init")
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        _lib.check(None, _lib.lib().qk_comm_unique_id(buf), "qk_comm_unique_id")
        return bytes(buf)

    def allreduce(self, send, recv):
        self.ctx.check(self.ctx.lib.qk_allreduce(self.ctx.handle, self.handle, send.data_ptr(), recv.data_ptr(),
                                                 send.numel()), "qk_allreduce")

    def reduce(self, send, recv, root: int = 0):
        self.ctx.check(self.ctx.lib.qk_reduce(self.ctx.handle, self.handle, send.data_ptr(), _ptr(recv), send.numel(),
                                              root), "qk_reduce")

    def allgather(self, send, recv):
        self.ctx.check(self.ctx.lib.qk_allgather(self.ctx.handle, self.handle, send.data_ptr(), recv.data_ptr(),
                                                 send.numel()), "qk_allgather")

    def alltoall(self, send, recv, nranks: int):
        self.ctx.check(self.ctx.lib.qk_alltoall(self.ctx.handle, self.handle, send.data_ptr(), recv.data_ptr(),
                                                send.numel() // nranks), "qk_alltoall")

    def close(self):
        if self.handle:
            self.ctx.lib.qk_comm_destroy(self.handle)
            self.handle = None


def knit_dense(ctx: Context, virt, frags: list[FragmentState], qs: list, out=None,
               factored: bool = False, num_clbits: int | None = None, row_block=None):
    """Dense knit on the GPU: returns the float64 distribution over all meas clbits.

    ``row_block=(lo, hi)`` computes only columns ``[lo, hi)`` of the first
    contraction operand (output-sharded multi-GPU knit); other keys stay untouched.
    """
    T = torch()
    dev = T.device("cuda", ctx.device)
    N = virt.circuit.num_clbits if num_clbits is None else num_clbits
    ops = knit_operands(virt, frags, factored)
    if out is None:
        out = T.zeros(1 << N, dtype=T.float64, device=dev)
    mats = fragment_operands(ctx, ops, qs)
    if not mats:
        c = T.from_numpy(LabelSpace([g.operation.num_instantiations for g in virt.vgate_instructions],
                                    [g.operation.knit_coefficients() for g in virt.vgate_instructions]
                                    ).coefficients()).to(dev)
        out[0] = c.sum()
        return out
    return contract(ctx, mats, ops.clbits, out, row_block)


def contract_order(clbits: list) -> list:
    """Fragment order for the contraction: the one holding the lowest clbit goes last
    (it becomes the GEMM's N axis, whose 16 consecutive outcomes land on one 128-B run)."""
    return sorted(range(len(clbits)), key=lambda i: -(min(clbits[i]) if clbits[i] else 1 << 62))


_KEY_CACHE: dict = {}


def _device_keys(clbits: tuple, lo, hi, dev):
    """Output keys of a fragment's outcomes (deposit of x into its clbit positions), rows
    [lo, hi), as a device tensor. Cached: a pipeline step must not rebuild them on the host."""
    key = (clbits, lo, hi, str(dev))
    k = _KEY_CACHE.get(key)
    if k is None:
        T = torch()
        st = _affine_stride(list(clbits))
        if st is not None:
            lo_, hi_ = (0, 1 << len(clbits)) if lo is None else (lo, hi)
            k = T.arange(lo_, hi_, dtype=T.int64, device=dev) * st
        else:
            k = T.from_numpy(deposit_keys(list(clbits))).to(dev)
            if lo is not None:
                k = k[lo:hi].contiguous()
        if len(_KEY_CACHE) > 64:
            _KEY_CACHE.clear()
        _KEY_CACHE[key] = k
    return k


def contract(ctx, mats: list, clbits: list, out, row_block=None, gemm=None, kr=None):
    """Dense contraction of the per-fragment operands into `out` (see knit_dense).

    `gemm(A, B, **kw)` / `kr(A, B)` default to the HIP kernels of `ctx`.
    """
    gemm = gemm or (lambda A, B, **kw: gemm_keyed(ctx, A, B, **kw))
    kr = kr or (lambda A, B: khatri_rao(ctx, A, B))
    T = torch()
    dev = out.device
    order = contract_order(clbits)
    mats = [mats[i] for i in order]
    cls = [clbits[i] for i in order]

    def key_arg(c, lo=None, hi=None):
        st = _affine_stride(c)
        if st is not None and lo is None:
            return None, st
        return _device_keys(tuple(c), lo, hi, dev), 0

    if len(mats) == 1:
        A = mats[0]
        if row_block is not None:
            lo, hi = row_block
            A = A[:, lo:hi].contiguous()
            kA, sA = key_arg(cls[0], lo, hi)
        else:
            kA, sA = key_arg(cls[0])
        ones = T.ones((A.shape[0], 1), dtype=T.float64, device=dev)
        return gemm(A.contiguous(), ones, keyA=kA, strideA=sA, keyB=None, strideB=0, out=out)
    A = mats[0]
    if len(mats) > 2:
        kA = _device_keys(tuple(cls[0]), None, None, dev)
        for B, c in zip(mats[1:-1], cls[1:-1]):
            A = kr(A.contiguous(), B.contiguous())
            kB = _device_keys(tuple(c), None, None, dev)
            kA = (kA.view(1, -1) + kB.view(-1, 1)).reshape(-1)  # index i + j*M
        sA = 0
        if row_block is not None:
            lo, hi = row_block
            A, kA = A[:, lo:hi], kA[lo:hi].contiguous()
    elif row_block is not None:
        lo, hi = row_block
        A = A[:, lo:hi]
        kA, sA = key_arg(cls[0], lo, hi)
    else:
        kA, sA = key_arg(cls[0])
    B = mats[-1]
    kB, sB = key_arg(cls[-1])
    return gemm(A.contiguous(), B.contiguous(), keyA=kA, strideA=sA, keyB=kB, strideB=sB, out=out)


def nearest_probability_distribution(ctx: Context, dense, accuracy: float):
    """Reference-shaped result of a dense distribution, computed on the GPU.

    ``QuasiDistr`` truncation (``|v| > accuracy``, ``quasi_distr.py:7-10``) followed by
    ``nearest_probability_distribution`` (``quasi_distr.py:28-43``): returns
    ``(keys, values)`` host arrays in ascending value order (the reference dict's order).
    """
    T = torch()
    dense = dense.contiguous().view(-1)
    n = dense.numel()
    dev = dense.device
    ws_small = ctypes.c_int64()
    ctx.check(ctx.lib.qk_npd_workspace_bytes(n, 0, ctypes.byref(ws_small)), "qk_npd_workspace_bytes")
    ws = T.empty(max(ws_small.value, 1), dtype=T.uint8, device=dev)
    cnt = T.zeros(1, dtype=T.int64, device=dev)
    ctx.check(ctx.lib.qk_threshold_count(ctx.handle, n, dense.data_ptr(), float(accuracy), ws.data_ptr(),
                                         ws.numel(), cnt.data_ptr()), "qk_threshold_count")
    count = int(cnt.item())
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_npd_workspace_bytes(n, count, ctypes.byref(need)), "qk_npd_workspace_bytes")
    if need.value > ws.numel():
        ws = T.empty(need.value, dtype=T.uint8, device=dev)
    keys = T.empty(max(count, 1), dtype=T.int64, device=dev)
    vals = T.empty(max(count, 1), dtype=T.float64, device=dev)
    n_out = T.zeros(1, dtype=T.int64, device=dev)
    ctx.check(ctx.lib.qk_npd(ctx.handle, n, dense.data_ptr(), float(accuracy), count, ws.data_ptr(), ws.numel(),
                             keys.data_ptr(), vals.data_ptr(), n_out.data_ptr()), "qk_npd")
    k = int(n_out.item())
    return keys[:k].cpu().numpy(), vals[:k].cpu().numpy()


def knit_select(ctx: Context, A, B, clbits_a: list, clbits_b: list, nbits: int, accuracy: float, k_dev=None,
                capacity: int | None = None):
    """``qk_knit_select``: the entries ``|v| > accuracy`` of the two-fragment knit
    ``v[pdep(i, A bits) | pdep(j, B bits)] = sum_k A[k][i] B[k][j]`` (K <= 8), never forming the
    dense vector; tiles bounded below ``accuracy`` are skipped whole. Returns device ``(keys, vals)``
    in unspecified order (bit-identical values to the dense write). One host read of the count;
    reruns with exactly enough room when the first capacity was short."""
    T = torch()
    K = A.shape[0]
    # row-major operands; a column range of wider ones (a rank's slice) passes its row stride
    assert B.shape[0] == K and 1 <= K <= 8 and (A.stride(1) == 1 or A.shape[1] == 1) and (
        B.stride(1) == 1 or B.shape[1] == 1)
    lda, ldb = (A.stride(0) if K > 1 else A.shape[1]), (B.stride(0) if K > 1 else B.shape[1])
    mA, mB = sum(1 << c for c in clbits_a), sum(1 << c for c in clbits_b)
    dev = A.device
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_knit_select_workspace_bytes(nbits, mA, mB, ctypes.byref(need)),
              "qk_knit_select_workspace_bytes")
    work = T.empty(max(need.value // 8, 1), dtype=T.float64, device=dev)
    cnt = T.empty(1, dtype=T.int64, device=dev)
    cap = min(1 << nbits, 1 << 20) if capacity is None else capacity
    while True:
        keys = T.empty(max(cap, 1), dtype=T.int64, device=dev)
        vals = T.empty(max(cap, 1), dtype=T.float64, device=dev)
        ctx.check(ctx.lib.qk_knit_select(ctx.handle, nbits, K, A.data_ptr(), lda, B.data_ptr(), ldb,
                                         mA, mB, float(accuracy), _ptr(k_dev), work.data_ptr(), work.numel() * 8,
                                         cap, keys.data_ptr(), vals.data_ptr(), cnt.data_ptr()), "qk_knit_select")
        n = int(cnt.item())
        if n <= cap:
            return keys[:n], vals[:n]
        cap = n


def select_above(ctx: Context, dense, accuracy: float, key_base: int = 0):
    """``qk_select_above``: device ``(keys, vals)`` of the entries ``|v| > accuracy`` of a dense vector
    (keys = index + ``key_base``), unordered. One host read of the count; reruns with exactly enough
    room when the first capacity was short."""
    T = torch()
    dense = dense.contiguous().view(-1)
    n, dev = dense.numel(), dense.device
    cnt = T.empty(1, dtype=T.int64, device=dev)
    cap = min(n, 1 << 20)
    while True:
        keys = T.empty(max(cap, 1), dtype=T.int64, device=dev)
        vals = T.empty(max(cap, 1), dtype=T.float64, device=dev)
        ctx.check(ctx.lib.qk_select_above(ctx.handle, n, dense.data_ptr(), float(accuracy), int(key_base), cap,
                                          keys.data_ptr(), vals.data_ptr(), cnt.data_ptr()), "qk_select_above")
        k = int(cnt.item())
        if k <= cap:
            return keys[:k], vals[:k]
        cap = k


def npd_pairs(ctx: Context, keys, vals):
    """``qk_npd_pairs``: ``nearest_probability_distribution`` (quasi_distr.py:28-43) of already
    truncated (key, value) pairs on the GPU; host ``(keys, values)`` ascending by value."""
    T = torch()
    n = keys.numel()
    dev = keys.device
    need = ctypes.c_int64()
    ctx.check(ctx.lib.qk_npd_pairs_workspace_bytes(n, ctypes.byref(need)), "qk_npd_pairs_workspace_bytes")
    ws = T.empty(max(need.value, 1), dtype=T.uint8, device=dev)
    ok = T.empty(max(n, 1), dtype=T.int64, device=dev)
    ov = T.empty(max(n, 1), dtype=T.float64, device=dev)
    n_out = T.zeros(1, dtype=T.int64, device=dev)
    ctx.check(ctx.lib.qk_npd_pairs(ctx.handle, n, keys.contiguous().data_ptr(), vals.contiguous().data_ptr(),
                                   ws.data_ptr(), ws.numel(), ok.data_ptr(), ov.data_ptr(), n_out.data_ptr()),
              "qk_npd_pairs")
    k = int(n_out.item())
    return ok[:k].cpu().numpy(), ov[:k].cpu().numpy()


def hellinger_sums(ctx: Context, p, q):
    """``qk_hellinger``: device [3] = (sum sqrt(p q), sum p, sum q) over non-negative parts; the
    partial sums of disjoint shards add (multi-GPU fidelity: all_reduce, then the formula)."""
    T = torch()
    assert p.numel() == q.numel()
    acc = T.zeros(3, dtype=T.float64, device=p.device)
    if p.numel():
        ctx.check(ctx.lib.qk_hellinger(ctx.handle, p.numel(), p.contiguous().data_ptr(), q.contiguous().data_ptr(),
                                       acc.data_ptr()), "qk_hellinger")
    return acc


def fidelity_from_sums(s: float, sp: float, sq: float) -> float:
    return 0.0 if sp <= 0 or sq <= 0 else float((s / np.sqrt(sp * sq)) ** 2)


def hellinger_fidelity(ctx: Context, p, q) -> float:
    """Hellinger fidelity of two dense distributions (qiskit ``hellinger_fidelity``, as used at
    ``Utilities.py:222-224``): ``(sum sqrt(p q) / sqrt(sum p sum q))^2`` with negatives clipped."""
    s, sp, sq = hellinger_sums(ctx, p, q).cpu().numpy().tolist()
    if sp <= 0 or sq <= 0:
        return 0.0
    return float((s / np.sqrt(sp * sq)) ** 2)


def knit_quasi_distrs(virt, results: dict, device: int = 0, factored: bool = False):
    """GPU knit of reference-shaped inputs ``{fragment: [QuasiDistr per label]}``.

    Config bits (``N + j``) are folded with sign ``(-1)^m`` and fragment keys
    are compressed to the fragment's measured clbits before the dense knit.
    Fragments absent from ``results`` are treated as the reference does
    (skipped = contribute a factor 1).
    """
    T = torch()
    ctx = get_context(device)
    N = virt.circuit.num_clbits
    circ = virt.circuit
    cl = clbit_indexer(circ)
    vg = virt.vgate_instructions
    frags, qs = [], []
    for frag, distrs in results.items():
        fcirc = virt.fragment_circuits[frag]
        prog = compile_fragment(fcirc, frag, cl)
        labels = virt.get_instance_labels(frag)
        if len(distrs) != len(labels):
            raise ValueError(f"fragment {frag}: {len(distrs)} results for {len(labels)} labels")
        clbits = prog.clbits
        width = 1 << len(clbits)
        q = np.zeros((len(labels), width), dtype=np.float64)
        pos = {c: i for i, c in enumerate(clbits)}
        for li, d in enumerate(distrs):
            for key, val in d.items():
                data, cfg = key & ((1 << N) - 1), key >> N
                x = 0
                b = data
                while b:
                    low = b & -b
                    c = low.bit_length() - 1
                    if c not in pos:
                        raise ValueError(f"key {key} sets clbit {c} not measured by fragment")
                    x |= 1 << pos[c]
                    b ^= low
                q[li, x] += (-1.0) ** bin(cfg).count("1") * val
        touches = [bool(set(v.qubits) & set(frag)) for v in vg]
        frags.append(FragmentState(frag, labels, prog, None, None, touches))
        qs.append(T.from_numpy(q).to(T.device("cuda", device)))
    out = knit_dense(ctx, virt, frags, qs, factored=factored)
    return out
