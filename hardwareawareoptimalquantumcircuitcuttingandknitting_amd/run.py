"""``run_virtual_circuit``: the knitting hot path, MI355X-native.

Drop-in for ``third_party/qvm/qvm/run.py:23-71``: same name, same arguments,
same return shape ``(dict[int, float], RunTimeInfo)``. Differences, by design:

* by default instances are simulated exactly (fp64 statevector, HIP) instead of
  being sampled with ``shots`` (``run.py:42``); ``sample=True`` draws ``shots``
  outcomes per instance label from the exact distributions on the GPU
  (``engine.sample_fragment``: counter-based stream, ``seed``) and applies
  ``from_counts``' truncation, as the reference's Aer path does; fragments whose
  backend was replaced by a foreign (e.g. qiskit-aer) backend are run through the
  reference's own counts path;
* the knit is one dense fp64 MFMA contraction; ``QuasiDistr``'s ``ACCURACY``
  truncation is applied once to the final distribution instead of after every
  intermediate dict operation, then ``nearest_probability_distribution``
  (``quasi_distr.py:28-43``) as the reference does at ``run.py:71``;
* ``dense=True`` returns the full distribution as a device tensor (needed for
  32-bit outputs: 2^32 fp64 = 34.4 GB cannot be a Python dict).

Timing split (``RunTimeInfo``) follows ``run.py:35,60,65-67``: ``run_time``
covers instance preparation + simulation, ``knit_time`` the contraction.
"""
from __future__ import annotations

import hashlib
import logging
import threading
from collections import OrderedDict
from dataclasses import dataclass
from time import perf_counter

import numpy as np

from . import engine
from . import quasi_distr as _qd
from .backend import MI355XBackend
from .quasi_distr import QuasiDistr
from .virtual_circuit import VirtualCircuit, generate_instantiations

log = logging.getLogger(__name__)


@dataclass
class RunTimeInfo:
    run_time: float
    knit_time: float
    # multi-GPU runs: (first output, outputs) of this rank's contiguous share of the distribution
    shard: tuple | None = None


def _sync(device: int) -> None:
    engine.torch().cuda.synchronize(device)


def _foreign_fragment(virt: VirtualCircuit, fs: engine.FragmentState, backend, shots: int, device: int):
    """Reference counts path for a fragment bound to a non-MI355X backend (run.py:36-58)."""
    T = engine.torch()
    N = virt.circuit.num_clbits
    circuits = generate_instantiations(virt.fragment_circuits[fs.fragment], fs.labels)
    counts = backend.run(circuits, shots=shots).result().get_counts()
    counts = [counts] if isinstance(counts, dict) else counts
    pos = {c: i for i, c in enumerate(fs.prog.clbits)}
    q = np.zeros((len(fs.labels), 1 << len(pos)), dtype=np.float64)
    for li, c in enumerate(counts):
        for key, val in QuasiDistr.from_counts(c).items():
            data, cfg = key & ((1 << N) - 1), key >> N
            x = 0
            while data:
                low = data & -data
                x |= 1 << pos[low.bit_length() - 1]
                data ^= low
            q[li, x] += (-1.0) ** bin(cfg).count("1") * val
    return T.from_numpy(q).to(T.device("cuda", device))


def _direct_dense(virt: VirtualCircuit, shots: int, device: int, factored: bool, out, sample: bool, seed: int):
    """Sweep (or shot-sample) + knit without a cached plan: sampled runs, foreign backends and the
    explicit ``factored=True/False`` knits of ``engine.knit_dense``."""
    ctx = engine.get_context(device)
    # The factored knit folds labels whose side programs coincide into one operand row; sampled
    # labels differ in their shots even then, so sampling knits directly over the labels.
    factored = factored and not sample and engine.factored_ok(virt)
    now = perf_counter()
    native = all(isinstance(virt.get_backend(f), MI355XBackend) for f in virt.fragment_circuits if len(f))
    frags = engine.prepare_fragments(virt, device, basis=factored and native and not sample)
    qs = []
    for i, fs in enumerate(frags):
        backend = virt.get_backend(fs.fragment)
        if isinstance(backend, MI355XBackend) and not sample:
            qs.append(engine.sweep_fragment(ctx, fs))
            continue
        if isinstance(backend, MI355XBackend):
            qs.append(engine.sample_fragment(ctx, fs, shots, engine.fragment_seed(seed, i), _qd.ACCURACY))
        else:
            qs.append(_foreign_fragment(virt, fs, backend, shots, device))
        frags[i] = engine.label_rows(fs)  # one q row per reference label
    _sync(device)
    run_time = perf_counter() - now
    now = perf_counter()
    dense = engine.knit_dense(ctx, virt, frags, qs, out=out, factored=factored)
    _sync(device)
    knit_time = perf_counter() - now
    return dense, RunTimeInfo(run_time, knit_time)


# ---------------------------------------------------------------------------- plan cache
PLAN_CACHE_SIZE = 4  # compiled plans kept (LRU), per (circuit fingerprint, device, thread)
PLAN_CACHE_MAX_BYTES = 16 << 30  # plans holding more device memory (a 32-qubit uncut sweep: 100 GB) are not kept
PLAN_CACHE_TOTAL_BYTES = 32 << 30  # device bytes all cached plans may hold together (LRU eviction beyond)
_PLANS: OrderedDict = OrderedDict()
_PLANS_LOCK = threading.Lock()


def _param_key(p):
    """A parameter as hashed by circuit_fingerprint: arrays by dtype, shape and bytes (their repr
    rounds to 8 digits and elides long arrays), everything else by repr."""
    if isinstance(p, np.ndarray):
        return ("nd", p.dtype.str, p.shape, hashlib.sha1(np.ascontiguousarray(p).tobytes()).hexdigest())
    return repr(p)


def circuit_fingerprint(virt: VirtualCircuit) -> str:
    """Content hash of a cut circuit as the sweep and knit see it: every fragment circuit's
    operations (name, parameters, qubit and global clbit positions; for virtual-gate endpoints the
    gate type, its parameters and the endpoint side) and the output width. Two ``VirtualCircuit``
    objects built from the same cut share it, so a repeated ``run_virtual_circuit`` reuses the
    compiled plan. Cached on the ``VirtualCircuit`` per mutation generation (``_generation``) only:
    the caller's circuit can be edited in place between calls (``cut.data[i] = ...`` keeps the list
    and its length), so every new ``VirtualCircuit`` hashes its fragments again — when it is built
    (``VirtualCircuit.__init__``; syc 32 5: ~1.3 ms of the ~6 ms construction in the build container),
    as the reference builds one per call (``Utilities.py:74-79``)."""
    gen = getattr(virt, "_generation", 0)
    cached = getattr(virt, "_qk_fingerprint", None)
    if cached is not None and cached[0] == gen:
        return cached[1]
    h = hashlib.sha1()
    circ = virt.circuit
    h.update(repr((circ.num_qubits, circ.num_clbits, len(virt.vgate_instructions))).encode())
    for frag, fcirc in virt.fragment_circuits.items():
        h.update(repr(("frag", frag.name, len(frag))).encode())
        for instr in fcirc:
            op = instr.operation
            item = [op.name, tuple(_param_key(p) for p in getattr(op, "params", ())),
                    tuple(fcirc.find_qubit(q) for q in instr.qubits), tuple(fcirc.find_clbit(c) for c in instr.clbits)]
            vg = getattr(op, "_virtual_gate", None)
            if vg is not None:
                item += [op.vgate_idx, op.qubit_idx, type(vg).__name__,
                         tuple(_param_key(p) for p in getattr(vg, "_params", getattr(vg, "params", ())))]
            h.update(repr(item).encode())
    fp = h.hexdigest()
    virt._qk_fingerprint = (gen, fp)
    return fp


def _build_plan(virt: VirtualCircuit, device: int):
    """The benchmarked engine (bench.py): factored knit with light-cone basis + rank-compressed core
    and the per-step device data rank (``pipeline.KnitPipeline``). A circuit the
    factored planner refuses (a virtual gate with both endpoints in one fragment) gets the direct
    knit over all global labels through the same pipeline (``engine.factored_ok``)."""
    from .pipeline import KnitPipeline

    if not engine.factored_ok(virt):
        log.info("a virtual gate with both endpoints in one fragment: direct knit")
        return KnitPipeline(virt, device=device, factored=False)
    return KnitPipeline(virt, device=device, factored=True)


def cached_plan(virt: VirtualCircuit, device: int = 0, group=None, backend=None):
    """The compiled plan (``KnitPipeline``) of ``virt`` on ``device`` for the calling thread: built on
    the first call, reused while the circuit's fingerprint is unchanged (LRU of PLAN_CACHE_SIZE;
    plans above PLAN_CACHE_MAX_BYTES of device buffers are rebuilt per call instead).
    Plans are per thread: a plan owns its sweep buffers, and the reference calls
    ``run_virtual_circuit`` from concurrent threads (``Utilities.py:85-89``). ``group`` (a
    ``torch.distributed`` process group, or ``"WORLD"``): this rank's plan of the multi-GPU run
    (:func:`_build_sharded_plan`), keyed by the group as well. ``backend``: a pipeline backend other
    than the HIP one (CPU tests), part of the key."""
    key = (circuit_fingerprint(virt), device, threading.get_ident())
    if group is not None:
        import torch.distributed as dist

        g = None if group == "WORLD" else group
        gid = "WORLD" if g is None else (getattr(g, "group_name", None) or id(g))
        key += ("sharded", gid, dist.get_rank(g), dist.get_world_size(g))
    if backend is not None:
        key += ("backend", id(backend))
    with _PLANS_LOCK:
        pipe = _PLANS.get(key)
        if pipe is not None:
            _PLANS.move_to_end(key)
            pipe.plan_reused = True
            return pipe
    if group is None:
        pipe = _build_plan(virt, device)
    else:
        pipe = _build_sharded_plan(virt, device, None if group == "WORLD" else group, backend)
    pipe.plan_reused = False
    if pipe.plan_bytes() > PLAN_CACHE_MAX_BYTES:
        return pipe
    with _PLANS_LOCK:
        _PLANS[key] = pipe
        _PLANS.move_to_end(key)
        while len(_PLANS) > 1 and (len(_PLANS) > PLAN_CACHE_SIZE
                                   or sum(_plan_held_bytes(p) for p in _PLANS.values()) > PLAN_CACHE_TOTAL_BYTES):
            _PLANS.popitem(last=False)
    return pipe


def _plan_held_bytes(pipe) -> int:
    """Device bytes a cached plan holds: its buffers, the output mapping it keeps for reuse (the mapped
    bytes: whole 1-GiB chunks) and the output buffers of pipelined steps, if any."""
    total = pipe.plan_bytes()
    own = getattr(pipe, "_call_owner", None)
    if own is not None:
        total += own.mapped_bytes() if hasattr(own, "mapped_bytes") else 8 * own.n
    for t in getattr(pipe, "_outs", None) or []:
        total += t.numel() * t.element_size()
    return total


def clear_plan_cache() -> None:
    """Drop every cached plan (and the output mappings they keep): the device memory returns once
    no result tensor of theirs is alive."""
    with _PLANS_LOCK:
        _PLANS.clear()


def _is_oom(e: Exception) -> bool:
    T = engine.torch()
    msg = str(e)
    return (isinstance(e, T.cuda.OutOfMemoryError) or "out of memory" in msg.lower()
            or "hipErrorOutOfMemory" in msg)


def _planned_dense(virt: VirtualCircuit, device: int, out):
    """One step of the cached plan into a fresh (or the caller's) output buffer. ``run_time`` = host
    planning (first call) + the sweep (HIP events), ``knit_time`` = the rest of the wall time: the
    same split as run.py:35,60,65-67 without a host synchronisation between the two."""
    T = engine.torch()
    now = perf_counter()
    pipe = cached_plan(virt, device)
    t_plan = perf_counter()
    pipe.be.bind()
    if out is None:  # 1-GiB-mapped when large; the previous call's mapping once the caller dropped it
        out = pipe.take_out(defer_select=True)
    t_out = perf_counter()
    e0, e1 = T.cuda.Event(enable_timing=True), T.cuda.Event(enable_timing=True)
    host = perf_counter() - now
    timed = getattr(pipe, "_time_call_write", False) and not pipe.record_events
    n_ev = len(pipe.events)
    e0.record()
    pipe.out = out
    try:
        if timed:  # the call's own write times its un-checked output mapping (KnitPipeline.take_out)
            pipe.record_events = True
        qs = pipe.sweep()
        e1.record()
        t_sweep = perf_counter()
        pipe.knit(qs)
        t_knit = perf_counter()
        out = pipe.out
    finally:
        pipe.out = None
        if timed:
            pipe.record_events = False
    _sync(device)
    wall = perf_counter() - now
    if timed:
        pipe.note_call_write(n_ev)
        del pipe.events[n_ev:]
    if not pipe.plan_reused and not hasattr(pipe, "first_call_ms"):
        # where the first call's time goes: the plan's phases (KnitPipeline.plan_ms), the output buffer
        # (mapping + write-rate selection), the step itself (launches + device time to the sync)
        pipe.first_call_ms = {"plan": (t_plan - now) * 1e3, **{f"plan.{k}": v for k, v in pipe.plan_ms.items()},
                              "output_buffer": (t_out - t_plan) * 1e3, "step": (now + wall - t_out) * 1e3,
                              "step.sweep_launch": (t_sweep - t_out) * 1e3, "step.knit_launch": (t_knit - t_sweep) * 1e3,
                              "step.device_wait": (now + wall - t_knit) * 1e3, "total": wall * 1e3}
    pipe.sync_stats()
    run_time = host + e0.elapsed_time(e1) * 1e-3
    return out, RunTimeInfo(run_time, max(wall - run_time, 0.0)), pipe


def _planned_dict(virt: VirtualCircuit, device: int, accuracy: float):
    """The reference-shaped result from the cached plan (``KnitPipeline.knit_dict``): the
    thresholded knit where it applies, never the dense 2^N vector."""
    T = engine.torch()
    now = perf_counter()
    pipe = cached_plan(virt, device)
    pipe.be.bind()
    e0, e1 = T.cuda.Event(enable_timing=True), T.cuda.Event(enable_timing=True)
    host = perf_counter() - now
    e0.record()
    qs = pipe.sweep()
    e1.record()
    keys, vals = pipe.knit_dict(accuracy, qs)
    wall = perf_counter() - now
    pipe.sync_stats()
    run_time = host + e0.elapsed_time(e1) * 1e-3
    return keys, vals, RunTimeInfo(run_time, max(wall - run_time, 0.0))


def run_virtual_circuit_dense(virt: VirtualCircuit, shots: int = 20000, *, device: int = 0,
                              factored: bool | None = None, out=None, sample: bool = False, seed: int = 0):
    """Sweep (or shot-sample, ``sample=True``) + knit; returns ``(dense fp64 tensor [2^N] on
    device, RunTimeInfo)``.

    Default (``factored=None``, every fragment on the MI355X backend, exact instances): the cached
    plan (:func:`cached_plan`) — the engine ``bench.py`` times: factored light-cone knit, per-step
    device data rank, the write-bound blocked knit. ``factored=True/False`` force the uncached
    factored / direct ``engine.knit_dense``; sampling and foreign backends take the direct path."""
    log.info("Running virtualizer with %d %s fragments and %d vgates...",
             len(virt.fragment_circuits),
             tuple(len(f) for f in virt.fragment_circuits), len(virt.vgate_instructions))
    native = all(isinstance(virt.get_backend(f), MI355XBackend) for f in virt.fragment_circuits if len(f))
    if factored is None and native and not sample:
        try:
            dense, info, _ = _planned_dense(virt, device, out)
        except Exception as e:  # out of device memory: drop the cached plans (and their outputs), retry once
            if not _is_oom(e):
                raise
            log.warning("out of device memory (%s): clearing the plan cache and retrying", e)
            clear_plan_cache()
            engine.torch().cuda.empty_cache()
            dense, info, _ = _planned_dense(virt, device, out)
    else:
        dense, info = _direct_dense(virt, shots, device, bool(factored), out, sample, seed)
    log.info("Knitted in %.2fs.", info.knit_time)
    return dense, info


def run_virtual_circuit_sharded(virt: VirtualCircuit, group=None, *, device: int | None = None, backend=None):
    """Multi-GPU ``run_virtual_circuit`` (one process per GPU, ``torch.distributed`` initialised;
    ``group``: the process group, None = WORLD). The instance sweep is sharded over the ranks and
    the distribution assembled by the pipeline's collectives:

    * wide outputs (syc 32: 2^32 fp64 = 34 GB) in ``slice`` mode: rank r returns the contiguous
      outputs ``[r, r + 1) * 2^N / world`` of the reference-ordered distribution (concatenating the
      ranks' shards in rank order gives the whole array);
    * narrow outputs (bv / hwe / qft: at most the instance tensors' size) in ``reduce`` mode: one
      RCCL reduce; rank 0 holds the whole distribution, the others ``None``.

    Returns ``(tensor or None, RunTimeInfo)`` with ``info.shard = (first output, outputs)`` of the
    returned tensor. Exact instances only (the reference's ``shots`` sampling: single-GPU
    ``run_virtual_circuit(sample=True)``)."""
    import torch.distributed as dist

    T = engine.torch()
    rank = dist.get_rank(group)
    if device is None:
        device = T.cuda.current_device() if backend is None else 0
    log.info("Running virtualizer with %d %s fragments and %d vgates on %d ranks...",
             len(virt.fragment_circuits), tuple(len(f) for f in virt.fragment_circuits),
             len(virt.vgate_instructions), dist.get_world_size(group))
    on_gpu = backend is None
    now = perf_counter()
    pipe = cached_plan(virt, device, group="WORLD" if group is None else group, backend=backend)
    bind = getattr(pipe.be, "bind", None)
    if bind is not None:
        bind()
    # slice mode: the previous call's output mapping again once the caller dropped it (take_out);
    # reduce mode: a fresh (small) buffer per call, as the reference returns a new result per call
    pipe.out = pipe.take_out() if pipe.mode == "slice" else None
    try:
        qs = pipe.sweep()
        if on_gpu:
            _sync(device)
        run_time = perf_counter() - now
        now = perf_counter()
        out = pipe.knit(qs)
        if on_gpu:
            _sync(device)
    finally:
        pipe.out = None
    pipe.sync_stats()
    knit_time = perf_counter() - now
    log.info("Knitted in %.2fs.", knit_time)
    if pipe.mode == "slice":
        return out, RunTimeInfo(run_time, knit_time, tuple(pipe.slice))
    n = 1 << pipe.N
    return (out if rank == 0 else None), RunTimeInfo(run_time, knit_time, (0, n) if rank == 0 else (0, 0))


def _build_sharded_plan(virt: VirtualCircuit, device: int, group, backend):
    """This rank's plan of a multi-GPU run: slice mode for a factored two-fragment knit
    whose fragments partition the output bits, else the direct knit in reduce mode (one RCCL reduce)."""
    import torch.distributed as dist

    from .pipeline import KnitPipeline

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    kw = {"backend": backend} if backend is not None else {}
    if engine.factored_ok(virt):  # else (both endpoints of a gate in one fragment): direct knit, reduce mode
        pipe = KnitPipeline(virt, device=device, factored=True, rank=rank, world=world, group=group, **kw)
        if pipe.mode == "slice":
            return pipe
        del pipe
    return KnitPipeline(virt, device=device, factored=False, rank=rank, world=world, group=group, mode="reduce", **kw)


def _sharded_dict(virt: VirtualCircuit, group, device: int, accuracy: float):
    """The reference-shaped dict of a multi-GPU run, every rank the whole of it (``run.py:71``): slice
    mode selects the entries above ``accuracy`` per rank and runs the NPD of the gathered union
    (``KnitPipeline.knit_dict``, any output width); reduce mode's distribution (at most the instance
    tensors' size) is all-reduced and truncated as on one GPU."""
    T = engine.torch()
    now = perf_counter()
    pipe = cached_plan(virt, device, group="WORLD" if group is None else group)
    pipe.be.bind()
    if pipe.mode == "slice":
        e0, e1 = T.cuda.Event(enable_timing=True), T.cuda.Event(enable_timing=True)
        host = perf_counter() - now
        e0.record()
        qs = pipe.sweep()
        e1.record()
        keys, vals = pipe.knit_dict(accuracy, qs)
        wall = perf_counter() - now
        run_time = host + e0.elapsed_time(e1) * 1e-3
        return keys, vals, RunTimeInfo(run_time, max(wall - run_time, 0.0), tuple(pipe.slice))
    import torch.distributed as dist

    out, info = run_virtual_circuit_sharded(virt, group, device=device)
    full = T.zeros(1 << virt.circuit.num_clbits, dtype=T.float64, device=T.device("cuda", device))
    lo, cnt = info.shard
    if out is not None and cnt:
        full[lo:lo + cnt] = out[:cnt]
    dist.all_reduce(full, group=group)  # shards are disjoint: the sum assembles the distribution
    keys, vals = engine.nearest_probability_distribution(engine.get_context(device), full, accuracy)
    return keys, vals, info


def _run_reference_truncated(virt: VirtualCircuit, device: int, dense: bool):
    """``truncation="reference"``: the reference's knit with ``ACCURACY`` applied after every
    operation (truncated.knit_reference_truncated), then nearest_probability_distribution."""
    from .truncated import knit_reference_truncated

    if not all(isinstance(virt.get_backend(f), MI355XBackend) for f in virt.fragment_circuits if len(f)):
        raise ValueError("truncation='reference' needs every fragment on the MI355X backend")
    log.info("Running virtualizer with %d %s fragments and %d vgates (reference truncation)...",
             len(virt.fragment_circuits), tuple(len(f) for f in virt.fragment_circuits), len(virt.vgate_instructions))
    now = perf_counter()
    out = knit_reference_truncated(virt, device, _qd.ACCURACY)
    _sync(device)
    info = RunTimeInfo(0.0, perf_counter() - now)
    log.info("Knitted in %.2fs.", info.knit_time)
    if dense:
        return out, info
    keys, vals = engine.nearest_probability_distribution(engine.get_context(device), out, _qd.ACCURACY)
    return dict(zip(keys.tolist(), vals.tolist())), info


def run_virtual_circuit(virt: VirtualCircuit, shots: int = 20000, *, device: int = 0,
                        dense: bool = False, factored: bool | None = None, sample: bool = False, seed: int = 0,
                        group=None, truncation: str = "final"):
    """Reference-compatible entry point (``run.py:23-71``). ``group`` (a ``torch.distributed``
    process group, e.g. ``dist.group.WORLD``) runs it on every rank of the group
    (:func:`run_virtual_circuit_sharded`, the plan cached per group like the single-GPU one):
    ``dense=True`` returns the rank's shard, otherwise every rank returns the whole reference-shaped
    dict (slice mode: the entries above ``ACCURACY`` selected per rank, gathered, then the NPD — any
    output width, syc 32 included).

    ``truncation``: ``"final"`` (default) knits exactly and applies ``ACCURACY`` once, to the result;
    ``"reference"`` applies it after every operation as the reference's ``QuasiDistr`` dicts do
    (``quasi_distr.py:7-10``: from_counts, every merge, every per-gate ``+ - *``), on exact instance
    distributions, single GPU, at most 24 clbits (``dense=True``: the knit before NPD)."""
    if truncation not in ("final", "reference"):
        raise ValueError(f"truncation must be 'final' or 'reference', not {truncation!r}")
    if truncation == "reference":
        if group is not None or sample or factored is not None:
            raise ValueError("truncation='reference': single GPU, exact instances, the direct knit")
        if virt.circuit.num_clbits > 24:
            raise ValueError("truncation='reference' is for outputs of at most 24 clbits")
        return _run_reference_truncated(virt, device, dense)
    if group is not None:
        if sample:
            raise ValueError("multi-GPU runs sweep exact instances (sample=True: single GPU)")
        if dense:
            return run_virtual_circuit_sharded(virt, group, device=device)
        keys, vals, info = _sharded_dict(virt, group, device, _qd.ACCURACY)
        log.info("Knitted in %.2fs.", info.knit_time)
        return dict(zip(keys.tolist(), vals.tolist())), info
    else:
        native = all(isinstance(virt.get_backend(f), MI355XBackend) for f in virt.fragment_circuits if len(f))
        if not dense and factored is None and native and not sample:
            # reference-shaped result straight from the plan: entries above ACCURACY only
            log.info("Running virtualizer with %d %s fragments and %d vgates...",
                     len(virt.fragment_circuits), tuple(len(f) for f in virt.fragment_circuits),
                     len(virt.vgate_instructions))
            keys, vals, info = _planned_dict(virt, device, _qd.ACCURACY)
            log.info("Knitted in %.2fs.", info.knit_time)
            return dict(zip(keys.tolist(), vals.tolist())), info
        out, info = run_virtual_circuit_dense(virt, shots, device=device, factored=factored, sample=sample,
                                              seed=seed)
    if dense:
        return out, info
    keys, vals = engine.nearest_probability_distribution(engine.get_context(device), out, _qd.ACCURACY)
    return dict(zip(keys.tolist(), vals.tolist())), info
