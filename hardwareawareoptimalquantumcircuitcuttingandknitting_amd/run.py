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

import logging
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


def run_virtual_circuit_dense(virt: VirtualCircuit, shots: int = 20000, *, device: int = 0,
                              factored: bool = False, out=None, sample: bool = False, seed: int = 0):
    """Sweep (or shot-sample, ``sample=True``) + knit; returns ``(dense fp64 tensor [2^N] on
    device, RunTimeInfo)``."""
    ctx = engine.get_context(device)
    # The factored knit folds labels whose side programs coincide into one operand row; sampled
    # labels differ in their shots even then, so sampling knits directly over the labels.
    factored = factored and not sample
    log.info("Running virtualizer with %d %s fragments and %d vgates...",
             len(virt.fragment_circuits),
             tuple(len(f) for f in virt.fragment_circuits), len(virt.vgate_instructions))
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
    log.info("Knitted in %.2fs.", knit_time)
    return dense, RunTimeInfo(run_time, knit_time)


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

    from .pipeline import KnitPipeline

    T = engine.torch()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if device is None:
        device = T.cuda.current_device() if backend is None else 0
    log.info("Running virtualizer with %d %s fragments and %d vgates on %d ranks...",
             len(virt.fragment_circuits), tuple(len(f) for f in virt.fragment_circuits),
             len(virt.vgate_instructions), world)
    kw = {"backend": backend} if backend is not None else {}
    pipe = KnitPipeline(virt, device=device, factored=True, rank=rank, world=world, group=group, **kw)
    if pipe.mode != "slice":
        pipe = KnitPipeline(virt, device=device, factored=False, rank=rank, world=world, group=group,
                            mode="reduce", **kw)
    on_gpu = backend is None
    now = perf_counter()
    qs = pipe.sweep()
    if on_gpu:
        _sync(device)
    run_time = perf_counter() - now
    now = perf_counter()
    out = pipe.knit(qs)
    if on_gpu:
        _sync(device)
    knit_time = perf_counter() - now
    log.info("Knitted in %.2fs.", knit_time)
    if pipe.mode == "slice":
        return out, RunTimeInfo(run_time, knit_time, tuple(pipe.slice))
    n = 1 << pipe.N
    return (out if rank == 0 else None), RunTimeInfo(run_time, knit_time, (0, n) if rank == 0 else (0, 0))


def run_virtual_circuit(virt: VirtualCircuit, shots: int = 20000, *, device: int = 0,
                        dense: bool = False, factored: bool = False, sample: bool = False, seed: int = 0,
                        group=None):
    """Reference-compatible entry point (``run.py:23-71``). ``group`` (a ``torch.distributed``
    process group, e.g. ``dist.group.WORLD``) runs it on every rank of the group
    (:func:`run_virtual_circuit_sharded`): ``dense=True`` returns the rank's shard, otherwise every
    rank returns the whole reference-shaped dict (outputs of at most 24 clbits)."""
    if group is not None:
        if sample:
            raise ValueError("multi-GPU runs sweep exact instances (sample=True: single GPU)")
        out, info = run_virtual_circuit_sharded(virt, group, device=device)
        if dense:
            return out, info
        import torch.distributed as dist

        n_bits = virt.circuit.num_clbits
        if n_bits > 24:
            raise ValueError(f"a dict of 2^{n_bits} outcomes: use dense=True (each rank gets its shard)")
        T = engine.torch()
        full = T.zeros(1 << n_bits, dtype=T.float64, device=T.device("cuda", device))
        lo, cnt = info.shard
        if out is not None and cnt:
            full[lo:lo + cnt] = out[:cnt]
        dist.all_reduce(full, group=group)  # shards are disjoint: the sum assembles the distribution
        out = full
    else:
        out, info = run_virtual_circuit_dense(virt, shots, device=device, factored=factored, sample=sample,
                                              seed=seed)
    if dense:
        return out, info
    from . import quasi_distr

    keys, vals = engine.nearest_probability_distribution(engine.get_context(device), out,
                                                         quasi_distr.ACCURACY)
    return dict(zip(keys.tolist(), vals.tolist())), info
