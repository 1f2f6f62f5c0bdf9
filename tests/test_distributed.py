"""Multi-rank orchestration of KnitPipeline (world_size 2-4, gloo, CPU backend model).

Checks both collective modes against the oracle's dense knit:
* reduce: label-sliced sweep + partial contraction + one reduce to rank 0;
* gather: sharded sweep + all_to_all (row side) / all_gather (column side) of q_f +
  output-sharded contraction.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _collect(procs, q, timeout):
    """The result rank 0 puts on ``q``; a worker that dies fails the test at once instead of at the
    timeout."""
    import queue
    import time

    t_end = time.time() + timeout
    while True:
        try:
            return q.get(timeout=5)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"worker exited with {dead}"
            assert time.time() < t_end, "no result before the timeout"


def _case(name):
    import circuits
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    return {
        "cx_3cuts": lambda: circuits.two_fragment("cx", 3, 3, n_cuts=3),
        "three": lambda: circuits.three_fragment(seed=9, sizes=(3, 2, 3)),
        "move_gate": lambda: circuits.wire_cut(3, 2, extra_gate_cut=True),
        "hwe_p3": lambda: cutting.config_cut_circuit("hwe", 16, 1, 3)[:2],
    }[name]()


def _worker(rank, world, port, case, mode, factored, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cpu_backend import CpuBackend

        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, engine
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        _, cut = _case(case)
        pipe = KnitPipeline(VirtualCircuit(cut), rank=rank, world=world, mode=mode, factored=factored,
                            backend=CpuBackend(), data_rank=True)
        res = pipe.step().numpy().copy()
        if mode == "gather":
            # place this rank's (x_A block, x_B) rows at their global keys, then sum over ranks
            order = pipe.order
            cls = pipe.ops.clbits
            kA = deposit_keys(cls[order[0]])
            for i in order[1:-1]:
                kA = (kA[None, :] + deposit_keys(cls[i])[:, None]).reshape(-1)
            kB = deposit_keys(cls[order[-1]])
            lo, hi = pipe.row_block
            full = np.zeros(1 << pipe.N)
            blk = res[: (hi - lo) * kB.size].reshape(hi - lo, kB.size)
            full[(kA[lo:hi, None] + kB[None, :]).reshape(-1)] = blk.reshape(-1)
            t = torch.from_numpy(full)
            dist.reduce(t, dst=0)
            res = t.numpy()
        if rank == 0:
            q.put((pipe.mode, res, pipe.data_rank, pipe.last_rank, pipe.ops.num_terms))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,mode,factored,world", [
    ("cx_3cuts", "reduce", False, 2), ("cx_3cuts", "gather", False, 2), ("cx_3cuts", "gather", True, 2),
    ("three", "reduce", False, 2), ("three", "gather", True, 2), ("move_gate", "gather", False, 2),
    # 4 ranks: all_to_all split of the row side; 3 ranks: uneven shards, padded rows, no split
    ("cx_3cuts", "gather", True, 4), ("move_gate", "gather", True, 3),
])
def test_multi_rank_pipeline_matches_oracle(case, mode, factored, world):
    sys.path.insert(0, HERE)
    from oracle import dense

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, mode, factored, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got_mode, res, data_rank, last_rank, terms = _collect(procs, q, 240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got_mode == mode
    if factored and mode == "gather" and case != "three":
        # two fragments: each rank compresses its own row block to its data rank (no collective)
        assert data_rank and last_rank is not None and last_rank < terms
    _, cut = _case(case)
    ref = dense.run_dense(cut)
    np.testing.assert_allclose(res, ref, atol=1e-12, rtol=0)


def _slice_worker(rank, world, port, case, data_rank, q, veto_rank=None, row_jobs=None, prep="sharded"):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QKNIT_SLICE_PREP=prep)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cpu_backend import CpuBackend

        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, pipeline
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        if row_jobs is not None:
            pipeline.ROW_JOBS = row_jobs
        _, cut = _slice_case(case)
        pipe = KnitPipeline(VirtualCircuit(cut), rank=rank, world=world, factored=True, backend=CpuBackend(),
                            data_rank=data_rank)
        assert pipe.mode == "slice" and pipe.slice_prep == prep and pipe.sharded == (prep == "sharded")
        # pipelined steps rotate 2 output buffers at 2-4 ranks, 3 from 8 on (QKNIT_OUT_BUFFERS overrides)
        assert pipe.out_buffers == (3 if world >= 8 else 2 if world >= 2 else 1)
        if veto_rank == rank:  # this rank's probe check rejects every compression
            pipe.rank_tol = pipe.rank_tol_rel = float("nan")
        outs = []
        for _ in range(2):
            res = pipe.step().clone()
            parts = [torch.empty_like(res) for _ in range(world)]
            dist.all_gather(parts, res)
            outs.append(torch.cat(parts).numpy())
        pipe.sync_stats()
        if rank == 0:
            q.put((outs, pipe.slice, pipe.last_rank, pipe.rank_fallbacks, pipe.rank_incompressible, pipe.dev_rank,
                   pipe.last_prep, pipe._replicated_a_cols()))
    finally:
        dist.destroy_process_group()


def _slice_case(name):
    import circuits
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    return {
        "hwe_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[:2],
        "cx_8x8": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4),
        "cx_6x5": lambda: circuits.two_fragment("cx", 6, 5, n_cuts=2),
    }[name]()


@pytest.mark.parametrize("prep", ["sharded", "replicated"])
@pytest.mark.parametrize("case,world,data_rank,row_jobs", [("hwe_p2", 2, True, None), ("hwe_p2", 4, True, None),
                                                           ("cx_8x8", 2, True, None), ("cx_6x5", 2, True, None),
                                                           ("hwe_p2", 2, False, None), ("cx_6x5", 2, True, 1)])
def test_slice_mode_matches_oracle(case, world, data_rank, row_jobs, prep):
    """slice mode: each rank writes the contiguous range [rank, rank + 1) * 2^N / world of the
    reference-ordered distribution; the slices concatenate (no permutation) to the oracle's dense
    knit within 1e-12, twice in a row. cx_8x8's knit has rank > 8 (the exact contraction of the
    slice: from all-gathered operands when sharded, from the rank's own whole operands when
    replicated); the others compress on every step. Both preparations: rows dealt over the ranks with
    collectives (sharded) and every rank sweeping and preparing everything (replicated: no collective)."""
    from oracle import dense

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slice_worker, args=(r, world, port, case, data_rank, q, None, row_jobs, prep))
             for r in range(world)]
    for p in procs:
        p.start()
    outs, sl, last_rank, fallbacks, incompressible, dev, last_prep, a_cols = _collect(procs, q, 300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # replicated: rank 0 compresses and checks only the A columns its slice reads (the others NaN in the
    # CPU backend's A2, so a read outside them would show below)
    if prep == "replicated" and case == "hwe_p2":
        assert a_cols is not None and a_cols[1] < 1 << 8
    sys.path.insert(0, HERE)
    _, cut = _slice_case(case)
    ref = dense.run_dense(cut)
    for got in outs:
        np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0)
    assert sl == (0, ref.size // world)
    assert fallbacks == 0
    if data_rank and case != "cx_8x8":
        assert dev and last_rank is not None and incompressible == 0
    if case == "cx_8x8":
        assert incompressible == 2 and last_rank is None
    if data_rank:  # 128-column blocks take the fused preparation (qk_prep_operands' contract), others torch
        fused = (case, world) in (("hwe_p2", 2), ("cx_8x8", 2)) or (prep == "replicated" and case != "cx_6x5")
        assert last_prep == ("fused" if fused else "torch")


def _api_worker(rank, world, port, case, q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cpu_backend import CpuBackend

        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import run_virtual_circuit_sharded

        _, cut = _slice_case(case) if case != "cx_3cuts" else _case(case)
        out, info = run_virtual_circuit_sharded(VirtualCircuit(cut), backend=CpuBackend())
        lo, cnt = info.shard
        n = 1 << len([c for r in cut.cregs for c in r])
        full = torch.zeros(n, dtype=torch.float64)
        if out is not None and cnt:
            full[lo:lo + cnt] = out[:cnt]
        shards = [None] * world
        dist.all_gather_object(shards, (lo, cnt))
        dist.all_reduce(full)
        if rank == 0:
            q.put((full.numpy(), shards))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("hwe_p2", 2), ("cx_3cuts", 2), ("hwe_p2", 4)])
def test_run_virtual_circuit_sharded_api(case, world):
    """run_virtual_circuit_sharded (the group= form of run_virtual_circuit, run.py:23-71): slice mode
    (hwe 16: 2^16 outputs) hands each rank a contiguous shard, in rank order; reduce mode (cx_3cuts:
    2^6 outputs) the whole distribution on rank 0. Assembled, both equal the oracle's knit."""
    from oracle import dense

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_api_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, shards = _collect(procs, q, 300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, HERE)
    _, cut = _slice_case(case) if case != "cx_3cuts" else _case(case)
    np.testing.assert_allclose(full, dense.run_dense(cut), atol=1e-12, rtol=0)
    n = full.size
    if case == "cx_3cuts":
        assert shards[0] == (0, n) and all(s == (0, 0) for s in shards[1:])
    else:
        assert shards == [(r * n // world, n // world) for r in range(world)]


@pytest.mark.parametrize("prep", ["sharded", "replicated"])
def test_slice_mode_one_rank_rejects(prep):
    """A probe check that rejects on ONE rank only (that rank's tolerance forced below zero). Sharded:
    the MIN all-reduce of the accepted ranks sends every rank to the exact slice together (their
    collectives match: no hang). Replicated: no collective, so rank 0 keeps its accepted compression
    and only rank 1 writes its slice exactly. Either way the slices concatenate to the oracle's knit."""
    from oracle import dense

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_slice_worker, args=(r, world, port, "hwe_p2", True, q, 1, None, prep))
             for r in range(world)]
    for p in procs:
        p.start()
    outs, sl, last_rank, fallbacks, incompressible, dev, _, _ = _collect(procs, q, 300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, HERE)
    _, cut = _slice_case("hwe_p2")
    ref = dense.run_dense(cut)
    for got in outs:
        np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0)
    if prep == "sharded":
        assert dev and fallbacks == 2 and last_rank is None  # rank 0 accepted locally, yet took the exact path
    else:
        assert dev and fallbacks == 0 and last_rank is not None  # rank 0's own verdict
