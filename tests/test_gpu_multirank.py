"""Multi-rank KnitPipeline on the HIP backend: 2-4 ranks share the one GPU of a test box.

The 8-GPU node is not ours to launch (the driver runs the scaling bench), and RCCL refuses two
ranks on one device, so these tests run the ranks' real HIP kernels (sweeps, transforms,
qk_rank_factors, the range knit, the predicated exact contraction) with a gloo process group
over the ranks' device tensors. Same checks as tests/test_distributed.py (which runs the CPU
backend model): slices concatenate to the oracle's dense knit within 1e-12; reduce mode and
gather mode (advisor item: the gather data-rank branch on HIP) likewise; and the bench workload
syc 32 5 in slice mode against the single-GPU step, rank by rank.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-12


@pytest.fixture(autouse=True)
def _parent_releases_device_memory():
    """The ranks are spawned processes sharing the test box's one GPU; the pytest process itself may
    still hold device memory from earlier in-process GPU tests (cached plans with their 34-GB output
    mappings, torch's caching allocator). Release it first, so the ranks' allocations never compete
    with a parent that no longer needs its memory."""
    import gc

    import torch

    if torch.cuda.is_initialized():
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod

        runmod.clear_plan_cache()
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    yield


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(name):
    import circuits
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import cutting

    return {
        "hwe_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[:2],
        "cx_8x8": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4),
        "cx_3cuts": lambda: circuits.two_fragment("cx", 3, 3, n_cuts=3),
        "three": lambda: circuits.three_fragment(seed=9, sizes=(3, 2, 3)),
        "syc_32_5": lambda: cutting.config_cut_circuit("syc", 32, 5, 2)[:2],
    }[name]()


def _watchdog(rank, tag, after=100):
    """QKNIT_TB_DIR set: dump every thread's stack to <dir>/<tag>_rank<r>.tb after ``after`` s and
    exit (a rank stuck in a collective shows where, instead of a silent hang). Returns a progress
    logger (appends to <dir>/<tag>_rank<r>.log; a no-op without the directory)."""
    d = os.environ.get("QKNIT_TB_DIR")
    if not d:
        return lambda msg: None
    import faulthandler
    import time

    os.makedirs(d, exist_ok=True)
    f = open(os.path.join(d, f"{tag}_rank{rank}.tb"), "w")
    after = float(os.environ.get("QKNIT_TB_AFTER", after))  # a shorter fuse for a hang hunt
    faulthandler.dump_traceback_later(after, exit=True, file=f)
    t0 = time.time()

    def log(msg):
        with open(os.path.join(d, f"{tag}_rank{rank}.log"), "a") as g:
            g.write(f"{time.time() - t0:8.1f}s {msg}\n")

    return log


def _worker(rank, world, port, case, mode, factored, q, overlap=False, veto_rank=None, prep="auto"):
    log = _watchdog(rank, f"{case}_{mode}_{world}")
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QKNIT_SLICE_PREP=prep, QKNIT_POISON_UNUSED="1")
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        torch.cuda.set_device(0)
        _, cut = _case(case)
        pipe = KnitPipeline(VirtualCircuit(cut), device=0, rank=rank, world=world, mode=mode, factored=factored,
                            data_rank=factored)
        assert pipe.be.dev.type == "cuda"
        if overlap:  # pipelined steps (the multi-GPU bench default): a non-default caller stream
            torch.cuda.set_stream(torch.cuda.Stream())
            pipe.overlap = pipe.overlap_ok()
            assert pipe.overlap
        if veto_rank == rank:
            pipe.rank_tol = pipe.rank_tol_rel = float("nan")
        log(f"planned: mode {pipe.mode}")
        outs = []
        for it in range(2):
            res = pipe.step()
            torch.cuda.synchronize()
            res = res.cpu().clone()
            log(f"step {it}")
            if pipe.mode == "slice":
                parts = [torch.empty_like(res) for _ in range(world)]
                dist.all_gather(parts, res)
                full = torch.cat(parts).numpy()
            elif pipe.mode == "gather":
                cls = pipe.ops.clbits
                kA = deposit_keys(cls[pipe.order[0]])
                for i in pipe.order[1:-1]:
                    kA = (kA[None, :] + deposit_keys(cls[i])[:, None]).reshape(-1)
                kB = deposit_keys(cls[pipe.order[-1]])
                lo, hi = pipe.row_block
                f = np.zeros(1 << pipe.N)
                f[(kA[lo:hi, None] + kB[None, :]).reshape(-1)] = res.numpy()[: (hi - lo) * kB.size]
                t = torch.from_numpy(f)
                dist.all_reduce(t)
                full = t.numpy()
            else:
                full = res.numpy()
            outs.append(full)
        pipe.sync_stats()
        if rank == 0:
            q.put((pipe.mode, outs, pipe.last_rank, pipe.rank_fallbacks, pipe.rank_incompressible,
                   pipe.dev_rank, pipe.last_kernel, pipe.ops.num_terms))
    finally:
        dist.destroy_process_group()


def _run(target, world, *args, timeout=300, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time

    try:
        t_end = time.time() + timeout
        while True:  # a worker that dies (an assertion, a crash) fails the test now, not at the timeout
            try:
                got = q.get(timeout=5)
                break
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"worker exited with {dead}"
                assert time.time() < t_end, "no result before the timeout"
    finally:
        for p in procs:
            p.join(timeout=120)
    for p in procs:
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("case,mode,factored,world", [
    ("hwe_p2", "slice", True, 2), ("hwe_p2", "slice", True, 4), ("cx_8x8", "slice", True, 2),
    ("cx_3cuts", "reduce", False, 2), ("cx_3cuts", "gather", True, 2), ("three", "gather", True, 2),
])
def test_multi_rank_hip_matches_oracle(case, mode, factored, world):
    """Every mode's collectives over the ranks' HIP results, twice in a row, against the oracle.
    Two-fragment data-rank cases take the device data-rank path (hwe: an accepted rank on every step); cx_8x8's knit has
    rank > 8 and takes the exact contraction of each slice."""
    sys.path.insert(0, HERE)
    from oracle import dense

    got_mode, outs, last_rank, fallbacks, incompressible, dev, kernel, terms = _run(
        _worker, world, case, mode, factored)
    assert got_mode == mode
    _, cut = _case(case)
    ref = dense.run_dense(cut)
    for full in outs:
        np.testing.assert_allclose(full, ref, atol=TOL, rtol=0)
    assert fallbacks == 0
    if case == "hwe_p2":
        assert dev and last_rank is not None and last_rank <= terms and incompressible == 0
        assert kernel == "qk_knit_outer_blocked_kernel"
    if case == "cx_8x8":
        assert incompressible == 2 and last_rank is None
    if case == "cx_3cuts" and mode == "gather":
        assert last_rank is not None and last_rank < terms  # the gather-mode data-rank branch ran


@pytest.mark.timeout(400)
@pytest.mark.parametrize("case,world,veto,prep", [("hwe_p2", 8, None, "auto"), ("cx_8x8", 4, None, "auto"),
                                                  ("hwe_p2", 4, 2, "sharded"), ("hwe_p2", 4, 0, "replicated")])
def test_multi_rank_hip_overlapped_steps_match_oracle(case, world, veto, prep, monkeypatch):
    """Pipelined steps (step i+1's sweep, preparation (and, sharded, its collectives) on a CU-masked
    stream under step i's write: the multi-GPU bench default) in slice mode on 4-8 ranks sharing the
    GPU, twice in a row, against the oracle at 1e-12: hwe (compressed every step), cx_8x8 (rank > 8:
    the exact slice), and a probe check rejecting on one rank only — sharded: every rank takes the exact
    slice together (MIN all-reduce); replicated: only that rank does (no collective), its slice still
    exact. Every rank's slice is a qk_out_alloc mapping (QKNIT_OUT_MAPPED_MIN_BYTES=0: small outputs
    mapped too)."""
    monkeypatch.setenv("QKNIT_OUT_MAPPED_MIN_BYTES", "0")
    sys.path.insert(0, HERE)
    from oracle import dense

    got_mode, outs, last_rank, fallbacks, incompressible, dev, kernel, terms = _run(
        _worker, world, case, "slice", True, timeout=360, overlap=True, veto_rank=veto, prep=prep)
    assert got_mode == "slice" and dev
    _, cut = _case(case)
    ref = dense.run_dense(cut)
    for full in outs:
        np.testing.assert_allclose(full, ref, atol=TOL, rtol=0)
    if veto is not None:  # rank 0 reports: sharded, the shared verdict; replicated, its own (vetoed) one
        assert fallbacks == 2 and last_rank is None
    elif case == "hwe_p2":
        assert fallbacks == 0 and last_rank is not None
    else:
        assert incompressible == 2


def _syc_worker(rank, world, port, q, overlap=False, prep="auto"):
    log = _watchdog(rank, f"syc_32_5_{world}", after=700)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QKNIT_SLICE_PREP=prep, QKNIT_POISON_UNUSED="1")
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        torch.cuda.set_device(0)
        _, cut = _case("syc_32_5")
        virt = VirtualCircuit(cut)
        lo, cnt = rank * ((1 << 32) // world), (1 << 32) // world
        # the single-GPU step of the same workload, one rank at a time (memory); each rank keeps its range
        ref = None
        for r in range(world):
            dist.barrier()
            if r == rank:
                one = KnitPipeline(virt, device=0, factored=True)
                full = one.step()
                ref = full[lo:lo + cnt].clone()
                log("single-GPU step done")
                del one, full
                torch.cuda.empty_cache()
        dist.barrier()
        pipe = KnitPipeline(virt, device=0, rank=rank, world=world, factored=True)
        assert pipe.mode == "slice" and pipe.dev_rank and pipe.slice == (lo, cnt)
        if prep != "auto":
            assert pipe.slice_prep == prep
        if overlap:  # pipelined steps (the multi-GPU bench default): a non-default caller stream
            torch.cuda.set_stream(torch.cuda.Stream())
            pipe.overlap = pipe.overlap_ok()
            assert pipe.overlap
        log(f"planned ({pipe.slice_prep})")
        # plain first step, then pipelined (at 4 ranks: both output buffers, so every buffer is checked)
        err = torch.zeros(1, dtype=torch.float64)
        ptrs = set()
        for it in range(4):
            sl = pipe.step()
            torch.cuda.synchronize()
            err[0] = max(float(err[0]), float((sl - ref).abs().max()))
            ptrs.add(sl.data_ptr())
            log(f"step {it} compared")
        pipe.sync_stats()
        assert pipe.rank_fallbacks == 0 and pipe.last_rank is not None
        total = torch.tensor([float(sl.sum())], dtype=torch.float64)
        mn = float(sl.min())
        n_buf = torch.tensor([float(len(ptrs))])
        dist.all_reduce(total)
        dist.all_reduce(err, op=dist.ReduceOp.MAX)
        dist.all_reduce(n_buf, op=dist.ReduceOp.MIN)
        if rank == 0:
            q.put((float(total[0]), float(err[0]), mn, (lo, cnt), pipe.slice_prep, int(n_buf[0]), pipe.out_buffers))
        del pipe
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(1000)
@pytest.mark.parametrize("world,overlap,prep", [(2, False, "auto"), (4, True, "auto"), (8, True, "auto"),
                                                (8, True, "sharded")])
def test_syc_32_5_slice_mode_equals_single_gpu(world, overlap, prep):
    """The bench workload's multi-GPU path (slice mode, device data rank) at 2 ranks (plain steps) and
    at 4 and 8 ranks with pipelined steps (the multi-GPU bench default, BASELINE config 5: syc 32 5
    sharded over 8 GPUs; at 4 ranks two output buffers alternate, QKNIT_OUT_BUFFERS), with the
    preparation the cost model picks (replicated: no collective) and, at 8 ranks, the sharded one:
    the slice returned by EVERY one of four steps (a plain one, then pipelined ones: both output buffers
    at 4 ranks) equals the same range of the single-GPU step within 1e-12, the slices sum to 1 and no
    entry is below -1e-13. The exact-slice fallback is predicated on the device (no host sync in the step)."""
    total, err, mn, sl, chosen, n_buf, buffers = _run(_syc_worker, world, timeout=900, overlap=overlap, prep=prep)
    assert sl == (0, (1 << 32) // world)
    assert err <= TOL
    assert abs(total - 1.0) <= 1e-10
    assert mn >= -1e-13
    assert chosen == ("replicated" if prep == "auto" else prep)
    assert n_buf == (buffers if overlap else 1)


def _nccl_worker(rank, world, port, case, prep, buffers, veto, q):
    """One rank of a real RCCL group (world size 1: the test box has one GPU): slice mode forced,
    pipelined steps on the CU-masked streams, so every collective of the sharded step (all_to_all,
    Gram all_reduce, compressed-operand all_gather, MIN all_reduce, the async exact-operand
    all_gather) runs on nccl beside the masked write streams."""
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), QKNIT_SLICE_PREP=prep, QKNIT_POISON_UNUSED="1",
                      QKNIT_OUT_BUFFERS=str(buffers))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        _, cut = _case(case)
        virt = VirtualCircuit(cut)
        ref = None
        if case == "syc_32_5":
            one = KnitPipeline(virt, device=0, factored=True)
            ref = one.step().clone()
            del one
            torch.cuda.empty_cache()
        pipe = KnitPipeline(virt, device=0, rank=rank, world=world, mode="slice", factored=True,
                            group=dist.group.WORLD, data_rank=True)
        assert pipe.mode == "slice" and pipe.slice_prep == prep and pipe.dev_rank
        if veto:  # the probe check rejects: the predicated exact slice from the gathered operands
            pipe.rank_tol = pipe.rank_tol_rel = float("nan")
        torch.cuda.set_stream(torch.cuda.Stream())
        pipe.overlap = pipe.overlap_ok()
        assert pipe.overlap
        outs, errs = [], []
        for _ in range(4):
            out = pipe.step()
            torch.cuda.synchronize()
            if ref is not None:
                errs.append(float((out - ref).abs().max()))
            else:
                outs.append(out.cpu().numpy().copy())
        pipe.sync_stats()
        q.put((outs, errs, pipe.rank_fallbacks, pipe.last_rank, pipe.rank_incompressible, pipe.overlap_cus))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case,prep,buffers,veto", [
    ("hwe_p2", "sharded", 1, False), ("hwe_p2", "sharded", 2, False), ("hwe_p2", "sharded", 1, True),
    ("cx_8x8", "sharded", 2, False), ("hwe_p2", "replicated", 2, False), ("syc_32_5", "sharded", 1, False),
    ("syc_32_5", "replicated", 2, False), ("hwe_p2", "replicated", 3, True)])
def test_slice_mode_through_rccl(case, prep, buffers, veto):
    """Slice mode's collectives on RCCL (world size 1: one GPU per box; RCCL refuses two ranks on one
    device), pipelined steps on CU-masked streams with one or two output buffers: four steps each equal
    the oracle (small cases, 1e-12) or the single-GPU step (syc 32 5, all 2^32 entries, 1e-12);
    a forced rejection and cx_8x8's rank > 8 take the predicated exact slice from the gathered operands
    (replicated, three buffers: queued on the preparation stream ahead of the skipped write)."""
    from oracle import dense

    outs, errs, fallbacks, last_rank, incompressible, cus = _run(_nccl_worker, 1, case, prep, buffers, veto,
                                                                 timeout=500)
    assert cus is not None and cus[0] > 0
    if case == "syc_32_5":
        assert len(errs) == 4 and max(errs) <= TOL
        assert fallbacks == 0 and last_rank is not None
        return
    ref = dense.run_dense(_case(case)[1])
    for got in outs:
        np.testing.assert_allclose(got, ref, atol=TOL, rtol=0)
    if veto:
        assert fallbacks == 4 and last_rank is None
    elif case == "cx_8x8":
        assert incompressible == 4
    else:
        assert fallbacks == 0 and last_rank is not None


def _dict_worker(rank, world, port, q):
    """run_virtual_circuit(virt, group=WORLD) on syc 32 5 (2^32 outcomes): the reference-shaped dict on
    every rank, from the cached sharded plan, against the single-GPU result (computed first on rank 0)."""
    log = _watchdog(rank, f"dict_syc_32_5_{world}", after=800)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

        torch.cuda.set_device(0)
        _, cut = _case("syc_32_5")
        ref = {}
        if rank == 0:  # the single-GPU dict result (ACCURACY 1e-5) and the thresholded one at 3e-9
            one = KnitPipeline(VirtualCircuit(cut), device=0, factored=True)
            log("single-GPU plan built")
            for acc in (1e-5, 3e-9):
                ref[acc] = one.knit_dict(acc)
                log(f"single-GPU dict at {acc}: {ref[acc][0].size} entries")
            del one
            torch.cuda.empty_cache()
            log("single-GPU dicts done")
        dist.barrier()
        res, reused, digests = {}, [], []
        d, info = runmod.run_virtual_circuit(VirtualCircuit(cut), group=dist.group.WORLD)
        res[1e-5] = d
        plans = [p for k, p in runmod._PLANS.items() if "sharded" in k]
        assert len(plans) == 1
        reused.append(plans[0].plan_reused)
        log(f"dict 1e-5: {len(d)} entries, prep {plans[0].slice_prep}")
        d2, _ = runmod.run_virtual_circuit(VirtualCircuit(cut), group=dist.group.WORLD)  # second call: cached
        reused.append(plans[0].plan_reused)
        assert d2 == d
        keys, vals, _ = runmod._sharded_dict(VirtualCircuit(cut), None, 0, 3e-9)
        log(f"dict 3e-9: {keys.size} entries")
        digests = torch.tensor([float(keys.size), float(np.sum(keys % 1000003)), float(np.sum(vals))],
                               dtype=torch.float64)
        alld = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(alld, digests)
        same = all(bool(torch.equal(a, alld[0])) for a in alld)
        if rank == 0:
            ok_acc = d == dict(zip(ref[1e-5][0].tolist(), ref[1e-5][1].tolist()))
            ok_small = bool(np.array_equal(keys, ref[3e-9][0]) and np.array_equal(vals, ref[3e-9][1]))
            q.put((ok_acc, len(d), ok_small, int(keys.size), reused, same, info.shard))
        del keys, vals
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.timeout(1000)
def test_syc_32_5_sharded_dict_equals_single_gpu():
    """BASELINE config 5's reference-shaped result through run_virtual_circuit(virt, group=...) at 8
    ranks (gloo over the one test GPU): every rank returns the dict; it equals the single-GPU
    run_virtual_circuit(virt) result at ACCURACY 1e-5 (empty: no outcome of 2^32 reaches it) and, through
    the same sharded path at 3e-9 (2^28 kept entries: per-rank qk_knit_select of the slice, gathered,
    qk_npd_pairs), the single-GPU thresholded dict key for key and bit for bit; the second call reuses
    the cached plan (no re-planning, as the reference's per-call VirtualCircuit rebuild would need)."""
    ok_acc, n_acc, ok_small, n_small, reused, same, shard = _run(_dict_worker, 8, timeout=950)
    assert ok_acc and n_acc == 0
    assert ok_small and n_small > (1 << 27)
    assert reused == [False, True]
    assert same
    assert shard == (0, (1 << 32) // 8)
