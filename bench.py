#!/usr/bin/env python3
"""Benchmark of the knitting hot path on MI355X (BASELINE.json metric).

metric: subcircuit-instances/s + full-knit wall time, syc 32 p=2, 1/2/4/8 GPUs.
A step = one full run of the hot path for the workload: batched exact sweep of
every cut instance of every fragment + the dense fp64 knit of the complete
2^32-entry distribution (inputs = compiled plan, resident on the GPU).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload syc_32_5_p2] [--direct]
  N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
       or plain `python bench.py --gpus N`, which starts that launcher itself as a child process
       (WORLD_SIZE set and different from N is an error)

value = reference-counted instances (sum over fragments of their label lists, run.py:37-39)
processed per second by the whole job, timed between barriers, max over ranks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X dense FP64 matrix, spec (MI355X_MICROARCH.md has no measured f64 row)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X dense FP64 vector (v_fma_f64), spec
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="syc_32_5_p2")
    ap.add_argument("--direct", action="store_true",
                    help="direct knit over all global labels (K = prod n_inst) instead of the "
                         "default rank-factored knit (K = 4^cuts; exact, same result)")
    ap.add_argument("--no-light-cone", action="store_true",
                    help="plain factored knit: no light-cone basis projections, no core rank "
                         "compression (K = 4^cuts; exact, same result)")
    ap.add_argument("--no-data-rank", action="store_true",
                    help="contract the light-cone terms as they are (no per-step data-rank compression)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the syc 32 1 sweep-only measurement (north_star_sweep)")
    ap.add_argument("--no-sweep-full", action="store_true",
                    help="skip sweep_full (the direct plan's sweep of every unique instance, timed alone)")
    ap.add_argument("--cpu-sample-labels", type=int, default=12)
    ap.add_argument("--no-npd", action="store_true", help="skip the NPD timing on the 2^N output")
    ap.add_argument("--no-drop-in", action="store_true",
                    help="skip the drop_in block (run_virtual_circuit(virt, dense=True), first call + steady state)")
    ap.add_argument("--no-general", action="store_true",
                    help="skip knit_general (the same step without data-rank compression)")
    ap.add_argument("--pipeline", action="store_true",
                    help="one GPU: pipelined steps, the next step's sweep + data-rank preparation on a CU-masked "
                         "stream under the current step's write (DESIGN.md §4; off by default on one GPU)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="several GPUs: plain steps instead of the default pipelined ones")
    return ap.parse_args()


def cpu_baseline(cut, n_labels_sample: int):
    """Oracle (numpy) timing on a bounded sample of the same workload, extrapolated."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import dense, qvm
    from oracle.statevector import simulate

    try:
        from threadpoolctl import threadpool_info

        threads = max([t.get("num_threads", 1) for t in threadpool_info()] + [1])
    except Exception:
        threads = os.cpu_count() or 1
    view = qvm.CutView(cut)
    frags = [list(r) for r in view.qregs if len(r)]
    t0 = time.perf_counter()
    done = 0
    per_frag_labels = []
    for f in frags:
        labels = view.labels(f)
        per_frag_labels.append(len(labels))
        cl = dense.fragment_clbits(view, f)
        for label in labels[:n_labels_sample]:
            d = simulate(view.instance_ops(f, label), len(f))
            dense.fold(d, view.num_clbits, cl)
            done += 1
    t_inst = (time.perf_counter() - t0) / max(done, 1)
    # knit: one GEMM slice of the contraction (same K and N, a block of M rows)
    L = len(view.global_labels())
    widths = [1 << len(dense.fragment_clbits(view, f)) for f in frags]
    M = widths[0]
    Nw = int(np.prod(widths[1:])) if len(widths) > 1 else 1
    rows = min(M, 512)
    rng = np.random.default_rng(0)
    A = rng.standard_normal((L, rows))
    B = rng.standard_normal((L, Nw))
    t1 = time.perf_counter()
    A.T @ B
    t_knit = (time.perf_counter() - t1) * (M / rows)
    total_inst = sum(per_frag_labels)
    t_total = t_inst * total_inst + t_knit
    return {
        "value": total_inst / t_total,
        "unit": "instances/s",
        "cores": int(threads),
        "kind": "port",
        "sample": (f"oracle numpy: {done} instances exactly simulated (branching statevector, "
                   f"{t_inst * 1e3:.1f} ms each) + knit GEMM slice {rows}x{Nw}x{L} "
                   f"(numpy BLAS, {threads} threads), extrapolated to {total_inst} instances and "
                   f"{M}x{Nw}x{L}: {t_total:.1f} s per full knit"),
        "full_knit_s": t_total,
    }


QVM_MAX_CLBITS = 20  # literal dict knit cap: 2^N dict entries per merged label (syc 32: DNF)


def host_info() -> dict:
    """Cores this process may run on (``sched_getaffinity``) and the host CPU model."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"affinity_cores": len(os.sched_getaffinity(0)), "cpu_model": model}


def cpu_baseline_qvm(cut, processes: int = 8, accuracy: float = 1e-5, return_result: bool = False) -> dict:
    """The reference's own CPU algorithm, restated (``oracle/qvm.py``): exact instance
    distributions (numpy statevector in place of Aer's sampling, ``run.py:36-58``), then the
    literal dict merge + per-gate knit through ``Pool(processes)`` (``run.py:64-67``,
    ``virtual_circuit.py:50-68,216-228``) with ``QuasiDistr``'s shipped ``ACCURACY`` truncation,
    then ``nearest_probability_distribution`` (``run.py:71``). Timed as ``RunTimeInfo``. Outputs of
    more than ``QVM_MAX_CLBITS`` clbits (syc 32: 2^32 dict entries) are reported DNF."""
    from multiprocessing import Pool

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import qvm

    n = sum(len(c) for c in cut.cregs)
    info = {"kind": "port", "algorithm": "qvm literal: exact instances + dict merge/knit in Pool(%d)" % processes,
            "processes": processes, **host_info()}
    if n > QVM_MAX_CLBITS:
        return {**info, "status": "DNF", "reason": f"{n} clbits: the dict knit holds up to 2^{n} entries per "
                                                   f"label (cap {QVM_MAX_CLBITS} clbits)"}
    times = {}
    t0 = time.perf_counter()
    pool = Pool(processes=processes)
    try:
        _, npd = qvm.run(cut, accuracy, pool=pool, times=times)
    finally:
        _close_pool(pool)
    wall = time.perf_counter() - t0
    view = qvm.CutView(cut)
    inst = sum(len(view.labels(list(r))) for r in view.qregs if len(r))
    out = {**info, "status": "ok", "run_time_s": times["run_time"], "knit_time_s": times["knit_time"],
           "wall_s": wall, "instances_ref": inst, "value": inst / (times["run_time"] + times["knit_time"]),
           "unit": "instances/s", "result_entries": len(npd)}
    if return_result:
        out["result"] = dict(npd)
    return out


_KW = {}


def _close_pool(pool) -> None:
    """Stop a worker pool and reap every worker (``with Pool()`` only terminates them: the driver saw
    a child process still alive when the bench exited)."""
    pool.close()
    pool.join()


def cpu_workers() -> tuple[int, str]:
    """Worker processes of the CPU baselines: the box's per-GPU CPU share (``OMP_NUM_THREADS``, which
    the GPU pool sets to it; its rules cap worker pools there, while ``sched_getaffinity`` lists every
    core of the host), else every core this process may run on."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) < aff:
        return int(env), f"OMP_NUM_THREADS={env}: the GPU box's CPU share per GPU ({aff} host cores visible)"
    return aff, "all cores in sched_getaffinity"


def _byte_pext_tables(clbits):
    import numpy as np

    t = np.zeros((4, 256), dtype=np.int64)
    for byte in range(4):
        for v in range(256):
            x = v << (8 * byte)
            t[byte, v] = sum(1 << j for j, c in enumerate(clbits) if (x >> c) & 1)
    return t


def _instance_worker(job):
    """One exact instance (oracle statevector + signed fold) of the cut in _KW (forked worker)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import dense
    from oracle.statevector import simulate

    fi, li = job
    view, f = _KW["view"], _KW["frags"][fi]
    dense.fold(simulate(view.instance_ops(f, view.labels(f)[li]), len(f)), view.num_clbits,
               dense.fragment_clbits(view, f))
    return fi


def _knit_worker_init(A2, B2, tA, tB):
    _KW.update(A2=A2, B2=B2, tA=tA, tB=tB)


def _knit_worker_chunk(rng):
    """Outputs [lo, hi) of the compressed two-fragment knit in output order (numpy; one process)."""
    import numpy as np

    lo, hi = rng
    A2, B2, tA, tB = _KW["A2"], _KW["B2"], _KW["tA"], _KW["tB"]
    o = np.arange(lo, hi, dtype=np.int64)
    ia = tA[0][o & 255] | tA[1][(o >> 8) & 255] | tA[2][(o >> 16) & 255] | tA[3][(o >> 24) & 255]
    ib = tB[0][o & 255] | tB[1][(o >> 8) & 255] | tB[2][(o >> 16) & 255] | tB[3][(o >> 24) & 255]
    out = np.take(A2[0], ia) * np.take(B2[0], ib)
    for k in range(1, A2.shape[0]):
        out += np.take(A2[k], ia) * np.take(B2[k], ib)
    return float(out.sum())


def cpu_baseline_same(pipe, cut, qs_host, n_inst_sample: int = 8, out_block_bits: int = 24) -> dict:
    """The builder's algorithm on the host cores (one process per core; numpy + BLAS threads for
    the transforms), timed on a bounded sample of the syc 32 5 step and extrapolated (factors
    stated): exact instances (oracle statevector: one batch of one instance per process, scaled
    to the swept instance count), then on the
    real swept rows (copied from the GPU run): operand transforms, Grams, data-rank factors
    (data_rank.rank_factors, the host form of qk_rank_factors), compressed operands, the 16-probe
    check, and the streaming knit (byte-table pext index gathers, numpy) of 4 x procs chunks of
    2^(out_block_bits - 2) outputs spread over one process per host core, scaled to 2^N."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import dense, qvm
    from oracle.statevector import simulate

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import data_rank

    from multiprocessing import Pool

    view = qvm.CutView(cut)
    frags = [list(r) for r in view.qregs if len(r)]
    procs, procs_why = cpu_workers()
    jobs = []
    for fi, f in enumerate(frags):
        jobs += [(fi, li) for li in range(min(len(view.labels(f)), max(1, procs // len(frags))))]
    _KW.update(view=view, frags=frags)  # inherited by the forked workers
    pool = Pool(procs)
    try:
        t0 = time.perf_counter()
        pool.map(_instance_worker, jobs)  # one exact instance per process, all at once
        t_batch = time.perf_counter() - t0
    finally:
        _close_pool(pool)
    done = len(jobs)
    t_inst = t_batch  # wall time of one concurrent batch of `done` instances
    swept = pipe.instance_counts()["instances_swept"]
    t_sweep = t_batch * -(-swept // done)
    ia, ib = pipe.order[0], pipe.order[-1]
    t1 = time.perf_counter()
    A = pipe.row_transform(ia) @ qs_host[ia]
    B = pipe.row_transform(ib) @ qs_host[ib]
    f = data_rank.rank_factors(A @ A.T, B @ B.T)
    TA, TB = f
    A2, B2 = TA @ A, TB @ B
    x = np.random.default_rng(1234).standard_normal((B.shape[1], 16))
    err = np.linalg.norm(A.T @ (B @ x) - A2.T @ (B2 @ x), axis=0).max()
    t_prep = time.perf_counter() - t1
    cA, cB = pipe.ops.clbits[ia], pipe.ops.clbits[ib]
    chunk = 1 << (out_block_bits - 2)
    tasks = 4 * procs
    nblk = chunk * tasks
    pool = Pool(procs, initializer=_knit_worker_init, initargs=(A2, B2, _byte_pext_tables(cA), _byte_pext_tables(cB)))
    try:
        pool.map(_knit_worker_chunk, [(0, 1024)] * procs)  # workers up
        t2 = time.perf_counter()
        out = pool.map(_knit_worker_chunk, [(i * chunk, (i + 1) * chunk) for i in range(tasks)])
        t_blk = time.perf_counter() - t2
    finally:
        _close_pool(pool)
    scale = (1 << pipe.N) // nblk
    total = t_sweep + t_prep + t_blk * scale
    del out
    aff = len(os.sched_getaffinity(0))
    return {
        "value": pipe.instance_counts()["instances_ref"] / total,
        "unit": "instances/s",
        "cores": int(procs),
        "cores_why": procs_why,
        # every visible core at perfect scaling (an upper bound on this baseline, not measured)
        "value_all_cores_bound": pipe.instance_counts()["instances_ref"] / total * aff / procs,
        "kind": "port",
        "algorithm": "same as the GPU step (basis-reduced exact instances, factored light-cone knit, "
                     "data-rank compression, output-order write)",
        **host_info(),
        "sample": (f"{done} exact instances at once on {procs} processes in {t_inst * 1e3:.0f} ms "
                   f"(x{-(-swept // done)} batches to the {swept} swept); transforms + Grams + factors + probes on the real swept rows "
                   f"{t_prep * 1e3:.0f} ms (rank {A2.shape[0]}, probe err {err:.1e}); knit of {nblk} outputs "
                   f"on {procs} processes {t_blk * 1e3:.0f} ms (x{scale} to 2^{pipe.N}): {total:.1f} s per full knit"),
        "full_knit_s": total,
    }


def knit_general(pipe_kw: dict, steps: int) -> dict:
    """The same workload without the per-step data-rank compression: the K = 64 light-cone
    contraction on the MFMA kernel (qk_gemm_glds_kernel), its own timing and roofline."""
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    pipe = KnitPipeline(data_rank=False, **pipe_kw)
    for _ in range(2):
        pipe.step()
    torch.cuda.synchronize()
    pipe.record_events = True
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    gemm_ms = sum(s.elapsed_time(e) for s, e in pipe.events) / max(len(pipe.events), 1)
    M, N, K = pipe.gemm_shape()
    flops = 2.0 * M * N * K
    out = {"ms_per_step": ms, "kernel": "qk_gemm_wave_kernel<16> (K = %d light-cone terms, fp64 MFMA "
                                         "v_mfma_f64_16x16x4_f64, per-wave LDS rings)" % K,
           "gemm_mnk": [M, N, K], "avg_launch_ms": gemm_ms, "achieved_TFs": flops / (gemm_ms * 1e-3) / 1e12,
           "peak_TFs": FP64_MFMA_PEAK_TFLOPS, "frac": flops / (gemm_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
           "traffic": traffic_per_launch(M, N, K)}
    # MFMA counters of the same contraction (profiles/*gemm_k64_pmc.json, tools/gemm_pmc_json.py): the
    # counted fp64 MFMA flops (512 x SQ_INSTS_VALU_MFMA_MOPS_F64) over THIS run's launch time, and the
    # profiled run's MFMA busy fraction and clock (the spec peak assumes 2.4 GHz; a power-limited clock
    # lowers the reachable rate in proportion)
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*gemm_k64_pmc.json"))):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("gemm_mnk") == [M, N, K] and "mfma_busy_frac" in rec:
            out["counters"] = {"source": os.path.basename(f), "flops_counted": rec["flops_counted"],
                               "counted_TFs_this_run": rec["flops_counted"] / (gemm_ms * 1e-3) / 1e12,
                               "frac_counted": rec["flops_counted"] / (gemm_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                               "mfma_busy_frac_profiled": rec["mfma_busy_frac"],
                               "effective_clock_GHz_profiled": rec["effective_clock_GHz"],
                               "hbm_bytes_per_launch": rec["hbm_bytes_per_launch"]}
    del pipe
    torch.cuda.empty_cache()
    return out


def drop_in_timing(cut, ref_out, steps: int, device: int) -> dict:
    """The reference API on the same workload: ``run_virtual_circuit(virt, dense=True)``
    (``run.py:23-71``, called at ``Utilities.py:79``), which runs the cached plan of the benched
    engine. ``first_call_ms``: plan cache empty (fragment compile, job tables, transforms, uploads;
    the hiprtc sweep modules are already cached in this process by the bench's own pipeline);
    ``steady_ms``: later calls on a fresh ``VirtualCircuit`` of the same cut (the plan is found by the
    circuit's content hash), each result freed before the next call; ``reselect_calls_ms``: a call
    that replaced the first call's un-checked output mapping (its write was below the write-rate stop)
    by a selected one, reported apart from the steady state. ``max_abs_diff_vs_step``: the drop-in's
    distribution against the bench step's output, every one of the 2^N entries."""
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import clear_plan_cache, run_virtual_circuit

    clear_plan_cache()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    virt0 = VirtualCircuit(cut)
    out, info = run_virtual_circuit(virt0, dense=True, device=device)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import cached_plan

    plan0 = cached_plan(virt0, device)
    placement = getattr(plan0, "out_alloc", None)
    breakdown = {k: round(v, 2) for k, v in getattr(plan0, "first_call_ms", {}).items()}
    diff = 0.0
    chunk = 1 << 28
    for i in range(0, out.numel(), chunk):
        diff = max(diff, float((out[i:i + chunk] - ref_out[i:i + chunk]).abs().max()))
    del out
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    times, infos, builds, reselect = [], [], [], []
    for _ in range(max(steps, 3)):
        tb = time.perf_counter()
        virt = VirtualCircuit(cut)  # the reference builds one per call (Utilities.py:74-79)
        builds.append(time.perf_counter() - tb)
        n_sel = len(engine.out_selections)
        t0 = time.perf_counter()
        out, info = run_virtual_circuit(virt, dense=True, device=device)
        dt = time.perf_counter() - t0
        if len(engine.out_selections) > n_sel:
            # this call replaced the first call's un-checked output mapping by a write-rate-selected one
            # (its own write was slow: run.py / KnitPipeline.take_out): reported apart
            reselect.append(dt)
        else:
            times.append(dt)
            infos.append(info)
        del out
    # the reference-shaped result (run.py:71): entries above ACCURACY + NPD, thresholded knit
    dict_times, entries = [], 0
    # the first dict call allocates the select / NPD buffers of this plan (reported apart, as the dense
    # API's first call is); steady state = the calls after it
    t0 = time.perf_counter()
    run_virtual_circuit(VirtualCircuit(cut), device=device)
    dict_first = time.perf_counter() - t0
    for _ in range(max(steps, 3)):
        virt = VirtualCircuit(cut)
        t0 = time.perf_counter()
        res, _ = run_virtual_circuit(virt, device=device)
        dict_times.append(time.perf_counter() - t0)
        entries = len(res)
    clear_plan_cache()
    torch.cuda.empty_cache()
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import quasi_distr

    return {"api": "run_virtual_circuit(virt, dense=True)", "first_call_ms": first * 1e3,
            "first_call_breakdown_ms": breakdown,
            "dict_api": "run_virtual_circuit(virt): qk_knit_select (entries above ACCURACY only) + qk_npd_pairs",
            "dict_first_ms": dict_first * 1e3,
            "dict_steady_ms": float(sum(dict_times) / len(dict_times)) * 1e3, "dict_min_ms": min(dict_times) * 1e3,
            "dict_entries": entries, "accuracy": quasi_distr.ACCURACY,
            "steady_ms": float(sum(times) / len(times)) * 1e3, "steady_min_ms": min(times) * 1e3,
            "reselect_calls_ms": [round(x * 1e3, 2) for x in reselect],
            "run_time_ms": float(sum(i.run_time for i in infos) / len(infos)) * 1e3,
            "knit_time_ms": float(sum(i.knit_time for i in infos) / len(infos)) * 1e3,
            "calls": len(times) + len(reselect), "max_abs_diff_vs_step": diff, "out_alloc": placement,
            # host: VirtualCircuit(cut) per call (fragment circuits + the cut's content hash, the plan key)
            "virtual_circuit_ms": float(sum(builds) / len(builds)) * 1e3}


def npd_timing(dense, accuracy: float) -> dict:
    """``QuasiDistr`` truncation + ``nearest_probability_distribution`` (quasi_distr.py:7-10,28-43,
    run.py:71) on the GPU over the step's 2^N output: qk_threshold_count then qk_npd, timed apart
    from the knit."""
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine

    ctx = engine.get_context(dense.device.index or 0)
    engine.nearest_probability_distribution(ctx, dense, accuracy)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    keys, vals = engine.nearest_probability_distribution(ctx, dense, accuracy)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    return {"ms": ms, "accuracy": accuracy, "kept_entries": int(len(keys)), "entries": int(dense.numel()),
            "sum_kept": float(vals.sum()) if len(vals) else 0.0}


def north_star_sweep(steps: int) -> dict:
    """BASELINE.json north-star target: the batched statevector sweep for syc 32 1 at p=2 on one
    MI355X against the HBM roofline. Per variant (the reference cut: 0 cuts, 2 instances; the
    forced 4-cut variant: the full 4^k instance batch) the sweep of every fragment is timed alone
    with HIP events on the launch stream. ``hbm_frac``: the bytes the kernels actually move (modelled,
    DESIGN.md §3) / time / 8 TB/s. ``model_bytes_frac``: SURVEY.md §8d's per-gate algorithmic bytes
    (one read + write of the complex128 state per fused op per branch job) on the same scale — a
    model, not a ceiling (a pass touches the state once for all its gates, so it exceeds 1). With
    one or a few 16-qubit instances the sweep is latency-bound: two dependent launches (INIT, FINAL)
    of a few microseconds each, ~1 MB of state."""
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    out = {}
    for key in ("syc_32_1_p2", "syc_32_1_p2_forced"):
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        _, cut, desc = cutting.config_cut_circuit(name, n, d, p, var)
        # per-program kernels even for this small batch: the 2-instance sweep is latency-bound
        pipe = KnitPipeline(VirtualCircuit(cut), factored=(var == "forced"), jit=True)

        def timed(fn):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(steps):
                fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) / steps

        ways = {("eager, one launch per pass round for all fragments" if pipe._multi is not None
                 else "eager, fragments in sequence"): timed(pipe.sweep)}
        pipe.fork = True  # one stream per fragment (independent sweeps overlap)
        ways["eager, fragments on forked streams"] = timed(pipe.sweep)
        pipe.capture_sweep()  # the same launches as one HIP graph
        ways["hipGraph replay, forked streams"] = timed(pipe.replay_sweep)
        launch = min(ways, key=ways.get)
        ms = ways[launch]
        tr = pipe.sweep_traffic()
        counts = pipe.instance_counts()
        out[key] = {
            "workload": f"{name} {n} {d} p={p}" + (" (forced cuts)" if var == "forced" else ""),
            "cuts": desc,
            "instances_ref": counts["instances_ref"],
            "branch_jobs": counts["branch_jobs"],
            "ms_per_sweep": ms,
            "launch": launch,
            "ms_by_launch": ways,
            "bound": "latency (2 dependent launches, single-instance 16-qubit fragments)",
            "hbm_bytes": tr["hbm"],
            "hbm_frac": tr["hbm"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "algorithmic_bytes_model": tr["algorithmic"],
            "model_bytes_frac": tr["algorithmic"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        }
        del pipe
        torch.cuda.empty_cache()
    return out


def sweep_full(steps: int) -> dict:
    """The sweep kernels at a size where HBM could matter (verdict r5, north_star "HBM GB/s on the
    batched statevector sweep"): syc 32 5 with basis reduction, light cone and row pruning off —
    the direct plan's sweep of every unique instance of both 16-qubit fragments with all their branch
    jobs (2 x 625 instances of the reference's 2 x 1296, 2 x 1296 branch jobs), timed alone with HIP
    events on the launch stream. ``algorithmic_bytes``: SURVEY.md §8d (one read + write of the
    complex128 state per fused gate per branch job) — a model that counts every gate as a pass over
    HBM, not a ceiling (a pass touches the state once for all of its gates). ``counters``: the
    profiled HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) and fp64 VALU instructions of
    the same sweep (profiles/*sweep_full_pmc.json, rocprofv3 --pmc passes over tools/sweep_run.py
    --full), divided by THIS run's time: the fractions of 8 TB/s and of the 78.6 TF/s fp64 vector peak
    that bound it."""
    import torch

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=False)
    for _ in range(2):
        pipe.sweep()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        pipe.sweep()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / steps
    tr = pipe.sweep_traffic()
    counts = pipe.instance_counts()
    out = {"workload": "syc 32 5 p=2, direct plan (no basis reduction / light cone / row pruning)",
           "instances_ref": counts["instances_ref"], "instances_swept": counts["instances_swept"],
           "branch_jobs": counts["branch_jobs"], "ms_per_sweep": ms,
           "hbm_bytes_model": tr["hbm"], "hbm_GBs_model": tr["hbm"] / (ms * 1e-3) / 1e9,
           "algorithmic_bytes": tr["algorithmic"], "algorithmic_GBs": tr["algorithmic"] / (ms * 1e-3) / 1e9,
           "fp64_flops_model": tr["flops"]}
    cnt = sweep_counters("syc 32 5 p=2 (full sweep)", pattern="*sweep_full_pmc.json")
    if cnt is not None:
        src, c = cnt
        out.update({"counters": src, "hbm_bytes": c["hbm_bytes"],
                    "hbm_GBs": c["hbm_bytes"] / (ms * 1e-3) / 1e9,
                    "hbm_frac": c["hbm_bytes"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    "fp64_flops": c["fp64_flops"], "fp64_TFs": c["fp64_flops"] / (ms * 1e-3) / 1e12,
                    "fp64_valu_frac": c["fp64_flops"] / (ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS})
        for k in ("f64_issue_frac", "valu_busy_frac", "lds_bank_conflict_frac", "per_kernel"):
            if k in c:
                out[k] = c[k]
        out["bound"] = ("fp64 VALU issue" if c.get("valu_busy_frac", 0) > out["hbm_frac"] else "HBM")
    del pipe
    torch.cuda.empty_cache()
    return out


def traffic_per_launch(M, N, K):
    """HBM bytes per knit-GEMM launch from the committed PMC summary (profiles/*traffic*.json,
    written by tools/pmc_traffic.py from a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass of this
    bench), matched on the GEMM shape; None if no summary for this shape exists."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("gemm_mnk") == [M, N, K]:
            best = rec
    return None if best is None else best["hbm_bytes_per_launch"]


def sweep_counters(workload: str, pattern: str = "*sweep_pmc.json"):
    """Counter-measured sweep bytes / flops per step (profiles/*sweep_pmc.json, written from
    rocprofv3 --pmc passes over tools/sweep_bench.py): the HBM bytes the sweep kernels really moved
    (2 x FETCH_SIZE + WRITE_SIZE) and the fp64 flops they executed (SQ_INSTS_VALU_{ADD,MUL,FMA}_F64),
    per step, for the workload; None without a summary."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("workload", "") == workload or (pattern == "*sweep_pmc.json" and rec.get("workload", "").startswith(workload)):
            best = (os.path.basename(f), rec["per_step"])
    return best


def launch_plan(gpus: int, env) -> tuple:
    """What ``bench.py --gpus N`` does in this environment (checked before anything touches a GPU):
    ("run", world) — this process is one rank (WORLD_SIZE set by a launcher, equal to N; or N = 1);
    ("spawn", N) — no launcher: start N ranks as a child ``torch.distributed.run`` and relay its line
    (the reference spreads its knit over ``Pool(processes=8)`` itself, run.py:64-67);
    ("error", message) — a launcher's WORLD_SIZE that contradicts --gpus."""
    if gpus < 1:
        return ("error", f"--gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        return ("spawn", gpus) if gpus > 1 else ("run", 1)
    try:
        world = int(ws)
    except ValueError:
        return ("error", f"WORLD_SIZE={ws!r} is not an integer")
    if world != gpus:
        return ("error", f"--gpus {gpus} but WORLD_SIZE={world}: the launcher started a different number of "
                         f"ranks than the job asks for")
    return ("run", world)


def spawn_command(gpus: int, argv: list, port: int) -> list:
    """The child launcher's command line: one process per GPU of this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def spawn_ranks(gpus: int, argv: list) -> int:
    """Run the N-rank bench as a child process (nothing here has touched the GPU) and relay its output;
    returns the child's exit code. The JSON line is rank 0's (the ranks' max-over-ranks timing)."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = spawn_command(gpus, argv, port)
    print(f"bench.py: no launcher, starting {gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:  # relay as it comes (the JSON line included)
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def main():
    args = parse()
    plan = launch_plan(args.gpus, os.environ)
    if plan[0] == "error":
        print(f"bench.py: {plan[1]}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan[0] == "spawn":
        sys.exit(spawn_ranks(plan[1], sys.argv[1:]))
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # QKNIT_DIST_BACKEND=gloo + fewer GPUs than ranks: a rehearsal of the multi-GPU path with
        # several ranks per device (RCCL refuses that); the default is RCCL, one rank per GPU
        backend = os.environ.get("QKNIT_DIST_BACKEND", "nccl")
        if backend != "nccl":
            local %= torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, variant = cutting.BASELINE_CONFIGS[args.workload]
    circ, cut, desc = cutting.config_cut_circuit(name, n, d, p, variant)
    virt = VirtualCircuit(cut)
    torch.cuda.set_device(local)
    # all work on a non-default stream: pipelined steps keep the legacy null stream idle
    torch.cuda.set_stream(torch.cuda.Stream())
    pipe = KnitPipeline(virt, device=local, factored=not args.direct, rank=rank, world=world,
                        light_cone=not args.no_light_cone, data_rank=False if args.no_data_rank else None)
    # pipelined steps: step i+1's sweep + data-rank preparation (+ its collectives) run on a CU-masked
    # stream while step i's write streams on the other CUs; every step still does all of its work.
    # Default on several GPUs (rank_sim with modelled xGMI, 8 ranks: 0.96 ms vs 1.17 ms per step,
    # profiles/r03_rank_sim.jsonl), opt-in (--pipeline) on one (measured 6.28 vs 6.20 ms: the write
    # loses more on 160 CUs than the 0.37 ms of sweep + preparation it hides)
    want = args.pipeline if world == 1 else not args.no_pipeline
    pipe.overlap = bool(want and pipe.overlap_ok())
    counts = pipe.instance_counts()

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    for _ in range(args.warmup):
        pipe.step()
    # pipelined steps: their rotating output buffers are made and selected here, not in a timed step
    # (with --warmup 1 the second step would make them)
    pipe.prepare_pipelined()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    pipe.record_events = True
    pipe.events.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pipe.sync_stats()  # device data rank: accepted ranks / fallbacks of the timed steps
    gemm_ms = sum(s.elapsed_time(e) for s, e in pipe.events) / max(len(pipe.events), 1)
    pipelined = None
    if pipe.overlap:
        # the latency of one full knit (plain steps: nothing of the next step runs under the write), and
        # the sweep / preparation times on the whole chip
        pipelined = {"prep_cus": pipe.overlap_cus[0], "write_cus": pipe.overlap_cus[1],
                     "out_buffers": pipe.out_buffers,
                     "ms_per_step_pipelined": elapsed / args.steps * 1e3,
                     "pipelined_write_ms": gemm_ms}
        pipe.overlap = False
        pipe.step()
        pipe.events.clear()
        pipe.sweep_events.clear()
        pipe.prep_events.clear()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            pipe.step()
        torch.cuda.synchronize()
        pipelined["full_knit_latency_ms"] = (time.perf_counter() - t1) / args.steps * 1e3
        pipelined["plain_write_ms"] = sum(s.elapsed_time(e) for s, e in pipe.events) / max(len(pipe.events), 1)
        pipe.sync_stats()
    sweep_ms = sum(s.elapsed_time(e) for s, e in pipe.sweep_events) / max(len(pipe.sweep_events), 1)
    traffic = pipe.sweep_traffic()
    M, Nn, K = pipe.gemm_shape()
    flops = 2.0 * M * Nn * K
    # algorithmic bytes of the contraction: both operands read once, the output written once
    gbytes = 8.0 * (M * Nn + K * (M + Nn))
    t_mfma, t_hbm = flops / (FP64_MFMA_PEAK_TFLOPS * 1e12), gbytes / (HBM_PEAK_GBS * 1e9)
    if t_mfma >= t_hbm:
        roof = {"bound": "mfma", "achieved": flops / (gemm_ms * 1e-3) / 1e12, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s"}
    else:
        roof = {"bound": "hbm", "achieved": gbytes / (gemm_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    kernel = ("qk_knit_outer_blocked_kernel (data-rank knit: 2^16-output tasks, operands staged in LDS, "
              "output-write bound)" if pipe.last_kernel == "qk_knit_outer_blocked_kernel" else
              "qk_knit_outer_stream_kernel (data-rank knit written in output order, output-write bound)"
              if pipe.last_kernel == "qk_knit_outer_stream_kernel" else
              "qk_gemm_smallk_kernel<true> (data-rank knit: keyed outer product, output-write bound)"
              if pipe.last_kernel == "qk_gemm_smallk_kernel<true>" else
              "qk_gemm_smallk_kernel (knit outer product, output-write bound)" if K <= 8 else
              "qk_gemm_glds_kernel (knit contraction, LDS-DMA ring)" if K % 16 == 0 else
              "qk_gemm_keyed_kernel (knit contraction, register-staged)")
    if rank != 0:
        return
    ms_per_step = elapsed / args.steps * 1e3
    value = counts["instances_ref"] * args.steps / elapsed
    line = {
        "metric": "subcircuit-instances/s (full-knit wall time = ms_per_step), syc 32 p=2",
        "value": value,
        "unit": "instances/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded circuit generators, random.seed(1234))",
        "config": {
            "workload": f"{name} {n} {d} p={p}" + (" (forced cuts)" if variant == "forced" else ""),
            "cuts": desc,
            "instances_ref": counts["instances_ref"],
            "instances_unique": counts["instances_unique"],
            "instances_swept": counts["instances_swept"],
            "rows_swept": counts["rows_swept"],
            "branch_jobs": counts["branch_jobs"],
            "labels": counts["labels_ref"],
            "knit": ("direct" if args.direct else
                     "factored" + ("" if args.no_light_cone else ", light-cone basis + rank-compressed core")
                     + (", data-rank compressed per step" if pipe.data_rank else "")),
            "knit_terms": {"labels": counts["labels_ref"], "factored": counts["terms_factored"],
                           "light_cone": counts["labels"], "contracted": K,
                           "data_rank": pipe.data_rank, "rank_fallbacks": pipe.rank_fallbacks,
                           "device_rank": pipe.dev_rank},
            "gemm_mnk": [M, Nn, K],
            "output_entries": 1 << pipe.N,
            "parallelism": f"labels x{world} ({pipe.mode})",
            "slice_prep": pipe.slice_prep,  # slice mode: "replicated" (no collective) or "sharded"
            "slice_cost_model_ms": pipe.slice_costs,
        },
        "roofline": {
            "kernel": kernel,
            **roof,
            "frac": roof["achieved"] / roof["peak"],
            "traffic": traffic_per_launch(M, Nn, K),
            "flops_per_launch": flops,
            "algorithmic_bytes_per_launch": gbytes,
            "avg_launch_ms": gemm_ms,
        },
        "sweep": {
            "kernel": "per-program sweep kernels (sweep_codegen + hiprtc): shared INIT tiles (one per distinct "
                      "INIT-slot prefix), FINAL pass on narrowed single-wave tiles summing each label's branch "
                      "jobs, labels heaviest first, XCD-grouped tile order (all fragments, per step, this rank)",
            "bound": "latency: 250 branch jobs after row pruning (the column side's 192 rows the knit does not "
                     "depend on are not swept; 750 before): the FINAL pass is 8320 single-wave workgroups at 2 "
                     "waves per SIMD (172 VGPRs, 16-KiB tiles), VALU busy 0.46 of its cycles, f64 issue 0.37 "
                     "(mostly adds: the normalised +-1/+-i gate entries fold multiplies away), waves waiting 0.33 "
                     "of their cycles; its last fiber group is reached by v_permlane16/32_swap butterflies, not "
                     "LDS (round 6); the INIT pass is one wave's serial op chain per prefix; HBM ~0.09 GB per step "
                     "(counters, profiles/r04s2_sweep_pmc.json); at scale see sweep_full",
            "ms_per_step": sweep_ms,
            "branch_jobs": counts["branch_jobs"],
            "hbm_bytes_model": traffic["hbm"],
            "hbm_GBs_model": traffic["hbm"] / (sweep_ms * 1e-3) / 1e9,
            "algorithmic_bytes": traffic["algorithmic"],
            "algorithmic_GBs": traffic["algorithmic"] / (sweep_ms * 1e-3) / 1e9,
            "fp64_flops_model": traffic["flops"],
        },
    }
    cnt = sweep_counters(line["config"]["workload"]) if world == 1 else None
    if cnt is not None:  # counter bytes / flops per step (one GPU's whole sweep), over this run's sweep time
        src, c = cnt
        line["sweep"].update({
            "counters": src,
            "hbm_bytes": c["hbm_bytes"],
            "hbm_GBs": c["hbm_bytes"] / (sweep_ms * 1e-3) / 1e9,
            "hbm_frac": c["hbm_bytes"] / (sweep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "fp64_flops": c["fp64_flops"],
            "fp64_TFs": c["fp64_flops"] / (sweep_ms * 1e-3) / 1e12,
            "fp64_valu_frac": c["fp64_flops"] / (sweep_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS,
        })
        for k in ("f64_issue_frac", "valu_busy_frac"):  # SIMD issue cycles over the counted run's step
            if k in c:
                line["sweep"][k] = c[k]
    if pipe.out_alloc is not None:
        # the output buffer: one allocation, mapped from 1-GiB physical chunks (qk_out_alloc)
        line["out_alloc"] = pipe.out_alloc
    prep = [s.elapsed_time(e) for s, e in pipe.prep_events]
    if prep:
        line["rank_compress_ms"] = sum(prep) / len(prep)  # sweep end -> knit start (transforms, factors, probes)
    if pipelined is not None and roof["bound"] == "hbm":
        # pipelined steps overlap out_buffers writes, so one launch's duration spans several steps: the
        # rank's HBM rate is the step's algorithmic bytes over the step time (the per-launch figure above
        # follows the contract's definition)
        per_step = gbytes / (ms_per_step * 1e-3) / 1e9
        line["roofline"]["per_step"] = {"achieved": per_step, "frac": per_step / HBM_PEAK_GBS,
                                        "concurrent_writes": pipe.out_buffers,
                                        "note": "algorithmic bytes of one step's write / ms_per_step"}
    if pipelined is not None:
        pipelined["note"] = ("value / ms_per_step: pipelined steps (step i+1's sweep + data-rank preparation on "
                             f"{pipelined['prep_cus']} CUs under step i's write on the other {pipelined['write_cus']}); "
                             "full_knit_latency_ms: plain steps, one full knit each; roofline: the write launches of "
                             "the timed (pipelined) steps; sweep / rank_compress_ms: the plain steps (whole chip)")
        line["pipelined"] = pipelined
    if world == 1 and not args.no_npd:
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import quasi_distr

        line["npd"] = npd_timing(pipe.out, quasi_distr.ACCURACY)
    if world == 1 and not args.no_drop_in:
        line["drop_in"] = drop_in_timing(cut, pipe.out, args.steps, local)
        line["drop_in"]["vs_ms_per_step"] = line["drop_in"]["steady_ms"] / ms_per_step
    qs_host = None
    if world == 1 and not args.no_cpu_baseline and pipe.dev_rank:
        qs_host = [q.contiguous().cpu().numpy() for q in pipe.sweep()]
    if world == 1 and not args.no_general and pipe.data_rank:
        line["knit_general"] = knit_general(dict(virt=virt, device=local, factored=not args.direct,
                                                 light_cone=not args.no_light_cone), max(2, args.steps // 4))
    if world == 1 and not args.no_north_star:
        line["north_star_sweep"] = north_star_sweep(args.steps)
    if world == 1 and not args.no_sweep_full:
        line["sweep_full"] = sweep_full(max(3, args.steps // 4))
    if world == 1 and not args.no_cpu_baseline:
        if qs_host is not None:
            line["cpu_baseline"] = cpu_baseline_same(pipe, cut, qs_host)
            line["cpu_baseline"]["naive"] = cpu_baseline(cut, args.cpu_sample_labels)
        else:
            line["cpu_baseline"] = cpu_baseline(cut, args.cpu_sample_labels)
        line["cpu_baseline"]["qvm_literal"] = cpu_baseline_qvm(cut)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
