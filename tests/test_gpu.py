"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden fixtures.

Tolerances: fp64, max|delta| <= 1e-12 per entry against the oracle; the
reference-knit fixtures (ACCURACY=0) the same; full-size properties at 1e-12.
"""
import ctypes
import glob
import json
import math
import os

import numpy as np
import pytest

import circuits
from oracle import dense, qvm

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import run_virtual_circuit, run_virtual_circuit_dense

pytestmark = pytest.mark.gpu
TOL = 1e-12
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def T(require_gpu):
    import torch

    return torch


def test_gemm_keyed_matches_numpy(T):
    ctx = engine.get_context(0)
    rng = np.random.default_rng(0)
    for (K, M, N) in [(1, 1, 1), (3, 5, 7), (16, 128, 128), (37, 200, 130), (1296, 256, 64), (6, 16, 1)]:
        A = rng.standard_normal((K, M))
        B = rng.standard_normal((K, N))
        ref = A.T @ B
        out = T.zeros(M * N, dtype=T.float64, device="cuda")
        engine.gemm_keyed(ctx, T.from_numpy(A).cuda(), T.from_numpy(B).cuda(), out=out, strideA=N)
        np.testing.assert_allclose(out.cpu().numpy().reshape(M, N), ref, atol=1e-12 * max(1, K), rtol=0)
        # keyed scatter: transpose via keys + accumulate
        kA = T.arange(M, dtype=T.int64, device="cuda")
        kB = T.arange(N, dtype=T.int64, device="cuda") * M
        out2 = T.ones(M * N, dtype=T.float64, device="cuda")
        engine.gemm_keyed(ctx, T.from_numpy(A).cuda(), T.from_numpy(B).cuda(), keyA=kA, keyB=kB, out=out2, beta=1)
        np.testing.assert_allclose(out2.cpu().numpy().reshape(N, M), ref.T + 1, atol=1e-12 * max(1, K), rtol=0)


@pytest.mark.parametrize("K,M,N,keyed", [
    (16, 128, 128, False), (16, 4096, 4096, False), (32, 4096, 4096, True), (272, 4096, 2048, False),
    (48, 8192, 1024, True), (256, 1024, 8192, False), (8, 4096, 4096, True),  # K % 16: register kernel
    (64, 128, 256, False), (64, 8192, 8192, False), (64, 2048, 4096, True), (32, 1024, 2048, False),
    (64, 4096, 2048, "odd"), (64, 8192, 4096, "rowkeys"),
])
def test_gemm_keyed_full_tile_pipeline_matches_torch(T, K, M, N, keyed):
    """Full-tile shapes take the LDS-DMA kernels: K in {16, 32, 64} the wave-private ring
    (qk_gemm_wave_kernel), other multiples of 16 the shared ring (qk_gemm_glds_kernel). One or
    several tiles per workgroup, rings that wrap across tile ends, the paired-store epilogue, the
    per-element epilogue (transposing keys; odd output offsets that break 16-B pairs) and keyed
    rows with paired columns, against torch's fp64 GEMM."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K + M + N)
    A = T.randn(K, M, dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, N, dtype=T.float64, device="cuda", generator=g)
    ref = A.T @ B
    out = T.full((M * N + 2,), float("nan"), dtype=T.float64, device="cuda")
    if keyed == "odd":  # out[1 + i * N + j]: every pair start odd -> per-element stores
        engine.gemm_keyed(ctx, A, B, keyA=T.arange(M, dtype=T.int64, device="cuda") * N + 1,
                          keyB=T.arange(N, dtype=T.int64, device="cuda"), out=out)
        got = out[1:1 + M * N].view(M, N)
    elif keyed == "rowkeys":  # rows reversed through keys, columns paired
        rows = T.arange(M, dtype=T.int64, device="cuda").flip(0) * N
        engine.gemm_keyed(ctx, A, B, keyA=rows, keyB=T.arange(N, dtype=T.int64, device="cuda"), out=out)
        got = out[:M * N].view(M, N).flip(0)
    elif keyed:  # out[j * M + i]: column keys step by M, so no paired stores
        engine.gemm_keyed(ctx, A, B, keyA=T.arange(M, dtype=T.int64, device="cuda"),
                          keyB=T.arange(N, dtype=T.int64, device="cuda") * M, out=out)
        got = out[:M * N].view(N, M).T
    else:
        engine.gemm_keyed(ctx, A, B, out=out, strideA=N)
        got = out[:M * N].view(M, N)
    T.cuda.synchronize()
    err = float((got - ref).abs().max())
    assert err <= 1e-12 * K, err


def test_khatri_rao_and_gather(T):
    ctx = engine.get_context(0)
    rng = np.random.default_rng(1)
    A, B = rng.standard_normal((5, 3)), rng.standard_normal((5, 4))
    out = engine.khatri_rao(ctx, T.from_numpy(A).cuda(), T.from_numpy(B).cuda()).cpu().numpy()
    ref = np.stack([np.outer(B[k], A[k]).reshape(-1) for k in range(5)])
    np.testing.assert_array_equal(out, ref)
    src = rng.standard_normal((7, 9))
    idx = np.array([6, 0, 3, 3], dtype=np.int64)
    coef = rng.standard_normal(4)
    g = engine.gather_rows(ctx, T.from_numpy(src).cuda(), T.from_numpy(idx).cuda(), T.from_numpy(coef).cuda())
    np.testing.assert_array_equal(g.cpu().numpy(), coef[:, None] * src[idx])


CASES = {
    "cx": lambda: circuits.two_fragment("cx"),
    "cz": lambda: circuits.two_fragment("cz"),
    "cy": lambda: circuits.two_fragment("cy"),
    "rzz": lambda: circuits.two_fragment("rzz"),
    "rzz_pi": lambda: circuits.two_fragment("rzz", angle=math.pi),
    "rzz_0": lambda: circuits.two_fragment("rzz", angle=0.0),
    "cp": lambda: circuits.two_fragment("cp"),
    "cx_3cuts": lambda: circuits.two_fragment("cx", 3, 3, n_cuts=3),
    "cx_wide": lambda: circuits.two_fragment("cx", 7, 6, n_cuts=2, seed=3),
    "move": lambda: circuits.wire_cut(),
    "move_gate": lambda: circuits.wire_cut(3, 2, extra_gate_cut=True),
    "three": lambda: circuits.three_fragment(),
    "three_wide": lambda: circuits.three_fragment(seed=9, sizes=(5, 4, 3)),
    "partial": lambda: circuits.partial_measure(),
    "bv_5_1_p2": lambda: cutting.config_cut_circuit("bv", 5, 1, 2)[:2],
    "hwe_16_1_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[:2],
    "hwe_16_1_p3": lambda: cutting.config_cut_circuit("hwe", 16, 1, 3)[:2],
    "same_fragment": lambda: circuits.same_fragment_cut(),
    "many_traced": lambda: circuits.many_traced(),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_fragment_sweep_matches_oracle(T, case):
    _, cut = CASES[case]()
    virt = VirtualCircuit(cut)
    view = qvm.CutView(cut)
    ctx = engine.get_context(0)
    for fs in engine.prepare_fragments(virt, 0):
        ref, _ = dense.fragment_q(view, list(fs.fragment))
        if ref is None:
            assert fs.dropped
            continue
        q = engine.sweep_fragment(ctx, fs).cpu().numpy()[fs.row_of_label()]
        np.testing.assert_allclose(q, ref, atol=TOL, rtol=0)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("factored", [False, True])
def test_run_virtual_circuit_dense_matches_oracle(T, case, factored):
    circ, cut = CASES[case]()
    virt = VirtualCircuit(cut)
    out, info = run_virtual_circuit_dense(virt, factored=factored)
    ref = dense.run_dense(cut)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=TOL, rtol=0)
    assert info.run_time > 0 and info.knit_time > 0


@pytest.mark.parametrize("case", sorted(CASES))
def test_run_virtual_circuit_default_plan_matches_oracle(T, case):
    """The default drop-in path (run.py: the cached plan, i.e. the benched KnitPipeline — factored
    light-cone knit, device data rank where it applies) against the oracle; a second call on a fresh
    VirtualCircuit of the same cut finds the same plan by content hash and gives the same result."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod

    circ, cut = CASES[case]()
    virt = VirtualCircuit(cut)
    out, info = run_virtual_circuit_dense(virt)
    ref = dense.run_dense(cut)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=TOL, rtol=0)
    assert info.run_time > 0 and info.knit_time >= 0
    pipe = runmod.cached_plan(virt, 0)
    virt2 = VirtualCircuit(cut)
    assert runmod.circuit_fingerprint(virt2) == runmod.circuit_fingerprint(virt)
    out2, _ = run_virtual_circuit_dense(virt2)
    assert runmod.cached_plan(virt2, 0) is pipe
    assert T.equal(out2, out)


KNIT_FILES = sorted(f for f in glob.glob(os.path.join(GOLD, "knit_*.json")) if "knit_samples_" not in f)


@pytest.mark.parametrize("path", KNIT_FILES, ids=[os.path.basename(p)[5:-5] for p in KNIT_FILES])
def test_gpu_knit_of_reference_inputs_matches_reference_knit(T, path):
    """VirtualCircuit.knit (GPU) on the reference's own inputs == reference knit (ACCURACY=0)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr import QuasiDistr
    import test_golden

    import hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr as pqd

    gold = json.load(open(path))
    _, cut = test_golden._case_circuits(gold["case"])
    virt = VirtualCircuit(cut)
    frags = [f for f in virt.fragment_circuits if len(f)]
    results = {}
    old, pqd.ACCURACY = pqd.ACCURACY, 0.0  # the reference was fed untruncated inputs
    try:
        for fi, f in enumerate(frags):
            if str(fi) in gold["inputs"]:
                results[f] = [QuasiDistr(dict((int(k), v) for k, v in x)) for x in gold["inputs"][str(fi)]]
    finally:
        pqd.ACCURACY = old
    dense_out = engine.knit_quasi_distrs(virt, results).cpu().numpy()
    ref = np.zeros_like(dense_out)
    for k, v in gold["knit_acc_0"]:
        ref[int(k)] = v
    np.testing.assert_allclose(dense_out, ref, atol=TOL, rtol=0)
    # reference-shaped result: same keys above the truncation threshold
    qd = virt.knit(results)
    big = {int(k) for k, v in gold["knit_acc_0"] if abs(v) > 1e-5 + 1e-9}
    assert big <= set(qd)


def test_run_virtual_circuit_dict_api(T):
    _, cut = cutting.config_cut_circuit("hwe", 16, 1, 2)[:2]
    virt = VirtualCircuit(cut)
    res, info = run_virtual_circuit(virt, shots=1000)
    gold = json.load(open(os.path.join(GOLD, "knit_hwe_16_1_p2.json")))
    ref = {int(k): v for k, v in gold["npd_acc_1e-05"]}
    assert set(res) == set(ref)
    for k in ref:
        assert abs(res[k] - ref[k]) <= 1e-9
    assert info.run_time > 0


@pytest.mark.parametrize("seed,n", [(0, 1), (1, 37), (2, 1000), (3, 1 << 16)])
def test_gpu_npd_matches_oracle(T, seed, n):
    """GPU truncation + nearest_probability_distribution == quasi_distr.py:7-10,28-43 (oracle)."""
    from oracle.quasi import QD

    rng = np.random.default_rng(seed)
    v = rng.standard_normal(n) * np.where(rng.random(n) < 0.3, 1e-6, 1e-2)
    v[rng.random(n) < 0.2] *= -1.0
    ctx = engine.get_context(0)
    keys, vals = engine.nearest_probability_distribution(ctx, T.from_numpy(v).cuda(), 1e-5)
    ref = QD({i: float(x) for i, x in enumerate(v)}, 1e-5).npd()
    assert list(keys) == list(ref.keys())  # same entries, same (ascending-value) order
    np.testing.assert_allclose(vals, list(ref.values()), rtol=0, atol=1e-15)


def test_gpu_hellinger_and_compare_original_with_cut(T):
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import fidelity

    rng = np.random.default_rng(5)
    p, q = rng.random(4096), rng.random(4096)
    f = fidelity.hellinger_fidelity_dense(T.from_numpy(p).cuda(), T.from_numpy(q).cuda())
    ref = (np.sum(np.sqrt(p * q)) / np.sqrt(p.sum() * q.sum())) ** 2
    assert abs(f - ref) <= 1e-13
    for case in ("cx_3cuts", "three_wide", "move_gate"):
        circ, cut = CASES[case]()
        cmp = fidelity.compare_original_with_cut(circ, cut)
        assert abs(cmp.cut_vs_uncut_fidelity - 1.0) <= 1e-12
        np.testing.assert_allclose(cmp.uncut.cpu().numpy(), dense.uncut_distribution(circ), atol=TOL, rtol=0)


@pytest.mark.parametrize("case", ["cx_3cuts", "move_gate", "three_wide"])
def test_foreign_cut_circuit_runs(T, case):
    """A qiskit-shaped cut circuit goes through run_virtual_circuit unchanged (cut-spec ingestion)."""
    from foreign import to_foreign

    _, cut = CASES[case]()
    out, _ = run_virtual_circuit_dense(VirtualCircuit(to_foreign(cut)))
    np.testing.assert_allclose(out.cpu().numpy(), dense.run_dense(cut), atol=TOL, rtol=0)


def test_split_mode_fragment_matches_oracle(T):
    """16-qubit fragments (SPLIT mode, multi-pass) of syc 32 5: all 1296 labels swept, 6 checked."""
    _, cut = cutting.config_cut_circuit("syc", 32, 5, 2)[:2]
    virt = VirtualCircuit(cut)
    view = qvm.CutView(cut)
    ctx = engine.get_context(0)
    from oracle.statevector import simulate

    for fs in engine.prepare_fragments(virt, 0):
        assert not fs.dprog.enc.packed and len(fs.dprog.enc.passes) >= 2
        q = engine.sweep_fragment(ctx, fs).cpu().numpy()[fs.row_of_label()]
        for li in (0, 7, 215, 431, 1000, 1295):
            d = simulate(view.instance_ops(list(fs.fragment), fs.labels[li]), len(fs.fragment))
            ref = dense.fold(d, view.num_clbits, fs.prog.clbits)
            np.testing.assert_allclose(q[li], ref, atol=TOL, rtol=0)


def test_syc_32_5_basis_rows_match_oracle(T):
    """Every swept row of the bench plan's syc 32 5 sweep (basis-reduced, light cone: 64 + 256
    instances of two 16-qubit fragments, per-program kernels) against the oracle statevector
    (golden/basis_rows_syc_32_5_p2.json, tests/golden/make_rows.py): per row 24 seeded entries
    (1e-12), the sum, the squared norm and four seeded Rademacher projections of all 2^16 entries
    (1e-11: each sums 2^16 terms)."""
    from golden import make_rows

    gold = json.load(open(os.path.join(GOLD, "basis_rows_syc_32_5_p2.json")))
    _, cut = cutting.config_cut_circuit("syc", 32, 5, 2)[:2]
    frags = engine.prepare_fragments(VirtualCircuit(cut), 0, basis=True)
    ctx = engine.get_context(0)
    assert len(frags) == len(gold["fragments"])
    for fs, g in zip(frags, gold["fragments"]):
        assert [list(lab) for lab in fs.basis_labels] == g["basis_labels"]
        assert fs.dprog.module is not None  # the compiled per-program kernels the bench runs
        q = engine.sweep_fragment(ctx, fs).cpu().numpy()
        assert q.shape == (len(g["rows"]), 1 << fs.prog.m)
        pos, proj = make_rows.probes(q.shape[1])
        assert list(pos) == g["positions"]
        for row, ref in zip(q, g["rows"]):
            np.testing.assert_allclose(row[pos], ref["samples"], atol=1e-12, rtol=0)
            assert abs(row.sum() - ref["sum"]) <= 1e-11
            assert abs(row @ row - ref["sumsq"]) <= 1e-12
            np.testing.assert_allclose(proj @ row, ref["proj"], atol=1e-11, rtol=0)


def test_compiled_sweep_matches_interpreter(T):
    """Per-program kernels (sweep_codegen + hiprtc, qk_sweep_compiled) == the interpreter kernel
    (qk_sweep) on every branch job of both syc 32 5 fragments (basis-reduced: 625 jobs each)."""
    import dataclasses

    _, cut = cutting.config_cut_circuit("syc", 32, 5, 2)[:2]
    virt = VirtualCircuit(cut)
    ctx = engine.get_context(0)
    for fs in engine.prepare_fragments(virt, 0, basis=True, relevance=False):
        assert fs.dprog.module is not None, "SPLIT programs run as compiled kernels"
        slot_t, sign_t, _ = engine.jobs_to_device(fs.jobs, 0)
        jit, _ = engine.sweep_jobs(ctx, fs.dprog, slot_t, sign_t, fs.jobs.n_jobs)
        assert fs.dprog.enc.tile_bits == 13
        interp_prog = engine.DeviceProgram.upload(fs.prog, 0, jit=False)  # 12-bit tiles
        interp, _ = engine.sweep_jobs(ctx, interp_prog, slot_t, sign_t, fs.jobs.n_jobs)
        T.cuda.synchronize()
        assert float((jit - interp).abs().max()) <= 1e-13
        # fused FINAL pass (qk_sweep_compiled_labels) == per-job rows + qk_reduce_labels; not bit
        # for bit since the per-program kernels scale by program_scale^2 (the fused sum may contract
        # the scaled sign into an fma): one rounding per term
        off_t = T.from_numpy(fs.jobs.label_offsets.copy()).cuda()
        n_rows = len(fs.jobs.label_offsets) - 1
        fused, _ = engine.sweep_labels(ctx, fs.dprog, slot_t, sign_t, fs.jobs.n_jobs, off_t, n_rows)
        ref = engine.reduce_labels(ctx, jit, off_t, n_rows)
        assert T.allclose(fused, ref, rtol=1e-14, atol=1e-18)


def _uncut_dense_gpu(circ):
    """Exact uncut distribution on the GPU: the whole circuit as one 0-cut fragment."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.circuit import QuantumCircuit, QuantumRegister
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.cutting import CutSpec, cut_circuit

    one = cut_circuit(circ, CutSpec([list(range(circ.num_qubits))]))
    out, _ = run_virtual_circuit_dense(VirtualCircuit(one))
    return out


def _chunked_max_abs_diff(a, b, chunk=1 << 28):
    m = 0.0
    for i in range(0, a.numel(), chunk):
        m = max(m, float((a[i:i + chunk] - b[i:i + chunk]).abs().max()))
    return m


@pytest.mark.slow
@pytest.mark.parametrize("depth,variant,factored", [(1, "forced", False), (1, "ref", None), (5, "ref", True),
                                                    (5, "ref", None)])
def test_syc_32_full_knit_equals_uncut(T, depth, variant, factored):
    """Full size (2^32 outputs): knit of the cut syc 32 circuit == uncut 32-qubit sweep.

    Size-independent known answer for the headline workload (syc 32 5: 4 VirtualCX,
    2592 reference instances): the knitted distribution sums to 1 and equals the
    exact distribution of the uncut circuit, computed as ONE 32-qubit fragment.
    """
    circ, cut = cutting.config_cut_circuit("syc", 32, depth, 2, variant)[:2]
    knit, _ = run_virtual_circuit_dense(VirtualCircuit(cut), factored=factored)
    total = float(knit.sum())
    assert abs(total - 1.0) <= 1e-10
    assert float(knit.min()) >= -1e-13
    T.cuda.empty_cache()
    unc = _uncut_dense_gpu(circ)
    err = _chunked_max_abs_diff(knit, unc)
    assert err <= TOL
    del unc, knit
    T.cuda.empty_cache()


@pytest.mark.parametrize("factored,data_rank", [(False, None), (True, None), (True, True)])
def test_gather_mode_through_rccl_single_rank(T, factored, data_rank):
    """The multi-GPU gather path (job-dealt rows, all_to_all of the row side, all_gather of the
    column side, output-row block contraction) on the HIP backend with a real RCCL
    process group of world size 1 (the only size one GPU allows; 2-4 ranks run under gloo in
    test_distributed.py); with data_rank=True the per-step compression of the row block (forced on
    for these small outputs) must give the exact contraction's result."""
    import socket

    import torch.distributed as dist

    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=T.device("cuda", 0))
    try:
        for name in ("cx_3cuts", "three_wide", "move_gate", "hwe_16_1_p3"):
            _, cut = CASES[name]()
            pipe = KnitPipeline(VirtualCircuit(cut), factored=factored, rank=0, world=1, mode="gather",
                                data_rank=data_rank)
            res = pipe.step().cpu().numpy()
            cls = pipe.ops.clbits
            kA = deposit_keys(cls[pipe.order[0]])
            for i in pipe.order[1:-1]:
                kA = (kA[None, :] + deposit_keys(cls[i])[:, None]).reshape(-1)
            kB = deposit_keys(cls[pipe.order[-1]])
            lo, hi = pipe.row_block
            full = np.zeros(1 << pipe.N)
            full[(kA[lo:hi, None] + kB[None, :]).reshape(-1)] = res[: (hi - lo) * kB.size]
            np.testing.assert_allclose(full, dense.run_dense(cut), atol=TOL, rtol=0)
    finally:
        dist.destroy_process_group()


def test_qft_16_1_p3_config_matches_oracle(T):
    """BASELINE config qft 16 1 p=3: the cutter keeps all 16 lines in one fragment (0 cuts, two
    empty fragments); 586 fused ops on one instance (interpreter kernel)."""
    name, n, d, p, var = cutting.BASELINE_CONFIGS["qft_16_1_p3"]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    out, _ = run_virtual_circuit_dense(VirtualCircuit(cut))
    np.testing.assert_allclose(out.cpu().numpy(), dense.run_dense(cut), atol=TOL, rtol=0)


SAMPLE_CASES = ["cx", "rzz", "cx_3cuts", "move", "move_gate", "three", "partial", "bv_5_1_p2", "hwe_16_1_p2"]


@pytest.mark.parametrize("case", SAMPLE_CASES)
def test_sampled_fragments_match_oracle_draw_for_draw(T, case):
    """qk_sweep + qk_sample_cdf/counts + qk_fold_counts == oracle/sampling.py (the same SplitMix64
    stream and inverse-CDF draw over the exact instance distribution, from_counts truncation at
    1e-5, signed fold) for every reference label. The fold sums in another order than numpy, so q
    agrees to rounding (1e-15); one differing draw would move an entry by 1/shots = 3.3e-4."""
    from oracle import sampling

    _, cut = CASES[case]()
    virt = VirtualCircuit(cut)
    view = qvm.CutView(cut)
    ctx = engine.get_context(0)
    shots, seed, acc = 3000, 17, 1e-5
    for i, fs in enumerate(engine.prepare_fragments(virt, 0)):
        q = engine.sample_fragment(ctx, fs, shots, engine.fragment_seed(seed, i), acc).cpu().numpy()
        if fs.dropped:
            continue
        ref = np.stack([r[1] for r in sampling.sampled_fragment(view, list(fs.fragment), i, shots, seed, acc)])
        np.testing.assert_allclose(q, ref, atol=1e-15, rtol=0)


@pytest.mark.parametrize("case", ["cx", "move_gate", "three", "cx_3cuts"])
@pytest.mark.parametrize("factored", [False, True])
def test_sampled_run_matches_oracle_knit(T, case, factored):
    """run_virtual_circuit_dense(sample=True) == dense knit of the oracle's sampled fragments."""
    import hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr as pqd
    from oracle import sampling

    _, cut = CASES[case]()
    out, _ = run_virtual_circuit_dense(VirtualCircuit(cut), shots=4000, sample=True, seed=3, factored=factored)
    view = qvm.CutView(cut)
    qs, cls = {}, {}
    for i, f in enumerate([list(r) for r in view.qregs if len(r)]):
        if qvm.instance_distributions(view, f) is None:  # dropped fragment (run.py:49-58)
            continue
        qs[tuple(f)] = np.stack([q for _, q in sampling.sampled_fragment(view, f, i, 4000, 3, pqd.ACCURACY)])
        cls[tuple(f)] = dense.fragment_clbits(view, f)
    np.testing.assert_allclose(out.cpu().numpy(), dense.dense_knit(view, qs, cls), atol=TOL, rtol=0)


def test_sample_counts_split_over_calls_and_oracle(T):
    """Raw C ABI: counts do not depend on how labels are split over calls (label_base), every
    label draws exactly `shots`, and each label's counts equal the oracle's draws."""
    from oracle import sampling

    ctx = engine.get_context(0)
    rng = np.random.default_rng(0)
    W, shots, seed = 64, 5000, 99
    seg_off = np.array([0, 1, 3, 4], dtype=np.int64)  # instance 1 has two branch rows
    p = rng.random((4, W)) * np.array([[1.0], [1.0], [-1.0], [1.0]])
    label_seg = np.array([0, 1, 2, 1, 0], dtype=np.int64)
    per = np.diff(seg_off)[label_seg]
    row_off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    d = lambda a: T.from_numpy(np.ascontiguousarray(a)).cuda()
    pj, so, ls, ro = d(p), d(seg_off), d(label_seg), d(row_off)
    cdf = T.empty_like(pj)
    ctx.check(ctx.lib.qk_sample_cdf(ctx.handle, 3, so.data_ptr(), W, pj.data_ptr(), cdf.data_ptr()), "cdf")
    full = T.zeros((int(row_off[-1]), W), dtype=T.int32, device="cuda")
    ctx.check(ctx.lib.qk_sample_counts(ctx.handle, 5, 0, ls.data_ptr(), so.data_ptr(), ro.data_ptr(), W,
                                       cdf.data_ptr(), shots, seed, full.data_ptr()), "counts")
    split = T.zeros_like(full)
    ro2 = d(row_off[2:] - row_off[2])
    ctx.check(ctx.lib.qk_sample_counts(ctx.handle, 2, 0, ls.data_ptr(), so.data_ptr(), ro.data_ptr(), W,
                                       cdf.data_ptr(), shots, seed, split.data_ptr()), "counts a")
    ctx.check(ctx.lib.qk_sample_counts(ctx.handle, 3, 2, ls[2:].data_ptr(), so.data_ptr(), ro2.data_ptr(), W,
                                       cdf.data_ptr(), shots, seed, split[int(row_off[2]):].data_ptr()), "counts b")
    full_h, split_h = full.cpu().numpy(), split.cpu().numpy()
    np.testing.assert_array_equal(full_h, split_h)
    for l, s in enumerate(label_seg):
        c = full_h[row_off[l]:row_off[l + 1]].reshape(-1)
        assert c.sum() == shots
        ref = sampling.sample_counts(p[seg_off[s]:seg_off[s + 1]].reshape(-1), seed, l, shots)
        np.testing.assert_array_equal(c, ref)


def test_foreign_backend_fragment_rows_per_label(T):
    """A fragment bound to a non-MI355X backend goes through the reference counts path
    (run.py:36-58) with one q row per reference label, also where labels share an instance."""
    import hardwareawareoptimalquantumcircuitcuttingandknitting_amd.quasi_distr as pqd
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.backend import MI355XBackend

    class Foreign:  # duck-typed BackendV2 (exact probabilities as counts)
        def run(self, circuits, shots=None):
            return MI355XBackend().run(circuits, shots)

    old, pqd.ACCURACY = pqd.ACCURACY, 0.0
    try:
        for case in ("cx", "cx_3cuts", "move_gate"):
            for factored in (False, True):
                _, cut = CASES[case]()
                virt = VirtualCircuit(cut)
                frags = [f for f in virt.fragment_circuits if len(f)]
                virt.set_backend(frags[0], Foreign())
                out, _ = run_virtual_circuit_dense(virt, shots=1000, factored=factored)
                np.testing.assert_allclose(out.cpu().numpy(), dense.run_dense(cut), atol=1e-10, rtol=0)
    finally:
        pqd.ACCURACY = old


def test_chunked_sweep_and_sweep_graph_match_eager(T):
    """Chunked fused sweeps (Infinity-Cache-resident workspace) and the captured sweep graph
    (fragments on forked streams) give the eager pipeline's q_f bit for bit (syc 32 5, and the
    syc 32 1 reference cut on the interpreter kernel)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    for key, factored in (("syc_32_5_p2", True), ("syc_32_1_p2", False)):
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
        ref = [q.clone() for q in KnitPipeline(VirtualCircuit(cut), factored=factored).sweep()]
        if factored:
            got = KnitPipeline(VirtualCircuit(cut), factored=True, chunk_jobs=96).sweep()
            assert all(T.equal(a, b) for a, b in zip(got, ref))
        pipe = KnitPipeline(VirtualCircuit(cut), factored=factored)
        pipe.capture_sweep()
        for _ in range(2):
            got = pipe.replay_sweep()
        T.cuda.synchronize()
        assert all(T.equal(a, b) for a, b in zip(got, ref))
        del pipe
        T.cuda.empty_cache()


@pytest.mark.parametrize("K,M,N,odd_rows", [(1, 512, 4096, False), (3, 300, 1024, False), (8, 256, 2048, False),
                                            (2, 257, 512, True)])
def test_gemm_small_k_path_matches_torch(T, K, M, N, odd_rows):
    """K <= 8 contractions with contiguous columns take qk_gemm_smallk_kernel (the output-write
    bound outer product of syc 32 1's uncut knit), incl. row keys that break 16-B alignment."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K * M + N)
    A = T.randn(K, M, dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, N, dtype=T.float64, device="cuda", generator=g)
    ref = A.T @ B
    stride = N + 1 if odd_rows else N
    out = T.full((M * stride,), float("nan"), dtype=T.float64, device="cuda")
    engine.gemm_keyed(ctx, A, B, out=out, strideA=stride)
    T.cuda.synchronize()
    got = out.view(M, stride)[:, :N]
    assert float((got - ref).abs().max()) <= 1e-12 * K


def test_edge_cases_empty_and_degenerate(T):
    """K = 0 contraction writes zeros; zero labels / zero shots are no-ops; one shot per label
    puts all mass on one outcome; a fragment with one label samples like the oracle."""
    from oracle import sampling

    ctx = engine.get_context(0)
    out = T.full((64 * 64,), 7.0, dtype=T.float64, device="cuda")
    A = T.zeros((0, 64), dtype=T.float64, device="cuda")
    engine.gemm_keyed(ctx, A, T.zeros((0, 64), dtype=T.float64, device="cuda"), out=out, strideA=64)
    T.cuda.synchronize()
    assert float(out.abs().max()) == 0.0
    assert ctx.lib.qk_sample_counts(ctx.handle, 0, 0, None, None, None, 4, None, 10, 0, None) == 0
    assert ctx.lib.qk_sample_counts(ctx.handle, 3, 0, None, None, None, 4, None, 0, 0, None) == 0
    assert ctx.lib.qk_fold_counts(ctx.handle, 2, None, 4, None, None, 0, 0.0, None) != 0  # shots must be > 0
    _, cut = CASES["cx"]()
    virt = VirtualCircuit(cut)
    for i, fs in enumerate(engine.prepare_fragments(virt, 0)):
        q = engine.sample_fragment(ctx, fs, 1, engine.fragment_seed(5, i), 0.0).cpu().numpy()
        assert np.all(np.abs(q).sum(axis=1) == 1.0)  # one draw: a single +-1 entry per label
    _, cut = CASES["partial"]()
    view = qvm.CutView(cut)
    for i, fs in enumerate(engine.prepare_fragments(VirtualCircuit(cut), 0)):
        if fs.dropped:
            continue
        q = engine.sample_fragment(ctx, fs, 777, engine.fragment_seed(2, i), 1e-5).cpu().numpy()
        ref = np.stack([r[1] for r in sampling.sampled_fragment(view, list(fs.fragment), i, 777, 2, 1e-5)])
        np.testing.assert_allclose(q, ref, atol=1e-15, rtol=0)


def test_multi_fragment_sweep_matches_per_fragment(T, monkeypatch):
    """qk_sweep_compiled_multi (every fragment's pass r in one launch) == the per-fragment launch
    sequence, bit for bit: syc 32 5 (fused label rows) and syc 32 1 (per-job rows)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    for key, factored in (("syc_32_5_p2", True), ("syc_32_1_p2", False)):
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
        monkeypatch.setenv("QKNIT_SWEEP_MULTI", "0")
        ref = [q.clone() for q in KnitPipeline(VirtualCircuit(cut), factored=factored, jit=True).sweep()]
        monkeypatch.setenv("QKNIT_SWEEP_MULTI", "1")
        pipe = KnitPipeline(VirtualCircuit(cut), factored=factored, jit=True)
        assert pipe._multi is not None
        got = pipe.sweep()
        T.cuda.synchronize()
        assert all(T.equal(a, b) for a, b in zip(got, ref))


def test_shared_init_prefix_sweep_matches_per_job_init(T, monkeypatch):
    """qk_sweep_compiled_multi_shared (one INIT tile per distinct INIT prefix: 50 instead of 750 on
    syc 32 5) == the per-job INIT sweep, bit for bit."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS["syc_32_5_p2"]
    _, cut, _ = cutting.config_cut_circuit(name, n, d, p, var)
    monkeypatch.setenv("QKNIT_SWEEP_SHARE", "0")
    pipe0 = KnitPipeline(VirtualCircuit(cut), factored=True, jit=True)
    assert pipe0._multi is not None and len(pipe0._multi[1]) == 11
    ref = [q.clone() for q in pipe0.sweep()]
    monkeypatch.setenv("QKNIT_SWEEP_SHARE", "1")
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True, jit=True)
    assert len(pipe._multi[1]) == 14 and pipe.be.shared_init == [25, 25]
    got = pipe.sweep()
    T.cuda.synchronize()
    assert all(T.equal(a, b) for a, b in zip(got, ref))


@pytest.mark.parametrize("K,odd_rows", [(1, False), (2, False), (5, True), (8, False)])
def test_gemm_outer_paired_matches_torch(T, K, odd_rows):
    """qk_gemm_outer_paired: K <= 8 keyed outer product, N side = deposit keys of a fragment
    holding clbit 0 (adjacent column pairs), A side keyed (or affine with an odd stride, which
    breaks 16-B row alignment and takes the scalar path)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys

    ctx = engine.get_context(0)
    bits_b = [0, 1, 2, 5, 6, 9]  # holds clbit 0
    bits_a = [3, 4, 7, 8, 10]
    assert engine.paired_keys(bits_b)
    M, N = 1 << len(bits_a), 1 << len(bits_b)
    g = T.Generator(device="cuda").manual_seed(17 + K)
    A = T.randn(K, M, dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, N, dtype=T.float64, device="cuda", generator=g)
    kb = T.from_numpy(deposit_keys(bits_b)).cuda()
    ref = (A.T @ B)
    if odd_rows:
        stride = (1 << 11) + 1
        out = T.full((M * stride + N,), float("nan"), dtype=T.float64, device="cuda")
        engine.gemm_outer_paired(ctx, A, B, kb, strideA=stride, out=out)
        ka = T.arange(M, device="cuda", dtype=T.int64) * stride
    else:
        ka = T.from_numpy(deposit_keys(bits_a)).cuda()
        out = T.full((1 << 11,), float("nan"), dtype=T.float64, device="cuda")
        engine.gemm_outer_paired(ctx, A, B, kb, keyA=ka, out=out)
    T.cuda.synchronize()
    got = out[(ka[:, None] + kb[None, :]).reshape(-1)].view(M, N)
    assert float((got - ref).abs().max()) <= 1e-12 * K


@pytest.mark.parametrize("case", ["cx_6x6_3cuts", "cx_8x8_2cuts", "syc_16"])
@pytest.mark.parametrize("reject", [False, True])
def test_speculative_write_matches_oracle(T, case, reject):
    """Speculative write (QKNIT_SPEC_WRITE): the write runs at the factored rank while the probe check
    runs on a side stream; a rejected check (rank_tol NaN) or an incompressible knit (syc_16: rank
    above 8) still ends in the exact contraction over every output. Equal to the oracle (1e-12)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = {"cx_6x6_3cuts": lambda: circuits.two_fragment("cx", 6, 6, n_cuts=3)[1],
           "cx_8x8_2cuts": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=2)[1],
           "syc_16": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]}[case]()
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=True)
    pipe.spec_write = True
    if reject:
        pipe.rank_tol = pipe.rank_tol_rel = float("nan")
    ref = dense.run_dense(cut)
    for _ in range(3):
        if pipe.out is not None:
            pipe.out.fill_(float("nan"))
        got = pipe.step().cpu().numpy()
        np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0)
    pipe.sync_stats()
    assert pipe.dev_rank
    if pipe.last_prep == "fused":
        assert pipe._spec_stream is not None  # the check ran beside the write
        if reject:
            assert pipe.rank_fallbacks + pipe.rank_incompressible == 3 and pipe.last_rank is None
        elif case == "syc_16":
            assert pipe.rank_incompressible == 3
        else:
            assert pipe.rank_fallbacks == 0 and pipe.last_rank is not None


@pytest.mark.parametrize("prep_cus", ["96", "0"])
def test_pipelined_double_buffered_steps_match_oracle(T, prep_cus):
    """Pipelined steps with two output buffers and two write streams (QKNIT_OUT_BUFFERS=2): the steps
    alternate buffers, step i+1's write may run beside step i's; every step's returned buffer equals
    the oracle (1e-12), the two buffers are distinct, and a buffer is reused two steps later."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = circuits.two_fragment("cx", 8, 8, n_cuts=2)[1]
    ref = dense.run_dense(cut)
    saved = os.environ.get("QKNIT_PREP_CUS")
    os.environ["QKNIT_PREP_CUS"] = prep_cus
    try:
        with T.cuda.stream(T.cuda.Stream()):
            pipe = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=True)
            assert pipe.overlap_ok()
            pipe.overlap, pipe.out_buffers = True, 2
            outs = []
            for _ in range(5):
                out = pipe.step()
                outs.append(out)
                T.cuda.current_stream().synchronize()
                np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-12, rtol=0)
            assert outs[1].data_ptr() != outs[2].data_ptr() and outs[1].data_ptr() == outs[3].data_ptr()
    finally:
        if saved is None:
            os.environ.pop("QKNIT_PREP_CUS", None)
        else:
            os.environ["QKNIT_PREP_CUS"] = saved


@pytest.mark.parametrize("buffers", [1, 2])
def test_pipelined_steps_order_writes_after_caller_reads(T, buffers):
    """Pipelined steps against a consumer on the caller's stream with no host sync between steps
    (ADVICE r4): after every step the caller queues a slow read of the result (a spin, a clone) and
    then poisons the buffer with NaN. The write that reuses that buffer (the next step with one
    buffer, the one after with two) must wait for the poison, so every clone equals the oracle; a
    write running ahead of the caller's queue would be overwritten by the NaN its later clone sees."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = circuits.two_fragment("cx", 8, 8, n_cuts=2)[1]
    ref = dense.run_dense(cut)
    with T.cuda.stream(T.cuda.Stream()):
        pipe = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=True)
        assert pipe.overlap_ok()
        pipe.overlap, pipe.out_buffers = True, buffers
        clones = []
        for _ in range(8):
            out = pipe.step()
            T.cuda._sleep(2_000_000)  # the consumer is slow: ~1 ms of spinning on the caller's stream
            clones.append(out.clone())
            out.fill_(float("nan"))
        T.cuda.current_stream().synchronize()
    for c in clones:
        np.testing.assert_allclose(c.cpu().numpy(), ref, atol=1e-12, rtol=0)


@pytest.mark.parametrize("buffers", [2, 3])
def test_prepare_pipelined_makes_every_buffer_before_the_steps(T, monkeypatch, buffers):
    """bench.py's call after its warmup steps: with one step done, prepare_pipelined makes the rotating
    output buffers (mapped and write-rate selected: forced here on small outputs) and their streams, so
    the pipelined steps after it map nothing (qk_out_stats' reservation count unchanged), and every one of
    them equals the oracle; before any step it does nothing."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_SELECT_MIN_BYTES", 0)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=2)[1]
    ref = dense.run_dense(cut)
    with T.cuda.stream(T.cuda.Stream()):
        pipe = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=True)
        assert pipe.overlap_ok()
        pipe.overlap, pipe.out_buffers = True, buffers
        pipe.prepare_pipelined()
        assert pipe.out is None and pipe._outs is None
        outs = [pipe.step().clone()]
        pipe.prepare_pipelined()
        assert len(pipe._outs) == buffers and len({o.data_ptr() for o in pipe._outs}) == buffers
        reserved = engine.out_stats()["reserved"]
        for _ in range(2 * buffers):
            outs.append(pipe.step().clone())
        T.cuda.current_stream().synchronize()
        assert engine.out_stats()["reserved"] == reserved
    for o in outs:
        np.testing.assert_allclose(o.cpu().numpy(), ref, atol=1e-12, rtol=0)


@pytest.mark.slow
def test_syc_32_5_data_rank_step_matches_exact_step(T):
    """The bench step (factored knit, light-cone basis, data-rank compression: the rank-64
    contraction becomes a rank <= 8 keyed outer product) equals the exact rank-64 MFMA
    contraction entry for entry (1e-12) over all 2^32 outputs, with no probe fallback."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref")[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    assert pipe.data_rank
    got = pipe.step()
    pipe.sync_stats()
    assert pipe.dev_rank and pipe.last_kernel == "qk_knit_outer_blocked_kernel"
    assert pipe.rank_fallbacks == 0 and pipe.rank_incompressible == 0
    assert pipe.last_rank is not None and pipe.last_rank <= 8
    assert pipe.out_alloc.startswith("qk_out_alloc")  # 34 GB output mapped from 1-GiB chunks
    exact = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=False)
    ref = exact.step()
    T.cuda.synchronize()
    assert _chunked_max_abs_diff(got, ref) <= 1e-12
    assert abs(float(got.sum()) - 1.0) <= 1e-10
    del pipe, exact, got, ref
    T.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("seed", [None, 7, 42, 2024])
def test_syc_32_5_pruned_rows_step_matches_unpruned_step(T, monkeypatch, seed):
    """Row pruning (pipeline.ROW_PRUNE / PRUNE_TOL: swept rows whose compressed transform columns are
    zero to rounding are not swept, once the plan's bound on every output's change is <= 1e-13;
    the reference seed 1234 prunes 192 column-side rows: 250 of 750 branch jobs run) against the step
    that sweeps every row (ROW_PRUNE = 0), both through the data-rank write, on the generator seeds
    of profiles/r02c_configs_seeds.json too: every one of the 2^32 outputs within the bound."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import pipeline
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref", seed=seed)[1]
    pruned = KnitPipeline(VirtualCircuit(cut), factored=True)
    if seed is None:
        assert sum(sw["n_jobs"] for sw in pruned.sweeps) == 250
    assert pruned.prune_bound is None or pruned.prune_bound <= pipeline.PRUNE_TOL
    got = pruned.step()
    monkeypatch.setattr(pipeline, "ROW_PRUNE", 0.0)
    full = KnitPipeline(VirtualCircuit(cut), factored=True)
    assert full.prune_bound is None
    ref = full.step()
    pruned.sync_stats()
    full.sync_stats()
    assert pruned.rank_fallbacks == 0 and full.rank_fallbacks == 0
    T.cuda.synchronize()
    bound = pruned.prune_bound or 0.0
    # the bound covers the exact knit; both steps also carry the data-rank compression (<= 1e-13 each)
    assert _chunked_max_abs_diff(got, ref) <= bound + 2e-13
    print(f"seed {seed}: jobs {sum(sw['n_jobs'] for sw in pruned.sweeps)} of "
          f"{sum(sw['n_jobs'] for sw in full.sweeps)}, bound {bound:.3g}")
    del pruned, full, got, ref
    T.cuda.empty_cache()


@pytest.mark.parametrize("case", ["hwe_p2", "cx_8x8"])
def test_mapped_output_buffer_steps_match_oracle(T, case, monkeypatch):
    """Outputs in a qk_out_alloc mapping (OUT_MAPPED_MIN_BYTES=0: small outputs mapped too, one
    chunk at its power-of-two alignment): two steps write the oracle's distribution (1e-12) into it,
    the drop-in's second call reuses the mapping once the first result is dropped, and the mapping is
    released when its last tensor goes."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import _lib
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    cut = {"hwe_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[1],
           "cx_8x8": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]}[case]()
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    ref = dense.run_dense(cut)
    for _ in range(2):
        got = pipe.step().cpu().numpy()
        np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0)
    assert pipe.out_alloc.startswith("qk_out_alloc")
    ptr = pipe.out.data_ptr()
    size = ctypes.c_int64()
    assert _lib.lib().qk_out_mapped_bytes(ctypes.c_void_p(ptr), ctypes.byref(size)) == 0
    assert size.value >= 8 * pipe.out.numel()
    first = pipe.take_out()
    p0 = first.data_ptr()
    pipe.run_into(first)
    got = first.cpu().numpy()
    bad = np.flatnonzero(np.abs(got - ref) > 1e-12)
    pipe.sync_stats()
    assert bad.size == 0, (f"{bad.size} wrong entries [{bad[0]}, {bad[-1]}], kernel {pipe.last_kernel}, "
                           f"rank {pipe.last_rank}, out {first.data_ptr():#x}")
    second = pipe.take_out()  # the first result is still held: a new mapping
    assert second.data_ptr() != p0
    del first  # its mapping goes with it (no owner left)
    third = pipe.take_out()  # the second result is still held: another new mapping
    assert third.data_ptr() != second.data_ptr()
    owner = pipe._call_owner
    assert owner.ptr == third.data_ptr()
    del second, third
    assert not owner.in_use()
    assert pipe.take_out().data_ptr() == owner.ptr  # nothing holds it: handed out again


def test_output_falls_back_to_an_ordinary_allocation(T, monkeypatch):
    """A failed qk_out_alloc (address space of retired ranges full, no physical chunk): engine.out_buffer
    hands out an ordinary torch allocation, records it, and the knit into it equals the oracle."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import _lib
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)

    class Failing(engine.MappedOut):
        def __init__(self, ctx, n):
            raise _lib.QknitError("qk_out_alloc failed (test)")

    monkeypatch.setattr(engine, "MappedOut", Failing)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    got = pipe.step().cpu().numpy()
    np.testing.assert_allclose(got, dense.run_dense(cut), atol=1e-12, rtol=0)
    assert pipe.out_alloc.startswith("torch (torch allocation")


def test_drop_in_first_call_defers_the_output_selection(T, monkeypatch):
    """The drop-in's first call maps its output without the write-rate check (no candidate mappings,
    no probe launches) and times its own write instead; a write below OUT_FAST_GBS (forced: inf) makes
    the next call take a write-rate-selected mapping; every call equals the oracle; qk_out_stats counts
    the reservations (one for the first call, OUT_TRIES for the replacement)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.run import cached_plan, clear_plan_cache

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_SELECT_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_FAST_GBS", float("inf"))
    monkeypatch.setattr(engine, "OUT_TRIES", 3)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
    ref = dense.run_dense(cut)
    clear_plan_cache()
    n_sel = len(engine.out_selections)
    st0 = engine.out_stats()
    out, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=TOL, rtol=0)
    pipe = cached_plan(VirtualCircuit(cut), 0)
    own = pipe._call_owner
    assert own is not None and own.write_gbs is not None and own.write_gbs > 0
    assert engine.out_stats()["reserved"] - st0["reserved"] == 1  # no candidates, no probes
    assert "replaced on the next call" in engine.out_selections[-1][0] and len(engine.out_selections) == n_sel + 1
    first_ptr = own.ptr
    del out, own
    out, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)  # first result dropped: replaced, selected
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=TOL, rtol=0)
    assert pipe._call_owner.ptr != first_ptr and getattr(pipe._call_owner, "write_gbs", None) is None
    assert len(engine.out_selections[-1]) == 3  # the three candidates' rates
    assert engine.out_stats()["reserved"] - st0["reserved"] == 4
    del out
    out, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)  # the selected mapping is kept
    assert out.data_ptr() == pipe._call_owner.ptr
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=TOL, rtol=0)
    del out
    clear_plan_cache()


def test_output_selection_keeps_fastest_and_frees_the_others(T, monkeypatch):
    """engine.out_buffer's write-rate selection (forced here on a 512-KiB output: every candidate
    tried): OUT_TRIES mappings are made and timed, the fastest is kept (its rate first in
    out_selections), the others are unmapped, and the knit into the kept one equals the oracle."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import _lib
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_SELECT_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_FAST_GBS", float("inf"))
    monkeypatch.setattr(engine, "OUT_TRIES", 3)
    made = []
    real = engine.MappedOut

    class Spy(real):
        def __init__(self, ctx, n):
            super().__init__(ctx, n)
            made.append(self.ptr)

    monkeypatch.setattr(engine, "MappedOut", Spy)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    got = pipe.step().cpu().numpy()
    np.testing.assert_allclose(got, dense.run_dense(cut), atol=1e-12, rtol=0)
    sel = engine.out_selections[-1]
    assert len(sel) == 3 and sel[0] == max(sel) and all(r > 0 for r in sel)
    assert "write-rate selected" in pipe.out_alloc and len(made) == 3
    kept = pipe.out.data_ptr()
    size = ctypes.c_int64()
    for ptr in made:
        rc = _lib.lib().qk_out_mapped_bytes(ctypes.c_void_p(ptr), ctypes.byref(size))
        assert (rc == 0) == (ptr == kept)


def test_output_selection_stops_after_a_slow_mapping(T, monkeypatch):
    """A candidate mapping slower than OUT_MAP_SLOW_MS ends the selection after its rate check (memory
    the driver is still clearing after another process: tools/map_stall_probe.py); forced here with a
    negative limit, so of OUT_TRIES = 3 only the first output and one candidate are made, the faster is
    kept, and the knit into it equals the oracle."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_SELECT_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_FAST_GBS", float("inf"))
    monkeypatch.setattr(engine, "OUT_TRIES", 3)
    monkeypatch.setattr(engine, "OUT_MAP_SLOW_MS", -1.0)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    got = pipe.step().cpu().numpy()
    np.testing.assert_allclose(got, dense.run_dense(cut), atol=1e-12, rtol=0)
    sel = engine.out_selections[-1]
    assert len(sel) == 2 and sel[0] == max(sel)
    log = engine.out_selection_log[-1]
    assert len(log["map_ms"]) == 1 and log["stopped"].startswith("mapping took")


def test_mapped_outputs_freed_and_remapped_read_back_exactly(T, monkeypatch):
    """Drop-in calls that keep some results and drop others: mappings are freed and new ones made
    between calls. Each result equals the oracle (1e-12) read back by the D2H copy. Freed ranges'
    addresses used to be reserved again for later mappings, and 32-KiB runs of those read back as
    zeros in 44 of 60 calls (qknit_mem.hip: retired ranges; tools/diag/mapped_loop.py)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    ref = dense.run_dense(cut)
    held, wrong = [], []
    for it in range(30):
        out = pipe.take_out()
        pipe.run_into(out)
        bad = int(np.count_nonzero(np.abs(out.cpu().numpy() - ref) > 1e-12))
        if bad:
            wrong.append((it, bad))
        if it % 3 == 0:
            held.append(out)  # kept: the next call maps a new buffer
        if len(held) > 2:
            held.pop(0)  # dropped: its mapping is freed
        del out
    assert not wrong, f"calls with wrong entries (call, count): {wrong}"


@pytest.mark.slow
def test_syc_32_5_drop_in_equals_exact_step(T):
    """run_virtual_circuit(virt, dense=True) on the headline workload runs the cached plan of the
    benched engine (device data rank, blocked write) and equals the exact K = 64 MFMA contraction
    within 1e-12 over all 2^32 outputs; the second call reuses the plan and writes the same values."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref")[1]
    runmod.clear_plan_cache()
    got, info = run_virtual_circuit(VirtualCircuit(cut), dense=True)
    pipe = runmod.cached_plan(VirtualCircuit(cut), 0)
    assert pipe.dev_rank and pipe.last_kernel == "qk_knit_outer_blocked_kernel"
    assert pipe.rank_fallbacks == 0 and pipe.last_rank is not None and pipe.last_rank <= 8
    assert not pipe._pending and pipe.out is None  # read back per call; the result is the caller's
    exact = KnitPipeline(VirtualCircuit(cut), factored=True, data_rank=False)
    ref = exact.step()
    T.cuda.synchronize()
    assert _chunked_max_abs_diff(got, ref) <= 1e-12
    del exact
    again, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)
    assert _chunked_max_abs_diff(again, got) == 0.0
    del got, again, ref
    runmod.clear_plan_cache()
    T.cuda.empty_cache()


SAMPLE_FILES = sorted(glob.glob(os.path.join(GOLD, "knit_samples_*.json")))


@pytest.mark.slow
@pytest.mark.parametrize("path", SAMPLE_FILES, ids=[os.path.basename(p)[13:-5] for p in SAMPLE_FILES])
def test_full_size_knit_matches_reference_knit_samples(T, path):
    """The 2^32-output BASELINE configs against the reference's own knit (vc:50-68, qd:55-60): the
    bench step (factored light-cone knit, device data rank, blocked write) and the drop-in
    run_virtual_circuit at the 4096 keys whose fragment outcomes make_golden.py sampled (the
    reference knit of exact instances restricted to those outcomes gives them exactly)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    gold = json.load(open(path))
    name, n, d, p, var = cutting.BASELINE_CONFIGS[gold["case"]]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    keys = T.tensor(gold["keys"], dtype=T.int64, device="cuda")
    ref = np.array(gold["values"])
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    out = pipe.step()
    got = out[keys].cpu().numpy()
    pipe.sync_stats()
    assert pipe.rank_fallbacks == 0
    del out, pipe
    T.cuda.empty_cache()
    err = np.abs(got - ref)
    assert err.max() <= TOL, err.max()
    big = np.abs(ref) > 1e-13
    assert (err[big] / np.abs(ref[big])).max() <= 1e-9  # relative, on the entries well above rounding
    assert np.count_nonzero(ref) >= len(ref) // 2
    runmod.clear_plan_cache()
    dense_out, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)
    got2 = dense_out[keys].cpu().numpy()
    del dense_out
    runmod.clear_plan_cache()
    T.cuda.empty_cache()
    assert np.abs(got2 - ref).max() <= TOL


@pytest.mark.parametrize("variant", ["ref", "forced"])
def test_syc_32_1_fragment_rows_match_oracle(T, variant):
    """Every swept row of both syc 32 1 fragments (the reference cut: one instance each; the forced
    4-cut variant: its swept basis instances, 6 checked per fragment) equals the oracle's exact
    instance distribution (branching statevector, signed fold)."""
    from oracle.statevector import simulate

    _, cut = cutting.config_cut_circuit("syc", 32, 1, 2, variant)[:2]
    virt = VirtualCircuit(cut)
    view = qvm.CutView(cut)
    ctx = engine.get_context(0)
    for fs in engine.prepare_fragments(virt, 0):
        q = engine.sweep_fragment(ctx, fs).cpu().numpy()[fs.row_of_label()]
        picks = sorted({i for i in (0, 1, 100, 555, 777, len(fs.labels) - 1) if i < len(fs.labels)})
        for li in picks:
            d = simulate(view.instance_ops(list(fs.fragment), fs.labels[li]), len(fs.fragment))
            np.testing.assert_allclose(q[li], dense.fold(d, view.num_clbits, fs.prog.clbits), atol=TOL, rtol=0)


@pytest.mark.parametrize("K,nbits,bits_b", [(1, 11, [0, 1, 2, 5, 6, 9]), (2, 11, [0, 3, 4, 5, 10]),
                                            (8, 11, [0, 1, 2, 3, 8, 9, 10]), (2, 3, [0, 2]), (3, 9, [0, 2, 5, 6]),
                                            (2, 17, [0, 1, 2, 3, 8, 9, 10, 11, 16]),
                                            (8, 18, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13])])
def test_knit_outer_stream_matches_torch(T, K, nbits, bits_b):
    """qk_knit_outer_stream: the small-K two-fragment knit written in output order equals A^T B
    scattered through the deposit keys of the two clbit sets. nbits 3: the per-output kernel on a
    single partial chunk (8 outputs, grid of 1); nbits >= 9: the blocked kernel (tasks of 2^TB
    outputs, TB <= 16, the operand stage in LDS); nbits 18 / K 8 / 14 low B bits: the B range of a
    task is too large to stage, the blocked kernel reads B from global memory (syc 32 1's layout)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys

    ctx = engine.get_context(0)
    bits_a = [b for b in range(nbits) if b not in bits_b]
    assert engine.stream_knit_ok(bits_a, bits_b, nbits)
    M, N = 1 << len(bits_a), 1 << len(bits_b)
    g = T.Generator(device="cuda").manual_seed(29 + K)
    A = T.randn(K, M, dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, N, dtype=T.float64, device="cuda", generator=g)
    out = T.full((1 << nbits,), float("nan"), dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, out)
    T.cuda.synchronize()
    ka = T.from_numpy(deposit_keys(bits_a)).cuda()
    kb = T.from_numpy(deposit_keys(bits_b)).cuda()
    got = out[(ka[:, None] + kb[None, :]).reshape(-1)].view(M, N)
    assert not bool(out.isnan().any())
    assert float((got - A.T @ B).abs().max()) <= 1e-12 * K


def test_knit_outer_stream_range_slices_and_device_k(T):
    """qk_knit_outer_stream_range: 4 task-aligned slices written separately concatenate to the
    whole knit bit for bit (multi-GPU slice mode); a device K of 0 writes nothing, a device K of 1
    keeps only the first term (predicated knit)."""
    ctx = engine.get_context(0)
    nbits, K = 18, 3
    bits_b = [0, 1, 2, 3, 8, 9, 10, 11, 16, 17]
    bits_a = [b for b in range(nbits) if b not in bits_b]
    g = T.Generator(device="cuda").manual_seed(5)
    A = T.randn(K, 1 << len(bits_a), dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, 1 << len(bits_b), dtype=T.float64, device="cuda", generator=g)
    full = T.empty(1 << nbits, dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, full)
    parts = []
    step = (1 << nbits) // 4
    for r in range(4):
        part = T.full((step,), float("nan"), dtype=T.float64, device="cuda")
        engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, part, o_begin=r * step, o_count=step)
        parts.append(part)
    T.cuda.synchronize()
    assert T.equal(T.cat(parts), full)
    kd = T.zeros(1, dtype=T.int32, device="cuda")
    sentinel = T.full((1 << nbits,), 7.0, dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, sentinel, k_dev=kd)
    T.cuda.synchronize()
    assert bool((sentinel == 7.0).all())
    kd.fill_(1)
    one = T.empty(1 << nbits, dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, one, k_dev=kd)
    ref = T.empty(1 << nbits, dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A[:1].contiguous(), B[:1].contiguous(), bits_a, bits_b, nbits, ref)
    T.cuda.synchronize()
    assert T.equal(one, ref)


@pytest.mark.parametrize("K,ra,rb,r", [(64, 8, 8, 2), (64, 5, 12, 4), (24, 3, 3, 3), (64, 20, 20, 8), (16, 16, 16, 12)])
def test_rank_factors_device_matches_host(T, K, ra, rb, r):
    """qk_rank_factors (one-workgroup pivoted Cholesky + complete-pivoting LU of the core) reproduces the
    low-rank product like data_rank.rank_factors (host form); rank > 8 reports r = 0 (exact path)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import data_rank

    rng = np.random.default_rng(K + ra + rb + r)
    M, N = 3000, 2000
    core = rng.standard_normal((ra, r)) @ rng.standard_normal((r, rb))
    PA = rng.standard_normal((K, ra))
    PB = np.linalg.pinv(PA.T) @ core
    XA, XB = rng.standard_normal((ra, M)), rng.standard_normal((rb, N))
    A, B = PA @ XA, PB @ XB
    R = A.T @ B
    At, Bt = T.from_numpy(A).cuda(), T.from_numpy(B).cuda()
    GA, GB = (At @ At.T).contiguous(), (Bt @ Bt.T).contiguous()
    TA, TB, rd = engine.rank_factors_device(engine.get_context(0), GA, GB)
    T.cuda.synchronize()
    got_r = int(rd.item())
    host = data_rank.rank_factors(GA.cpu().numpy(), GB.cpu().numpy())
    if r > 8:
        assert got_r == 0 and host is None
        return
    assert got_r == r and host is not None and host[0].shape[0] == r
    assert float(TA[r:].abs().sum()) == 0.0 and float(TB[r:].abs().sum()) == 0.0
    Rd = ((TA @ At).T @ (TB @ Bt)).cpu().numpy()
    Rh = (host[0] @ A).T @ (host[1] @ B)
    scale = np.abs(R).max()
    assert np.abs(Rd - R).max() <= 1e-9 * scale
    assert np.abs(Rh - R).max() <= 1e-9 * scale


@pytest.mark.parametrize("K,RA,RB,NA,NB", [(64, 64, 256, 65536, 65536), (64, 37, 130, 1024, 2048), (6, 4, 9, 128, 256),
                                           (64, 256, 64, 128, 8192)])
def test_prep_operands_matches_torch(T, K, RA, RB, NA, NB):
    """qk_prep_operands (one pass: X = Wt^T q on MFMA, per-workgroup Gram / probe partials, fixed-order
    reduction) against torch fp64: X, the two Grams and U = X_B P^T (relative 1e-13 of the norms).
    Shapes: syc 32 5's two sides, ragged instance-row counts, K < 16, more tiles on one side; an odd K
    (rows staged 16 B at a time) is refused."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K + RA + RB)
    WtA = T.randn(RA, K, dtype=T.float64, device="cuda", generator=g)
    WtB = T.randn(RB, K, dtype=T.float64, device="cuda", generator=g)
    qA = T.randn(RA, NA, dtype=T.float64, device="cuda", generator=g)
    qB = T.randn(RB, NB, dtype=T.float64, device="cuda", generator=g)
    P = T.randn(16, NB, dtype=T.float64, device="cuda", generator=g)
    XA, XB, G, U = engine.prep_operands(ctx, WtA, qA, WtB, qB, P)
    T.cuda.synchronize()
    rXA, rXB = WtA.T @ qA, WtB.T @ qB
    close = lambda a, b: float((a - b).abs().max()) <= 1e-13 * max(float(b.abs().max()), 1.0) * 64  # noqa: E731
    assert close(XA, rXA) and close(XB, rXB)
    assert close(G[0], rXA @ rXA.T) and close(G[1], rXB @ rXB.T)
    assert close(U, rXB @ P.T)
    XA2, XB2, G2, U2 = engine.prep_operands(ctx, WtA, qA, WtB, qB, P)
    T.cuda.synchronize()
    assert T.equal(G, G2) and T.equal(U, U2) and T.equal(XB, XB2)  # deterministic
    # the partials hold the upper 16 x 16 blocks only: the lower ones are their mirror, bit for bit
    assert T.equal(G[0], G[0].T) and T.equal(G[1], G[1].T)
    if NA >= 256:
        # q as a 128-aligned column window of wider rows (row stride > width): the window's X, Gram
        # and (B side) probe products, bit for bit those of the same columns copied out
        h = NA // 2
        qw = qA[:, h:]
        assert not qw.is_contiguous()
        XAw, _, Gw, _ = engine.prep_operands(ctx, WtA, qw, WtB, qB, P)
        XAc, _, Gc, _ = engine.prep_operands(ctx, WtA, qw.contiguous(), WtB, qB, P)
        T.cuda.synchronize()
        assert T.equal(XAw, XAc) and T.equal(Gw, Gc)
    if K == 6:
        assert not engine.prep_ok(5, NA, NB)
        with pytest.raises(engine._lib.QknitError):
            engine.prep_operands(ctx, WtA[:, :5].contiguous(), qA, WtB[:, :5].contiguous(), qB, P)


@pytest.mark.parametrize("K,RA,RB,NA,NB,rmax", [(64, 65, 65, 65536, 65536, 8), (64, 80, 17, 1024, 2048, 8),
                                                (6, 1, 9, 512, 512, 3), (64, 64, 64, 8192, 1536, 1), (32, 33, 48, 512, 4096, 8)])
def test_qprep_matches_torch(T, K, RA, RB, NA, NB, rmax):
    """The q-space preparation (qk_qprep_grams, qk_qprep_compress_check: no X = Wt^T q materialised) against
    torch fp64 on the X path's definitions: the Grams of X, U = X_B P^T, A2 = TA X_A, B2 = TB X_B and the
    probe check's squared errors (via the accepted rank at a tolerance set around them); deterministic.
    Shapes: syc 32 5's two sides (65 swept rows each), the 80-row maximum, one row, K < 16, rmax < 8."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K + RA + RB + NA)
    WtA = T.randn(RA, K, dtype=T.float64, device="cuda", generator=g)
    WtB = T.randn(RB, K, dtype=T.float64, device="cuda", generator=g)
    qA = T.randn(RA, NA, dtype=T.float64, device="cuda", generator=g)
    qB = T.randn(RB, NB, dtype=T.float64, device="cuda", generator=g)
    P = T.randn(16, NB, dtype=T.float64, device="cuda", generator=g)
    G, U = engine.qprep_grams(ctx, WtA, qA, WtB, qB, P)
    T.cuda.synchronize()
    XA, XB = WtA.T @ qA, WtB.T @ qB
    close = lambda a, b: float((a - b).abs().max()) <= 1e-13 * max(float(b.abs().max()), 1.0) * 64  # noqa: E731
    assert close(G[0], XA @ XA.T) and close(G[1], XB @ XB.T)
    assert close(U, XB @ P.T)
    TA = T.randn(rmax, K, dtype=T.float64, device="cuda", generator=g)
    TB = T.randn(rmax, K, dtype=T.float64, device="cuda", generator=g)
    r = T.tensor([rmax], dtype=T.int32, device="cuda")
    A2, B2, k, err = engine.qprep_compress_check(ctx, WtA, qA, WtB, qB, TA, TB, U, P, r, 1e300, 0.0)
    T.cuda.synchronize()
    assert close(A2, TA @ XA) and close(B2, TB @ XB)
    d = XA.T @ (XB @ P.T) - A2.T @ (B2 @ P.T)
    ref_err = float((d * d).sum(dim=0).max().sqrt())
    assert int(k) == rmax and abs(float(err) - ref_err) <= 1e-9 * ref_err
    _, _, k2, _ = engine.qprep_compress_check(ctx, WtA, qA, WtB, qB, TA, TB, U, P, r, 0.5 * ref_err, 0.0)
    assert int(k2) == 0  # the same error against half of it: rejected
    G2, U2 = engine.qprep_grams(ctx, WtA, qA, WtB, qB, P)
    A22, B22, _, err2 = engine.qprep_compress_check(ctx, WtA, qA, WtB, qB, TA, TB, U, P, r, 1e300, 0.0)
    T.cuda.synchronize()
    assert T.equal(G, G2) and T.equal(U, U2) and T.equal(A2, A22) and T.equal(B2, B22) and T.equal(err, err2)


@pytest.mark.parametrize("K,NA,NB,rmax", [(64, 4096, 1001, 8), (24, 129, 8192, 8), (64, 65536, 65536, 8),
                                          (24, 4096, 2048, 3), (17, 2050, 130, 8), (64, 2048, 4096, 1)])
def test_compress_operands_matches_torch(T, K, NA, NB, rmax):
    """qk_compress_operands against torch: odd column counts (rows not 16-B aligned: the K-split
    kernel), even ones (the column kernel, qk_compress_cols_kernel) with K below 64, K not a multiple
    of its 16-row load chunks, and fewer than 8 rows of T, ragged last column blocks."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K + NA + NB + rmax)
    TA, TB = (T.randn(rmax, K, dtype=T.float64, device="cuda", generator=g) for _ in range(2))
    XA = T.randn(K, NA, dtype=T.float64, device="cuda", generator=g)
    XB = T.randn(K, NB, dtype=T.float64, device="cuda", generator=g)
    A2, B2 = engine.compress_operands(ctx, TA, XA, TB, XB)
    T.cuda.synchronize()
    for got, ref in ((A2, TA @ XA), (B2, TB @ XB)):
        assert float((got - ref).abs().max()) <= 1e-13 * float(ref.abs().max())
    if NA % 4 == 0:
        # qk_compress_operands_ld, a replicated rank's form: A2's columns [base, base + n) only, from X_A's
        # same columns — bit for bit the full compression's there (same kernel per column), B2 unchanged
        base, n = NA // 4, NA // 2
        A2c, B2c = engine.compress_operands(ctx, TA, XA, TB, XB, a_cols=(base, n))
        T.cuda.synchronize()
        assert A2c.shape == A2.shape and T.equal(A2c[:, base:base + n], A2[:, base:base + n]) and T.equal(B2c, B2)


@pytest.mark.parametrize("K,NA,NB,rmax,a_cols", [(64, 65536, 65536, 8, None), (64, 65536, 65536, 8, (8192, 8192)),
                                                  (24, 4096, 2052, 3, None), (17, 2048, 132, 8, (512, 1024)),
                                                  (64, 1024, 8192, 1, None), (6, 128, 512, 2, (0, 64))])
def test_compress_probe_v_matches_separate_passes(T, K, NA, NB, rmax, a_cols):
    """qk_compress_probe_v (the compression with the probe check's V pass fused in) against the separate
    passes: A2 / B2 bit for bit those of qk_compress_operands(_ld) (same arithmetic per column), and the
    probe check from its V partials (qk_probe_errors_vpart) equal to qk_probe_errors' within 1e-12 —
    ragged widths (not multiples of the 512-column blocks), K below 64, rmax below 8, a column range
    of A given as a window of X_A and as its own [K, n] block."""
    ctx = engine.get_context(0)
    g = T.Generator(device="cuda").manual_seed(K + NA + NB + rmax)
    TA, TB = (T.randn(rmax, K, dtype=T.float64, device="cuda", generator=g) for _ in range(2))
    XA = T.randn(K, NA, dtype=T.float64, device="cuda", generator=g)
    XB = T.randn(K, NB, dtype=T.float64, device="cuda", generator=g)
    P = T.randn(16, NB, dtype=T.float64, device="cuda", generator=g)
    U = XB @ P.T
    r = T.tensor([rmax], dtype=T.int32, device="cuda")
    A2, B2 = engine.compress_operands(ctx, TA, XA, TB, XB, a_cols=a_cols)
    A2v, B2v, vp = engine.compress_probe_v(ctx, TA, XA, TB, XB, P, a_cols=a_cols)
    base, n = (0, NA) if a_cols is None else a_cols
    T.cuda.synchronize()
    assert T.equal(A2v[:, base:base + n], A2[:, base:base + n]) and T.equal(B2v, B2)
    assert vp.shape == (-(-NB // 512), 8, 16)
    ref = (B2 @ P.T).cpu()
    assert float((vp.sum(dim=0)[:rmax].cpu() - ref).abs().max()) <= 1e-12 * float(ref.abs().max())
    if rmax < 8:  # rows past the rank are zero
        assert float(vp[:, rmax:].abs().max()) == 0.0
    XAc = XA[:, base:base + n]
    e2, k, err = engine.probe_errors(ctx, XAc, A2, U, B2, P, r=r, tol=1e300, a2_cols=None if a_cols is None else a_cols)
    e2v, kv, errv = engine.probe_errors(ctx, XAc, A2v, U, B2v, P, r=r, tol=1e300,
                                        a2_cols=None if a_cols is None else a_cols, vpart=vp)
    T.cuda.synchronize()
    assert int(k) == int(kv) == rmax
    assert float((e2v - e2).abs().max()) <= 1e-12 * float(e2.abs().max())
    if a_cols is not None and n % 2 == 0:  # X_A's columns as their own [K, n] block
        A2w, _, vpw = engine.compress_probe_v(ctx, TA, XAc.contiguous(), TB, XB, P, a_cols=a_cols, a_width=NA)
        T.cuda.synchronize()
        assert T.equal(A2w[:, base:base + n], A2[:, base:base + n]) and T.equal(vpw, vp)


@pytest.mark.parametrize("K,ra,rb,r,noise", [(64, 8, 8, 2, 0.0), (64, 5, 12, 4, 0.0), (64, 20, 20, 8, 0.0),
                                             (64, 8, 8, 2, 1e-9), (24, 3, 3, 3, 0.0)])
def test_probe_check_and_compress(T, K, ra, rb, r, noise):
    """qk_compress_operands (A'' = T_A A, B'' = T_B B) and qk_probe_errors / qk_probe_accept (the
    acceptance check on the real operands without materialising the probe products) against torch:
    the probe errors ||(A^T B - A''^T B'') p_j|| within the fp64 floor of the two products (1e-13 of
    their norm),
    exact low-rank data accepted (k = r), a rank-2 product plus 1e-9 noise rejected (k = 0). Also the
    column-block form of the multi-GPU path: e2 over two halves of A's columns sums to the whole."""
    ctx = engine.get_context(0)
    rng = np.random.default_rng(K + ra + rb + r)
    M, N = 3072, 2048
    core = rng.standard_normal((ra, r)) @ rng.standard_normal((r, rb))
    PA = rng.standard_normal((K, ra))
    PB = np.linalg.pinv(PA.T) @ core
    A = PA @ rng.standard_normal((ra, M))
    B = PB @ rng.standard_normal((rb, N)) + noise * rng.standard_normal((K, N))
    At, Bt = T.from_numpy(A).cuda(), T.from_numpy(B).cuda()
    x = T.from_numpy(np.random.default_rng(1234).standard_normal((16, N))).cuda()
    GA, GB, U = (At @ At.T).contiguous(), (Bt @ Bt.T).contiguous(), (Bt @ x.T).contiguous()
    TA, TB, rd = engine.rank_factors_device(ctx, GA, GB)
    A2, B2 = engine.compress_operands(ctx, TA, At, TB, Bt)
    T.cuda.synchronize()
    got_r = int(rd.item())
    assert got_r == r if noise == 0.0 else 0 < got_r <= 8
    assert float((A2 - TA @ At).abs().max()) <= 1e-12 * float((TA @ At).abs().max())
    assert float((B2 - TB @ Bt).abs().max()) <= 1e-12 * float((TB @ Bt).abs().max())
    ref = ((At.T @ U - A2.T @ (B2 @ x.T)) ** 2).sum(dim=0)
    tol = 1e-12 * float((At.T @ U).norm(dim=0).max())  # exact data: ~1e-15 of it; the noise: ~1e-9
    e2f, k, err = engine.probe_errors(ctx, At, A2, U, B2, x, r=rd, tol=tol)
    h = M // 2
    e2a, _, _ = engine.probe_errors(ctx, At[:, :h].contiguous(), A2, U, B2, x, a2_cols=(0, h))
    e2b, _, _ = engine.probe_errors(ctx, At[:, h:].contiguous(), A2, U, B2, x, a2_cols=(h, h))
    k2, _ = engine.probe_accept(ctx, (e2a + e2b).contiguous(), rd, tol)
    # relative bound: the same decision with the floor at 0 and rel_tol * ||R p|| equal to tol
    refn = float((At.T @ U).norm(dim=0).max())
    k3, _ = engine.probe_accept(ctx, e2f, rd, 0.0, tol / refn)
    T.cuda.synchronize()
    e2, e2a, e2b = e2f[:16], e2a[:16], e2b[:16]
    assert abs(float(e2f[16:].max().sqrt()) - refn) <= 1e-12 * refn  # ||R p||^2 alongside the errors
    assert int(k3.item()) == int(k.item())
    # the error norms are differences of products of norm ~|A^T U|: both sides carry 1e-16-relative
    # rounding of those, so they agree to 1e-13 of |A^T U| (exact data: the norms are that noise)
    floor = 1e-13 * float((At.T @ U).norm(dim=0).max())
    assert float((e2.sqrt() - ref.sqrt()).abs().max()) <= floor
    assert float(((e2a + e2b).sqrt() - e2.sqrt()).abs().max()) <= floor
    assert abs(float(err.item()) - float(e2.max().sqrt())) <= 1e-12 * float(err.item()) + 1e-300
    if noise == 0.0:
        assert int(k.item()) == r and int(k2.item()) == r and float(err.item()) <= tol
    else:
        assert int(k.item()) == 0 and int(k2.item()) == 0 and float(err.item()) > tol


def test_rank_factors_device_degenerate(T):
    """A zero Gram (R = 0) and a non-PSD garbage Gram give r = 0 and zero factors."""
    ctx = engine.get_context(0)
    K = 16
    Z = T.zeros((K, K), dtype=T.float64, device="cuda")
    I = T.eye(K, dtype=T.float64, device="cuda")
    for GA, GB in ((Z, I), (I, Z), (-I, I)):
        TA, TB, rd = engine.rank_factors_device(ctx, GA.contiguous(), GB.contiguous())
        T.cuda.synchronize()
        assert int(rd.item()) == 0
        assert float(TA.abs().max()) == 0.0 and float(TB.abs().max()) == 0.0


@pytest.mark.parametrize("default_path", [False, True])
def test_concurrent_runs_from_two_threads(T, default_path, monkeypatch):
    """The reference calls run_virtual_circuit from several threads at once (Utilities.py:85-89,
    132-136, each with its own Pool(8)). Two threads here run different circuits concurrently (one
    qk context per thread, same device), twice each; every result equals the oracle's knit (1e-12).
    default_path: factored=None — each thread's cached plan (plan cache per thread) and its output
    mapping (qk_out_alloc: OUT_MAPPED_MIN_BYTES=0 maps even these small outputs)."""
    if default_path:
        monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    import threading

    from oracle import dense

    import circuits

    cases = {"hwe_16_1_p2": cutting.config_cut_circuit("hwe", 16, 1, 2)[1],
             "bv_5_1_p2": cutting.config_cut_circuit("bv", 5, 1, 2)[1],
             "cx_3cuts": circuits.two_fragment("cx", 3, 3, n_cuts=3)[1],
             "move_gate": circuits.wire_cut(3, 2, extra_gate_cut=True)[1]}
    refs = {k: dense.run_dense(c) for k, c in cases.items()}
    plan = [["hwe_16_1_p2", "cx_3cuts", "hwe_16_1_p2", "cx_3cuts"], ["bv_5_1_p2", "move_gate", "move_gate", "bv_5_1_p2"]]
    errs, failures = {}, []

    def worker(names):
        try:
            for k in names:
                factored = None if default_path else (k != "bv_5_1_p2")
                out, _ = run_virtual_circuit(VirtualCircuit(cases[k]), dense=True, factored=factored)
                T.cuda.current_stream().synchronize()
                errs.setdefault(k, []).append(float(np.abs(out.cpu().numpy() - refs[k]).max()))
        except Exception as e:  # surfaced below
            failures.append(repr(e))

    threads = [threading.Thread(target=worker, args=(p,)) for p in plan]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not failures, failures
    assert sorted(errs) == sorted(cases) and all(len(v) == 2 for v in errs.values())
    assert max(max(v) for v in errs.values()) <= 1e-12, errs


def test_npd_on_2_28_entries_known_answer(T):
    """qk_threshold_count + qk_npd over 2^28 entries (quasi_distr.py:7-10,28-43, run.py:71): sub-
    threshold noise everywhere plus 2000 planted entries above ACCURACY (a fifth negative); the
    truncation keeps exactly the planted ones and the projection equals the oracle's NPD of them."""
    from oracle.quasi import QD

    n = 1 << 28
    g = T.Generator(device="cuda").manual_seed(11)
    v = (T.rand(n, dtype=T.float64, device="cuda", generator=g) - 0.5) * 1.8e-5  # |v| < 0.9e-5
    rng = np.random.default_rng(12)
    idx = np.unique(rng.integers(0, n, 2000))
    vals = rng.uniform(2e-5, 1e-3, idx.size)
    vals[rng.random(idx.size) < 0.2] *= -1.0
    v[T.from_numpy(idx).cuda()] = T.from_numpy(vals).cuda()
    keys, got = engine.nearest_probability_distribution(engine.get_context(0), v, 1e-5)
    ref = QD({int(i): float(x) for i, x in zip(idx, vals)}, 1e-5).npd()
    assert list(keys) == list(ref.keys())
    np.testing.assert_allclose(got, list(ref.values()), rtol=0, atol=1e-15)
    del v
    T.cuda.empty_cache()


@pytest.mark.parametrize("case,factored", [("hwe_16_1_p2", True), ("hwe_16_1_p2", False), ("cx_3cuts", True),
                                           ("three", False), ("move_gate", True), ("bv_5_1_p2", False),
                                           ("syc_16", True)])
def test_plan_level_knit_c_entry(T, case, factored):
    """qk_knit (include/qknit.h): the whole knit of virtual_circuit.py:50-68 from the swept rows and
    the planner's transforms / clbit masks in one C call (what a non-Python host binds, see
    INTEGRATION.md) equals the oracle's dense knit (1e-12): 2 and 3 fragments, direct and factored
    transforms, wire cuts."""
    cut = {"hwe_16_1_p2": lambda: cutting.config_cut_circuit("hwe", 16, 1, 2)[1],
           "bv_5_1_p2": lambda: cutting.config_cut_circuit("bv", 5, 1, 2)[1],
           "cx_3cuts": lambda: circuits.two_fragment("cx", 3, 3, n_cuts=3)[1],
           "three": lambda: circuits.three_fragment(seed=9, sizes=(3, 2, 3))[1],
           "move_gate": lambda: circuits.wire_cut(3, 2, extra_gate_cut=True)[1],
           "syc_16": lambda: circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]}[case]()
    virt = VirtualCircuit(cut)
    ctx = engine.get_context(0)
    frags = engine.prepare_fragments(virt, 0, basis=factored)
    qs = [engine.sweep_fragment(ctx, fs) for fs in frags]
    got = engine.knit_plan_c(ctx, virt, frags, qs, factored=factored).cpu().numpy()
    assert np.abs(got - dense.run_dense(cut)).max() <= 1e-12


@pytest.mark.parametrize("K,nbits,bits_b,frac", [(1, 11, [0, 1, 2, 5, 6, 9], 0.3), (2, 11, [0, 3, 4, 5, 10], 0.05),
                                                 (8, 11, [0, 1, 2, 3, 8, 9, 10], 0.5), (2, 3, [0, 2], 0.5),
                                                 (3, 18, [0, 1, 2, 3, 8, 9, 10, 11, 16, 17], 0.001),
                                                 (5, 20, [0, 2, 4, 6, 8, 10, 12, 14, 16, 18], 0.0)])
def test_knit_select_matches_dense_threshold(T, K, nbits, bits_b, frac):
    """qk_knit_select: the entries |v| > acc of the small-K two-fragment knit, formed without the
    dense vector, are exactly (keys and bit-identical values) the thresholded dense write of
    qk_knit_outer_stream; acc at a quantile of |v| (frac kept; 0.0: above the largest, nothing kept);
    a capacity too small at first is detected and the call repeated with room."""
    ctx = engine.get_context(0)
    bits_a = [b for b in range(nbits) if b not in bits_b]
    M, N = 1 << len(bits_a), 1 << len(bits_b)
    g = T.Generator(device="cuda").manual_seed(101 + K)
    A = T.randn(K, M, dtype=T.float64, device="cuda", generator=g)
    B = T.randn(K, N, dtype=T.float64, device="cuda", generator=g)
    B[:, ::7] *= 1e-3  # column blocks of very different scale: some tiles bounded out
    dense_out = T.empty(1 << nbits, dtype=T.float64, device="cuda")
    engine.knit_outer_stream(ctx, A, B, bits_a, bits_b, nbits, dense_out)
    mags = dense_out.abs()
    acc = float(mags.max()) * 1.01 if frac == 0.0 else float(T.quantile(mags.cpu(), 1.0 - frac))
    ref_keys = T.nonzero(mags > acc).reshape(-1)
    keys, vals = engine.knit_select(ctx, A, B, bits_a, bits_b, nbits, acc, capacity=max(1, ref_keys.numel() // 3))
    order = T.argsort(keys)
    assert T.equal(keys[order], ref_keys)
    assert T.equal(vals[order], dense_out[ref_keys])
    # device K: 0 writes nothing, 1 keeps the first term only
    k0 = T.zeros(1, dtype=T.int32, device="cuda")
    keys0, _ = engine.knit_select(ctx, A, B, bits_a, bits_b, nbits, 0.0, k_dev=k0)
    assert keys0.numel() == 0


@pytest.mark.parametrize("seed,n", [(0, 1), (1, 37), (2, 1000), (3, 1 << 16), (4, 300001)])
def test_npd_pairs_matches_oracle(T, seed, n):
    """qk_npd_pairs on shuffled, already truncated (key, value) pairs == quasi_distr.py:28-43 (oracle)."""
    from oracle.quasi import QD

    rng = np.random.default_rng(seed)
    v = rng.standard_normal(n) * np.where(rng.random(n) < 0.3, 1e-4, 1e-2)
    v[rng.random(n) < 0.2] *= -1.0
    v[rng.random(n) < 0.05] = 3e-3  # ties
    keys = rng.permutation(1 << 20)[:n].astype(np.int64)
    ctx = engine.get_context(0)
    k, vals = engine.npd_pairs(ctx, T.from_numpy(keys).cuda(), T.from_numpy(v).cuda())
    ref = QD({int(a): float(b) for a, b in sorted(zip(keys, v))}, 0.0).npd()
    assert dict(zip(k.tolist(), vals.tolist())).keys() == ref.keys()
    got = dict(zip(k.tolist(), vals.tolist()))
    # the dropped negative mass (beta, qd:36-41) is summed sequentially by the reference and by a scan
    # here: ~3e4 terms of ~1e-2, so the shift beta / n agrees to a few 1e-16 of |beta| / n
    if ref:
        assert max(abs(got[a] - ref[a]) for a in ref) <= 1e-13
    assert list(vals) == sorted(vals)


@pytest.mark.parametrize("n,base", [(1, 0), (1000, 5), ((1 << 22) + 3, 1 << 40)])
def test_select_above_matches_numpy(T, n, base):
    """qk_select_above (the multi-GPU dict's dense fallback): exactly the entries |v| > acc, keys offset by
    the slice start, each once (unordered: compared as sorted sets)."""
    g = T.Generator(device="cuda").manual_seed(n)
    v = (T.rand(n, dtype=T.float64, device="cuda", generator=g) - 0.5) * 2e-5
    if n > 10:
        v[:: max(n // 50, 1)] = 3e-5
    keys, vals = engine.select_above(engine.get_context(0), v, 1e-5, key_base=base)
    h = v.cpu().numpy()
    idx = np.flatnonzero(np.abs(h) > 1e-5)
    order = np.argsort(keys.cpu().numpy())
    assert np.array_equal(keys.cpu().numpy()[order], idx + base)
    assert np.array_equal(vals.cpu().numpy()[order], h[idx])


@pytest.mark.parametrize("case", ["bv_5_1_p2", "hwe_16_1_p2", "hwe_16_1_p3"])
def test_run_virtual_circuit_dict_thresholded_matches_golden(T, case):
    """run_virtual_circuit(virt) (dict) through the cached plan's thresholded knit (qk_knit_select +
    qk_npd_pairs, no dense vector) == the reference's NPD result at ACCURACY 1e-5 (golden)."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import run as runmod

    _, cut = CASES[case]()
    res, _ = run_virtual_circuit(VirtualCircuit(cut))
    pipe = runmod.cached_plan(VirtualCircuit(cut), 0)
    gold = json.load(open(os.path.join(GOLD, f"knit_{case}.json")))
    ref = {int(k): v for k, v in gold["npd_acc_1e-05"]}
    assert set(res) == set(ref)
    assert max(abs(res[k] - ref[k]) for k in ref) <= 1e-9
    if case != "hwe_16_1_p3":  # three fragments: the dense knit + qk_npd
        assert pipe.last_kernel == "qk_knit_select_kernel"


TRUNC_CASES = ["bv_5_1_p2", "cp", "cx", "cx_3cuts", "cy", "cz", "hwe_16_1_p2", "hwe_16_1_p3", "move", "move_gate",
               "partial", "rzz", "rzz_0", "rzz_pi", "same_fragment", "three"]


def _truncation_bound(virt) -> float:
    """Bound on |exact-then-truncate - reference-truncated| per output (the default mode's documented
    difference): each truncation drops at most ACCURACY; a leaf merge of F fragment
    results carries F from_counts and F - 1 merge truncations; a gate's knit scales its inputs'
    errors by sum_i |a_i| and adds one truncation per + / - / scalar * (2 n + 1); the final
    truncation of the exact result adds one more."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import quasi_distr

    F = sum(1 for f in virt.fragment_circuits if len(f))
    e = 2 * F - 1
    for instr in reversed(virt.vgate_instructions):
        g = instr.operation
        e = sum(abs(a) for a in g.knit_coefficients()) * e + 2 * g.num_instantiations + 1
    return (e + 1) * quasi_distr.ACCURACY


@pytest.mark.parametrize("case", TRUNC_CASES)
def test_reference_truncation_matches_reference_knit(T, case):
    """run_virtual_circuit(truncation="reference"): ACCURACY applied after from_counts, every merge and
    every per-gate + - * (quasi_distr.py:7-10) on exact instances, on the GPU (qk_qd_*). The knit equals
    the reference VirtualCircuit.knit at ACCURACY 1e-5 (golden knit_acc_1e-05) and the dict equals its
    NPD (npd_acc_1e-05) key for key within 1e-12 — including cx_3cuts, move, move_gate, same_fragment and
    three, where truncating once at the end differs. The default mode stays within its bound."""
    _, cut = CASES[case]()
    gold = json.load(open(os.path.join(GOLD, f"knit_{case}.json")))
    knit_ref = {int(k): v for k, v in gold["knit_acc_1e-05"]}
    npd_ref = {int(k): v for k, v in gold["npd_acc_1e-05"]}
    d, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True, truncation="reference")
    d = d.cpu().numpy()
    nz = {int(k): float(d[k]) for k in np.flatnonzero(d)}
    assert set(nz) == set(knit_ref)
    assert max((abs(nz[k] - knit_ref[k]) for k in knit_ref), default=0.0) <= 1e-12
    res, _ = run_virtual_circuit(VirtualCircuit(cut), truncation="reference")
    assert set(res) == set(npd_ref)
    assert max((abs(res[k] - npd_ref[k]) for k in npd_ref), default=0.0) <= 1e-12
    virt = VirtualCircuit(cut)
    default, _ = run_virtual_circuit(virt, dense=True)
    default = default.cpu().numpy()
    keys = set(knit_ref) | {int(k) for k in np.flatnonzero(np.abs(default) > 1e-5)}
    diff = max((abs((default[k] if abs(default[k]) > 1e-5 else 0.0) - knit_ref.get(k, 0.0)) for k in keys),
               default=0.0)
    assert diff <= _truncation_bound(virt)


@pytest.mark.slow
def test_syc_32_5_thresholded_dict_equals_dense_npd(T):
    """Headline config: the dict result from the plan's thresholded knit (device data rank, then
    qk_knit_select on the compressed operands) equals the dense step + qk_threshold_count + qk_npd
    bit for bit — at ACCURACY = 1e-5 (empty: no outcome of the 2^32 reaches it) and at thresholds
    that keep a handful, thousands and 2^28 entries."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref")[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    dense_out = pipe.step()
    ctx = engine.get_context(0)
    top = float(dense_out.abs().max())
    for acc in (1e-5, 0.5 * top, 0.05 * top, 3e-9):  # nothing / the largest few / ~10^4-10^5 / 2^28 kept
        k_ref, v_ref = engine.nearest_probability_distribution(ctx, dense_out, acc)
        k, v = pipe.knit_dict(acc)
        assert pipe.last_kernel == "qk_knit_select_kernel"
        assert np.array_equal(k, k_ref) and np.array_equal(v, v_ref), (acc, len(k), len(k_ref))
        assert (len(k) == 0) == (acc == 1e-5)
    pipe.sync_stats()
    assert pipe.rank_fallbacks == 0
    del pipe, dense_out
    T.cuda.empty_cache()


@pytest.mark.parametrize("case,reject", [("hwe_16_1_p2", False), ("hwe_16_1_p2", True), ("cx_8x8", False),
                                         ("cx_8x8", True)])
def test_knit_lowrank_c_entry_matches_oracle(T, case, reject):
    """qk_knit_lowrank — the benched single-GPU knit (operands + Grams + probes, rank factors,
    compression, probe check, write-bound knit, predicated exact contraction) as ONE C call through
    ctypes — against the oracle's dense knit; reject=True (rank_tol < 0) forces the exact path."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    if case == "cx_8x8":
        circ, cut = circuits.two_fragment("cx", 8, 8, n_cuts=2, seed=11)
    else:
        circ, cut = CASES[case]()
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    qs = pipe.sweep()
    out, rank = engine.knit_lowrank_c(engine.get_context(0), pipe, qs, rank_tol=float("nan") if reject else None,
                                      rank_tol_rel=float("nan") if reject else None)
    np.testing.assert_allclose(out.cpu().numpy(), dense.run_dense(cut), atol=TOL, rtol=0)
    r = int(rank.item())
    assert (r == 0) if reject else (0 <= r <= 8)


@pytest.mark.slow
@pytest.mark.parametrize("qprep", [False, True])
def test_knit_lowrank_c_entry_syc_32_5_equals_bench_step(T, qprep, monkeypatch):
    """The one-call C entry on the headline workload writes the bench step's distribution bit for bit
    (same kernels, same probes and tolerances, chained in C instead of Python) — with the default
    X-path preparation and with the opt-in q-space chain (QKNIT_QPREP=1) on both sides."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "QPREP", qprep)
    monkeypatch.setenv("QKNIT_QPREP", "1" if qprep else "0")
    cut = cutting.config_cut_circuit("syc", 32, 5, 2, "ref")[1]
    pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
    ref = pipe.step()
    assert pipe.last_prep == ("qspace" if qprep else "fused")
    out, rank = engine.knit_lowrank_c(engine.get_context(0), pipe, pipe.sweep())
    assert 1 <= int(rank.item()) <= 8
    assert _chunked_max_abs_diff(out, ref) == 0.0
    del out, ref, pipe
    T.cuda.empty_cache()


def test_comm_collectives_c_entry_single_rank(T):
    """qk_comm_unique_id / qk_comm_init / qk_allreduce / qk_reduce / qk_allgather / qk_alltoall through
    ctypes on a world of one (RCCL allows one rank per GPU): each is the identity / a copy there."""
    ctx = engine.get_context(0)
    comm = engine.Comm(ctx, engine.Comm.unique_id(), 1, 0)
    try:
        x = T.arange(1000, dtype=T.float64, device="cuda") * 0.5
        for op in ("allreduce", "reduce", "allgather", "alltoall"):
            y = T.full_like(x, float("nan"))
            if op == "alltoall":
                comm.alltoall(x, y, 1)
            else:
                getattr(comm, op)(x, y)
            T.cuda.synchronize()
            assert T.equal(x, y), op
        n, r = ctypes_size(ctx, comm)
        assert (n, r) == (1, 0)
    finally:
        comm.close()


def ctypes_size(ctx, comm):
    import ctypes

    n, r = ctypes.c_int(), ctypes.c_int()
    ctx.check(ctx.lib.qk_comm_size(comm.handle, ctypes.byref(n), ctypes.byref(r)), "qk_comm_size")
    return n.value, r.value


@pytest.mark.parametrize("key", ["syc_32_5_p2", "syc_32_1_p2", "syc_32_1_p2_forced", "qft_16_1_p3"])
def test_lane_exchange_sweep_is_bit_identical(T, monkeypatch, key):
    """Per-program sweep kernels with cross-lane butterflies (v_permlane16/32_swap at 1-2-bit fiber-group
    boundaries, sweep_codegen._plan_layouts) against the same kernels through LDS only
    (QKNIT_SWEEP_LANE_XCHG=0), the shuffle form that keeps FINAL passes out of LDS (=2) and the opaque
    thread index of the FINAL job loop (QKNIT_SWEEP_OPAQUE_TID): the variants only move amplitudes
    between lanes or change register allocation, so every swept row is bit-identical; the bench plan
    (basis-reduced) and, for syc 32 5, the full direct plan."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import sweep_codegen
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    plans = [True, False] if key == "syc_32_5_p2" else [var == "forced" or key == "syc_32_5_p2"]
    for factored in plans:
        rows = {}
        for x, ot in (("0", "0"), ("1", "0"), ("1", "1"), ("2", "1")):
            monkeypatch.setenv("QKNIT_SWEEP_LANE_XCHG", x)
            monkeypatch.setenv("QKNIT_SWEEP_OPAQUE_TID", ot)
            pipe = KnitPipeline(VirtualCircuit(cut), factored=factored, jit=True)
            rows[x + ot] = [q.clone() for q in pipe.sweep()]
            del pipe
        for v in ("10", "11", "21"):
            assert len(rows[v]) == len(rows["00"])
            for a, b in zip(rows[v], rows["00"]):
                assert T.equal(a, b), v
    monkeypatch.setenv("QKNIT_SWEEP_LANE_XCHG", "1")
    assert sweep_codegen.lane_exchange_enabled()



def test_reference_truncation_refuses_huge_third_fragment_merges(T, monkeypatch):
    """truncation='reference' refuses a third-fragment merge beyond truncated.MAX_MERGE_ITEMS products
    per label (2^34 by default; forced to 1 here) with a ValueError that names the default truncation,
    instead of running for hours ("Reference truncation"); the default truncation of
    the same circuit still equals the oracle."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import truncated

    cut = circuits.three_fragment()[1]
    monkeypatch.setattr(truncated, "MAX_MERGE_ITEMS", 1)
    with pytest.raises(ValueError, match="use the default truncation"):
        run_virtual_circuit(VirtualCircuit(cut), dense=True, truncation="reference")
    d, _ = run_virtual_circuit(VirtualCircuit(cut), dense=True)
    np.testing.assert_allclose(d.cpu().numpy(), dense.run_dense(cut), atol=TOL, rtol=0)


def test_slice_buffers_selected_across_worlds_without_sync(T, monkeypatch):
    """Slice-mode pipelines of 2, then 4, then 8 ranks stepped in ONE process (rank 0's slice each;
    replicated preparation, no collective), every slice buffer chosen as the best of OUT_TRIES
    write-rate-checked mappings (forced on these 2^20-entry outputs), no synchronisation or collection
    between the worlds — the sequence of round 5's once-faulting rank_sim run (profiles/r05bb_*): every
    step's slice equals the oracle's, and qk_out_stats sees no failed reservation and no error left
    for a write-rate probe."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    monkeypatch.setattr(engine, "OUT_MAPPED_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_SELECT_MIN_BYTES", 0)
    monkeypatch.setattr(engine, "OUT_FAST_GBS", float("inf"))
    monkeypatch.setattr(engine, "OUT_TRIES", 3)
    monkeypatch.setenv("QKNIT_SLICE_PREP", "replicated")
    cut = circuits.two_fragment("cx", 10, 10, n_cuts=4)[1]  # 2^20 outputs: 1-MiB slices at 8 ranks
    ref = dense.run_dense(cut)
    st0 = engine.out_stats()
    stream = T.cuda.Stream()
    with T.cuda.stream(stream):
        for world in (2, 4, 8):
            pipe = KnitPipeline(VirtualCircuit(cut), factored=True, rank=0, world=world, mode="slice",
                                data_rank=True)
            assert pipe.slice_prep == "replicated" and pipe.overlap_ok()
            pipe.overlap = True  # pipelined steps over 2 / 2 / 3 rotating slice buffers
            o0, n = pipe.slice
            for _ in range(4):
                got = pipe.step()
                np.testing.assert_allclose(got[:n].cpu().numpy(), ref[o0:o0 + n], atol=TOL, rtol=0)
            del pipe, got
    st = engine.out_stats()
    assert st["reserve_failed"] == st0["reserve_failed"] and st["map_failed"] == st0["map_failed"]
    assert st["probe_pre_errors"] == st0["probe_pre_errors"]
    assert st["reserved"] > st0["reserved"]


@pytest.mark.slow
def test_syc_32_5_every_rank_slice_matches_reference_knit_samples(T):
    """The multi-GPU result pinned to the reference's own knit directly (not through the single-GPU
    step): for 2, 4 and 8 ranks, EVERY rank's slice-mode pipeline (replicated preparation, pipelined
    steps over its rotating slice buffers, no collective in the step — each rank runs standalone here)
    writes its contiguous share of the 2^32 outputs; the reference-knit keys (make_golden.py --samples:
    the reference VirtualCircuit.knit on exact instances at 4096 keys) falling into each slice equal the
    reference values (1e-12 absolute, 1e-9 relative above 1e-13), and the slices together cover all
    4096 keys once per world."""
    from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline

    gold = json.load(open(os.path.join(GOLD, "knit_samples_syc_32_5_p2.json")))
    name, n, d, p, var = cutting.BASELINE_CONFIGS[gold["case"]]
    cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
    keys_all = np.array(gold["keys"], dtype=np.int64)
    ref_all = np.array(gold["values"])
    stream = T.cuda.Stream()
    with T.cuda.stream(stream):
        for world in (2, 4, 8):
            covered = 0
            for rank in range(world):
                pipe = KnitPipeline(VirtualCircuit(cut), factored=True, rank=rank, world=world, mode="slice")
                assert pipe.slice_prep == "replicated"
                pipe.overlap = pipe.overlap_ok()
                o0, cnt = pipe.slice
                sel = (keys_all >= o0) & (keys_all < o0 + cnt)
                idx = T.tensor(keys_all[sel] - o0, dtype=T.int64, device="cuda")
                for _ in range(2):  # the first (plain) step and a pipelined one
                    out = pipe.step()
                    got = out[idx].cpu().numpy()
                    err = np.abs(got - ref_all[sel])
                    assert err.size == 0 or err.max() <= TOL, (world, rank, err.max())
                    big = np.abs(ref_all[sel]) > 1e-13
                    assert not big.any() or (err[big] / np.abs(ref_all[sel][big])).max() <= 1e-9
                pipe.sync_stats()
                assert pipe.rank_fallbacks == 0
                covered += int(sel.sum())
                del out, pipe
                T.cuda.empty_cache()
            assert covered == len(keys_all)
