"""Knit executor: a virtual circuit compiled once, then swept + knitted repeatedly.

``run_virtual_circuit`` (``run.py:23-71`` in the reference) rebuilds and re-runs
every instance each call. :class:`KnitPipeline` splits that into a *plan*
(fragment programs, job tables, knit operands and all device buffers, built
once) and a *step* (the hot path: batched sweep of every fragment instance,
then the dense knit), so repeated runs — and the benchmark — time only device
work. All device work goes through a backend object; the product backend is
:class:`HipBackend` (``libqknit.so``). Tests substitute a CPU model to exercise
the multi-rank orchestration with ``gloo``.

Multi-GPU (one process per GPU, ``torch.distributed`` over RCCL/xGMI): the
instance labels of every fragment are sharded contiguously across ranks; one
collective then assembles the reconstruction:

* ``reduce`` mode — each rank sweeps only the fragment rows its slice of global
  labels needs, contracts a partial distribution over that slice, and a single
  ``reduce`` (sum) lands the full distribution on rank 0. Chosen when the output
  (``2^N`` fp64) is smaller than the instance tensors (hwe/bv/qft sizes).
* ``gather`` mode — each rank sweeps its label shard, a single ``all_gather``
  replicates the signed instance tensors ``q_f`` (1.36 GB for syc 32 5), and each
  rank computes its own block of output rows (no 34 GB reduction; the result
  stays row-sharded in ``(x_A, x_B)`` order).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import engine
from .fragment_program import JobTable


def _shard(n: int, rank: int, world: int) -> tuple[int, int]:
    per = -(-n // world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


class HipBackend:
    """Device work of the pipeline on one GPU through the C ABI."""

    def __init__(self, device: int = 0):
        self.T = engine.torch()
        self.device = device
        self.dev = self.T.device("cuda", device)
        self.ctx = engine.get_context(device)

    def prepare_fragments(self, virt):
        return engine.prepare_fragments(virt, self.device)

    def upload_jobs(self, jobs: JobTable):
        return engine.jobs_to_device(jobs, self.device)

    def workspace_bytes(self, fs, n_jobs: int) -> int:
        need = ctypes.c_int64()
        self.ctx.check(self.ctx.lib.qk_sweep_workspace_bytes(ctypes.byref(fs.dprog.struct), n_jobs,
                                                             ctypes.byref(need)), "qk_sweep_workspace_bytes")
        return need.value

    def empty(self, shape, dtype):
        return self.T.empty(shape, dtype=dtype, device=self.dev)

    def zeros(self, shape, dtype):
        return self.T.zeros(shape, dtype=dtype, device=self.dev)

    def to_device(self, arr):
        return self.T.from_numpy(np.ascontiguousarray(arr)).to(self.dev)

    def sweep(self, fs, slot, sign, n_jobs, pjob, ws):
        engine.sweep_jobs(self.ctx, fs.dprog, slot, sign, n_jobs, pjob=pjob, workspace=ws)

    def reduce_labels(self, pjob, off, n_labels, q):
        return engine.reduce_labels(self.ctx, pjob, off, n_labels, q=q)

    def gather_rows(self, q, idx, coef):
        return engine.gather_rows(self.ctx, q, idx, coef)

    def gemm_keyed(self, A, B, **kw):
        return engine.gemm_keyed(self.ctx, A, B, **kw)

    def khatri_rao(self, A, B):
        return engine.khatri_rao(self.ctx, A, B)

    def event(self):
        return self.T.cuda.Event(enable_timing=True)


class KnitPipeline:
    def __init__(self, virt, device: int = 0, factored: bool = False, rank: int = 0, world: int = 1,
                 mode: str | None = None, group=None, backend=None):
        self.be = backend if backend is not None else HipBackend(device)
        self.T = engine.torch()
        self.virt = virt
        self.rank, self.world, self.group = rank, world, group
        self.factored = factored
        self.frags = self.be.prepare_fragments(virt)
        self.ops = engine.knit_operands(virt, self.frags, factored)
        self.N = virt.circuit.num_clbits
        q_bytes = sum(len(fs.labels) << fs.prog.m for fs in self.frags) * 8
        out_bytes = (1 << self.N) * 8
        if mode is None:
            mode = "single" if world == 1 else ("reduce" if (out_bytes <= q_bytes and not factored) else "gather")
        if mode == "reduce" and factored:
            raise ValueError("reduce mode needs the direct (label-sliced) knit")
        if mode not in ("single", "reduce", "gather"):
            raise ValueError(f"unknown mode {mode}")
        self.mode = mode
        self.events = []  # (start, end) events around the main contraction GEMM
        self.record_events = False
        self._plan()

    # ------------------------------------------------------------------ plan
    def _plan(self):
        T, be = self.T, self.be
        self.sweeps = []  # per fragment: device job tables and buffers, or None (dropped)
        L = self.ops.num_terms
        self.term_range = _shard(L, self.rank, self.world) if self.mode == "reduce" else (0, L)
        for i, fs in enumerate(self.frags):
            if fs.dropped:
                self.sweeps.append(None)
                continue
            nl = fs.n_rows
            if self.mode == "reduce":
                t0, t1 = self.term_range
                rows = np.unique(self.ops.rows[i][t0:t1])
                lo, hi = (int(rows.min()), int(rows.max()) + 1) if rows.size else (0, 0)
            elif self.mode == "gather":
                lo, hi = _shard(nl, self.rank, self.world)
            else:
                lo, hi = 0, nl
            jobs = fs.jobs
            j0, j1 = int(jobs.label_offsets[lo]), int(jobs.label_offsets[hi])
            sub = JobTable(jobs.slot_mats[j0:j1], jobs.sign[j0:j1], jobs.label_offsets[lo:hi + 1] - j0,
                           jobs.branch_bits[j0:j1])
            slot_t, sign_t, off_t = be.upload_jobs(sub)
            n_jobs = sub.n_jobs
            width = 1 << fs.prog.m
            need = be.workspace_bytes(fs, n_jobs) if n_jobs else 0
            self.sweeps.append(dict(lo=lo, hi=hi, slot=slot_t, sign=sign_t, off=off_t, n_jobs=n_jobs,
                                    pjob=be.empty((max(n_jobs, 1), width), T.float64),
                                    q=(be.empty((max(hi - lo, 1), width), T.float64)
                                       if n_jobs != hi - lo else None),
                                    ws=be.empty((max(need, 1),), T.uint8)))
        self._plan_knit()

    def _plan_knit(self):
        be, ops = self.be, self.ops
        self.gather_idx, self.gather_coef, self.transforms = [], [], []
        t0, t1 = self.term_range
        for i, fs in enumerate(self.frags):
            if ops.transforms[i] is not None:
                self.transforms.append(be.to_device(ops.transforms[i].T))
                self.gather_idx.append(None)
                self.gather_coef.append(None)
            else:
                self.transforms.append(None)
                sw = self.sweeps[i]
                base = sw["lo"] if (sw is not None and self.mode == "reduce") else 0
                self.gather_idx.append(be.to_device(ops.rows[i][t0:t1] - base))
                self.gather_coef.append(be.to_device(ops.coefs[i][t0:t1]))
        self.order = engine.contract_order(ops.clbits)
        self.row_block = None
        if self.mode == "gather":
            width_a = 1
            for i in self.order[:-1]:
                width_a <<= len(ops.clbits[i])
            self.row_block = _shard(width_a, self.rank, self.world)
        self.out = None

    # ------------------------------------------------------------------ step
    def sweep(self) -> list:
        """Instance sweep of every fragment; returns the per-label ``q_f`` tensors this rank needs."""
        T, be = self.T, self.be
        qs = []
        for i, fs in enumerate(self.frags):
            sw = self.sweeps[i]
            if sw is None:
                ones = be.zeros((fs.n_rows, 1), T.float64)
                ones += 1.0
                qs.append(ones)
                continue
            if sw["n_jobs"]:
                be.sweep(fs, sw["slot"], sw["sign"], sw["n_jobs"], sw["pjob"], sw["ws"])
            if sw["q"] is not None:
                q = be.reduce_labels(sw["pjob"], sw["off"], sw["hi"] - sw["lo"], sw["q"])
            else:
                q = sw["pjob"]
            q = q[: sw["hi"] - sw["lo"]]
            if self.mode == "gather":
                q = self._all_gather_rows(q, fs.n_rows)
            qs.append(q)
        return qs

    def _all_gather_rows(self, q, n_rows):
        import torch.distributed as dist

        T = self.T
        per = -(-n_rows // self.world)
        buf = self.be.zeros((per, q.shape[1]), q.dtype)
        buf[: q.shape[0]].copy_(q)
        full = self.be.empty((per * self.world, q.shape[1]), q.dtype)
        dist.all_gather_into_tensor(full, buf, group=self.group)
        return full[:n_rows]

    def operands(self, qs: list) -> list:
        T, be = self.T, self.be
        mats = []
        for i, q in enumerate(qs):
            q = q.contiguous()
            if self.transforms[i] is not None:
                W = self.transforms[i]
                a = be.empty((W.shape[1], q.shape[1]), T.float64)
                be.gemm_keyed(W, q, out=a, strideA=q.shape[1])
            else:
                a = be.gather_rows(q, self.gather_idx[i], self.gather_coef[i])
            mats.append(a)
        return mats

    def knit(self, qs: list):
        mats = self.operands(qs)
        if self.out is None:
            self.out = self._alloc_out(mats)
        if self.record_events:
            start, end = self.be.event(), self.be.event()
            start.record()
        res = self._contract(mats)
        if self.record_events:
            end.record()
            self.events.append((start, end))
        if self.mode == "reduce":
            import torch.distributed as dist

            dist.reduce(res, dst=0, group=self.group)
        return res

    def _alloc_out(self, mats):
        T = self.T
        if self.mode != "gather":
            return self.be.zeros((1 << self.N,), T.float64)
        lo, hi = self.row_block
        width_b = mats[self.order[-1]].shape[1]
        return self.be.zeros((max(hi - lo, 1) * width_b,), T.float64)

    def _contract(self, mats):
        if self.mode != "gather":
            return engine.contract(None, mats, self.ops.clbits, self.out, gemm=self.be.gemm_keyed,
                                   kr=self.be.khatri_rao)
        # output-sharded: compact [rows, 2^m_B] block in (x_A, x_B) order
        order = self.order
        A = mats[order[0]]
        for i in order[1:-1]:
            A = self.be.khatri_rao(A.contiguous(), mats[i].contiguous())
        B = mats[order[-1]]
        lo, hi = self.row_block
        A = A[:, lo:hi].contiguous()
        return self.be.gemm_keyed(A, B.contiguous(), keyA=None, strideA=B.shape[1], keyB=None, strideB=1,
                                  out=self.out)

    def step(self):
        return self.knit(self.sweep())

    # ------------------------------------------------------------------ accounting
    def instance_counts(self) -> dict:
        """Reference instance count (``run.py:37-39``: sum of per-fragment label lists) and jobs."""
        return {
            "instances_ref": int(sum(len(fs.labels) for fs in self.frags)),
            "instances_unique": int(sum(fs.n_rows for fs in self.frags)),
            "branch_jobs": int(sum(fs.jobs.n_jobs for fs in self.frags if not fs.dropped)),
            "labels": int(self.ops.num_terms),
        }

    def gemm_shape(self) -> tuple[int, int, int]:
        """(M, N, K) of the main contraction on this rank."""
        K = self.term_range[1] - self.term_range[0]
        widths = [1 << len(c) for c in self.ops.clbits]
        M = 1
        for i in self.order[:-1]:
            M *= widths[i]
        if self.row_block is not None:
            M = self.row_block[1] - self.row_block[0]
        return M, widths[self.order[-1]], K
