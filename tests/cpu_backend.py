"""CPU model of the pipeline backend — TEST INFRASTRUCTURE ONLY.

Implements the :class:`~...pipeline.HipBackend` interface on torch CPU tensors:
the sweep through tests/emulator.py (numpy model of the kernel semantics), the
keyed GEMM / Khatri-Rao / gathers in numpy. Lets tests run the multi-rank
orchestration of :class:`KnitPipeline` under ``gloo`` without a GPU.
"""
import numpy as np
import torch

from emulator import emulate

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import engine, sweep_plan


class _Ev:
    def record(self):
        pass

    def elapsed_time(self, other):
        return 0.0


class CpuBackend:
    def __init__(self):
        self.dev = torch.device("cpu")

    def prepare_fragments(self, virt, basis: bool = False, relevance: bool = True):
        return engine.prepare_fragments(virt, upload=False, basis=basis, relevance=relevance)

    def upload_jobs(self, jobs):
        return jobs.slot_mats, torch.from_numpy(jobs.sign.copy()), torch.from_numpy(jobs.label_offsets.copy())

    def workspace_bytes(self, fs, n_jobs):
        return 0

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype)

    def zeros(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype)

    def to_device(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr))

    def sweep(self, fs, slot, sign, n_jobs, pjob, ws):
        enc = sweep_plan.encode(fs.prog)
        pjob[:n_jobs] = torch.from_numpy(emulate(enc, slot[:n_jobs], sign.numpy()[:n_jobs]))

    def reduce_labels(self, pjob, off, n_labels, q):
        o = off.numpy()
        for l in range(n_labels):
            q[l] = pjob[o[l]:o[l + 1]].sum(0)
        return q

    def gather_rows(self, q, idx, coef):
        return coef[:, None] * q[idx]

    def gemm_keyed(self, A, B, keyA=None, strideA=0, keyB=None, strideB=1, out=None, beta=0):
        C = (A.T @ B).numpy()
        M, N = C.shape
        ka = keyA.numpy() if keyA is not None else np.arange(M, dtype=np.int64) * strideA
        kb = keyB.numpy() if keyB is not None else np.arange(N, dtype=np.int64) * strideB
        idx = (ka[:, None] + kb[None, :]).reshape(-1)
        o = out.numpy().reshape(-1)
        if beta:
            o[idx] += C.reshape(-1)
        else:
            o[idx] = C.reshape(-1)
        return out

    def gemm_outer_paired(self, A, B, keyB, keyA=None, strideA=0, out=None):
        kb = keyB.numpy()
        assert A.shape[0] <= 8 and (kb[1::2] == kb[0::2] + 1).all() and (kb[0::2] % 2 == 0).all()
        return self.gemm_keyed(A, B, keyA=keyA, strideA=strideA, keyB=keyB, out=out)

    def knit_outer_stream(self, A, B, clbits_a, clbits_b, nbits, out):
        from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.knit_plan import deposit_keys

        assert A.shape[0] <= 8 and engine.stream_knit_ok(clbits_a, clbits_b, nbits)
        ka, kb = (torch.from_numpy(deposit_keys(list(c))) for c in (clbits_a, clbits_b))
        return self.gemm_keyed(A, B, keyA=ka, keyB=kb, out=out)

    def khatri_rao(self, A, B):
        K = A.shape[0]
        return torch.stack([torch.outer(B[k], A[k]).reshape(-1) for k in range(K)])

    def event(self):
        return _Ev()
