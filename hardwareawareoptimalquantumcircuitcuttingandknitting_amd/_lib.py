"""ctypes binding of ``libqknit.so`` (declared in ``include/qknit.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc
--offload-arch=gfx950``). There is no fallback: if the shared object is missing
or fails to load, :func:`lib` raises, and so does every GPU entry point.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QKNIT_LIB") or os.path.join(_HERE, "libqknit.so")

c_i32, c_i64, c_u32, c_u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
c_vp, c_dp, c_lp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)


class QkPass(ctypes.Structure):
    _fields_ = [("tile_mask", c_u64), ("group_begin", c_i32), ("group_end", c_i32),
                ("flags", c_i32), ("traced_local", c_u32)]


class QkProgram(ctypes.Structure):
    _fields_ = [("n", c_i32), ("n_eff", c_i32), ("m", c_i32), ("n_slots", c_i32),
                ("packed", c_i32), ("n_passes", c_i32), ("passes", ctypes.POINTER(QkPass)),
                ("ops", c_vp), ("groups", c_vp), ("mats", c_vp)]


class QkLowrankPlan(ctypes.Structure):
    _fields_ = [("nbits", c_i32), ("terms", c_i32), ("rows_a", c_i64), ("rows_b", c_i64), ("mask_a", c_u64),
                ("mask_b", c_u64), ("wt_a", c_vp), ("wt_b", c_vp), ("probes", c_vp), ("lam_tol", ctypes.c_double),
                ("s_tol", ctypes.c_double), ("s_abs", ctypes.c_double), ("rank_tol", ctypes.c_double),
                ("rank_tol_rel", ctypes.c_double)]


class QkKnitPlan(ctypes.Structure):
    _fields_ = [("n_frag", c_i32), ("nbits", c_i32), ("terms", c_i64), ("rows", ctypes.POINTER(c_i64)),
                ("clbit_masks", ctypes.POINTER(c_u64)), ("transforms", ctypes.POINTER(c_vp))]


#: every symbol include/qknit.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "qk_version": (ctypes.c_char_p, []),
    "qk_ctx_create": (c_i32, [ctypes.c_int, ctypes.POINTER(c_vp)]),
    "qk_ctx_destroy": (c_i32, [c_vp]),
    "qk_ctx_set_stream": (c_i32, [c_vp, c_vp]),
    "qk_ctx_synchronize": (c_i32, [c_vp]),
    "qk_last_error": (ctypes.c_char_p, [c_vp]),
    "qk_stream_create_cu_masked": (c_i32, [ctypes.c_int, ctypes.POINTER(c_u32), ctypes.c_int, ctypes.POINTER(c_vp)]),
    "qk_stream_destroy": (c_i32, [c_vp]),
    "qk_stream_cu_count": (c_i32, [ctypes.c_int, c_vp, ctypes.POINTER(ctypes.c_int)]),
    "qk_out_alloc": (c_i32, [c_vp, c_i64, ctypes.POINTER(c_vp)]),
    "qk_out_free": (c_i32, [c_vp, c_vp]),
    "qk_out_mapped_bytes": (c_i32, [c_vp, ctypes.POINTER(c_i64)]),
    "qk_out_write_rate": (c_i32, [c_vp, c_vp, c_i64, ctypes.POINTER(ctypes.c_double)]),
    "qk_out_stats": (c_i32, [ctypes.POINTER(c_i64), c_i32]),
    "qk_sweep_workspace_bytes": (c_i32, [ctypes.POINTER(QkProgram), c_i64, ctypes.POINTER(c_i64)]),
    "qk_sweep": (c_i32, [c_vp, ctypes.POINTER(QkProgram), c_i64, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "qk_module_compile": (c_i32, [c_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                  ctypes.POINTER(c_vp)]),
    "qk_module_destroy": (c_i32, [c_vp]),
    "qk_module_load": (c_i32, [c_vp, c_vp, c_i64, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(c_vp)]),
    "qk_module_code": (c_i32, [c_vp, c_vp, ctypes.POINTER(c_i64)]),
    "qk_sweep_compiled": (c_i32, [c_vp, c_vp, ctypes.POINTER(QkProgram), c_i64, c_vp, c_vp, c_vp, c_i64,
                                  c_vp]),
    "qk_sweep_compiled_labels": (c_i32, [c_vp, c_vp, ctypes.POINTER(QkProgram), c_i64, c_vp, c_vp, c_i64, c_vp,
                                         c_vp, c_i64, c_vp]),
    "qk_sweep_compiled_multi": (c_i32, [c_vp, c_vp, ctypes.c_int, ctypes.POINTER(QkProgram), c_lp, c_vp, c_vp, c_lp,
                                        c_vp, c_vp, c_lp, c_vp, c_vp]),
    "qk_sweep_compiled_multi_shared": (c_i32, [c_vp, c_vp, ctypes.c_int, ctypes.POINTER(QkProgram), c_lp, c_vp, c_vp,
                                               c_lp, c_vp, c_vp, c_lp, c_vp, c_vp, c_lp, c_vp, c_vp]),
    "qk_reduce_labels": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "qk_gemm_keyed": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                              c_vp, c_i64, c_vp, ctypes.c_int]),
    "qk_gemm_keyed_pred": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                   c_vp, c_i64, c_vp, ctypes.c_int, c_vp]),
    "qk_gemm_outer_paired": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                     c_vp, c_vp]),
    "qk_knit_outer_stream": (c_i32, [c_vp, ctypes.c_int, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.c_uint64,
                                     ctypes.c_uint64, c_vp]),
    "qk_knit_outer_stream_kind": (c_i32, [ctypes.c_int, c_i64, c_u64, c_u64, c_i64, c_i64,
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "qk_knit_outer_stream_range": (c_i32, [c_vp, ctypes.c_int, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.c_uint64,
                                           ctypes.c_uint64, c_i64, c_i64, c_vp, c_vp]),
    "qk_rank_factors": (c_i32, [c_vp, c_i64, c_vp, c_vp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_int, c_vp, c_vp, c_vp]),
    "qk_prep_workspace_bytes": (c_i32, [c_vp, c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "qk_prep_operands": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_i64, c_vp, ctypes.c_int,
                                 c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64]),
    "qk_qprep_workspace_bytes": (c_i32, [c_vp, c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "qk_qprep_grams": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_i64, ctypes.c_int, c_vp, c_vp,
                               c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64]),
    "qk_qprep_compress_check": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_i64,
                                        ctypes.c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_vp, ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp, c_i64]),
    "qk_compress_operands": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                     c_vp]),
    "qk_compress_operands_ld": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp,
                                        c_vp, c_i64, c_i64, c_vp, c_i64]),
    "qk_compress_probe_v": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp,
                                    c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64]),
    "qk_probe_errors_vpart": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp,
                                      c_i64, c_vp, c_vp, ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp, c_i64,
                                      c_vp]),
    "qk_probe_workspace_bytes": (c_i32, [c_vp, c_i64, ctypes.POINTER(c_i64)]),
    "qk_probe_errors": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64,
                                c_i64, c_vp, c_i64, c_vp, c_vp, ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp,
                                c_i64]),
    "qk_probe_errors_tally": (c_i32, [c_vp, ctypes.c_int, ctypes.c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64,
                                c_i64, c_vp, c_i64, c_vp, c_vp, ctypes.c_double, ctypes.c_double, c_vp, c_vp, c_vp,
                                c_i64, c_vp]),
    "qk_probe_accept": (c_i32, [c_vp, c_vp, ctypes.c_int, c_vp, ctypes.c_double, ctypes.c_double, c_vp, c_vp]),
    "qk_rank_tally": (c_i32, [c_vp, c_vp, c_vp, c_vp]),
    "qk_knit_workspace_bytes": (c_i32, [ctypes.POINTER(QkKnitPlan), ctypes.POINTER(c_i64)]),
    "qk_knit": (c_i32, [c_vp, ctypes.POINTER(QkKnitPlan), c_vp, c_vp, c_i64, c_vp]),
    "qk_khatri_rao": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "qk_gather_rows": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "qk_npd_workspace_bytes": (c_i32, [c_i64, c_i64, ctypes.POINTER(c_i64)]),
    "qk_threshold_count": (c_i32, [c_vp, c_i64, c_vp, ctypes.c_double, c_vp, c_i64, c_vp]),
    "qk_npd": (c_i32, [c_vp, c_i64, c_vp, ctypes.c_double, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "qk_qd_from_rows": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, ctypes.c_double, c_vp]),
    "qk_qd_merge": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, ctypes.c_double, c_i64, c_vp]),
    "qk_qd_axpby": (c_i32, [c_vp, c_i64, ctypes.c_double, c_vp, ctypes.c_double, c_vp, ctypes.c_double, c_vp]),
    "qk_hellinger": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "qk_knit_lowrank_workspace_bytes": (c_i32, [c_vp, c_vp, ctypes.POINTER(c_i64)]),
    "qk_knit_lowrank": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "qk_comm_unique_id": (c_i32, [c_vp]),
    "qk_comm_init": (c_i32, [c_vp, c_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_vp)]),
    "qk_comm_destroy": (c_i32, [c_vp]),
    "qk_comm_size": (c_i32, [c_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "qk_allreduce": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64]),
    "qk_reduce": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.c_int]),
    "qk_allgather": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64]),
    "qk_alltoall": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64]),
    "qk_knit_select_workspace_bytes": (c_i32, [ctypes.c_int, c_u64, c_u64, ctypes.POINTER(c_i64)]),
    "qk_knit_select": (c_i32, [c_vp, ctypes.c_int, c_i64, c_vp, c_i64, c_vp, c_i64, c_u64, c_u64, ctypes.c_double,
                               c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "qk_select_above": (c_i32, [c_vp, c_i64, c_vp, ctypes.c_double, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "qk_npd_pairs_workspace_bytes": (c_i32, [c_i64, ctypes.POINTER(c_i64)]),
    "qk_npd_pairs": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "qk_sample_cdf": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "qk_sample_counts": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_u64, c_vp]),
    "qk_fold_counts": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, ctypes.c_double, c_vp]),
}

_lock = threading.Lock()
_lib = None


class QknitError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise QknitError(
                    f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                )
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
        return _lib


def check(ctx, status: int, what: str) -> None:
    if status != 0:
        msg = lib().qk_last_error(ctx)
        raise QknitError(f"{what} failed (status {status}): {msg.decode() if msg else ''}")
