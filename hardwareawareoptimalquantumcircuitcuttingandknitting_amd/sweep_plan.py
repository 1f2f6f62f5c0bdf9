"""Tile/pass/fiber schedule of a fragment program for the HIP sweep kernel.

The kernel (``csrc/qknit.hip``, ``qk_sweep_pass``) processes a *tile* of
``2^12`` complex128 amplitudes (64 KiB) per 256-thread workgroup in LDS:

* PACKED mode (``n_eff <= 12``): a tile holds ``2^(12-n_eff)`` whole jobs, so a
  fragment is swept in ONE launch with no statevector traffic to HBM at all;
* SPLIT mode (``n > 12``): a tile holds 12 of the ``n`` state bits of one job
  (always including state bits ``0..LOW_BITS-1`` so HBM accesses are
  contiguous runs); ops are scheduled into *passes*, each of which can only
  touch its tile bits except through diagonal action (controls, phases), which
  is evaluated from the fixed non-tile bits.

Inside a pass, ops are cut into *groups* of at most 4 tile positions (the
*fiber*); each thread loads the 16 amplitudes of its fiber from LDS into
registers, applies every op of the group in registers, and writes them back
(one LDS round trip per group instead of per gate).

This module turns a :class:`FragmentProgram` into the flat arrays the C-ABI
takes (``include/qknit.h``: ``qk_op``, ``qk_group``, ``qk_pass``).
"""
from __future__ import annotations

import dataclasses
import itertools
import math
import os
from dataclasses import dataclass

import numpy as np

from .fragment_program import FragmentProgram, HostOp

TILE_BITS = 12
FIBER_BITS = 4
LOW_BITS = 5  # state bits always resident in a SPLIT tile (512-B contiguous runs)

# op kinds (must match qknit.h)
K_U1, K_D1, K_SLOT, K_U2, K_D2, K_CX, K_SWAP, K_SCALE, K_U1R, K_U1X, K_D1R, K_D2R, K_SCALER = range(13)

OP_DTYPE = np.dtype([("kind", "<i4"), ("a", "<i4"), ("b", "<i4"), ("e1", "<i4"),
                     ("e2", "<i4"), ("slot", "<i4"), ("mat", "<i4"), ("pad", "<i4")])
GROUP_DTYPE = np.dtype([("pos", "<i4", (4,)), ("op_begin", "<i4"), ("op_end", "<i4"),
                        ("pad", "<i4", (2,))])
PASS_DTYPE = np.dtype([("tile_mask", "<u8"), ("group_begin", "<i4"), ("group_end", "<i4"),
                       ("flags", "<i4"), ("traced_local", "<u4")])
PASS_INIT, PASS_FINAL = 1, 2


# ----------------------------------------------------------------------------- analysis
_Z0 = np.array([1, -1, 1, -1], dtype=np.float64)  # 4x4 little-endian on (q0, q1): index b0 + 2 b1
_Z1 = np.array([1, 1, -1, -1], dtype=np.float64)
_DIAG_MEMO: dict = {}


def _diag_qubits(op: HostOp) -> frozenset:
    """Qubits on which the op acts diagonally (it commutes with Z there). Memoised on the op's
    kind, qubits and matrix bytes: the pass scheduler asks for every op of every candidate tile
    width (syc 32 5: ~8000 queries for ~190 ops)."""
    if op.kind == "slot":
        return frozenset()
    m = np.asarray(op.mat)
    key = (op.kind, tuple(op.qubits), m.dtype.str, m.shape, m.tobytes())
    hit = _DIAG_MEMO.get(key)
    if hit is not None:
        return hit
    if op.kind == "u1":
        out = frozenset({op.qubits[0]}) if _is_diag(m) else frozenset()
    else:
        # [M, Z] = 0 for diagonal Z  <=>  M[i, j] (z_j - z_i) = 0 for every entry
        q = []
        for z, qb in ((_Z0, op.qubits[0]), (_Z1, op.qubits[1])):
            if np.all(np.abs(m * (z[None, :] - z[:, None])) <= 1e-15):
                q.append(qb)
        out = frozenset(q)
    if len(_DIAG_MEMO) > 65536:
        _DIAG_MEMO.clear()
    _DIAG_MEMO[key] = out
    return out


def _is_diag(m: np.ndarray) -> bool:
    return bool(np.all(m[~np.eye(m.shape[0], dtype=bool)] == 0))


def op_need(op: HostOp) -> set:
    return set(op.qubits) - _diag_qubits(op)


def drop_trailing_phases(prog: FragmentProgram) -> FragmentProgram:
    """The program without its trailing phases: a diagonal op whose entries all have modulus 1 and
    after which no op acts non-diagonally on any of its qubits commutes with everything that follows
    it (later ops on its qubits are diagonal; slot ops count as non-diagonal), so it can move to the
    end, where it multiplies each amplitude by a unit phase that |z|^2 — every output the sweep makes,
    measured or traced — cannot see. syc 32 5 drops 14 and 7 of its fragments' 94 ops (most from the
    FINAL pass), syc 32 1 10 and 13 of 23, qft 16 105 of 586. ``QKNIT_DROP_PHASES=0`` keeps them."""
    if os.environ.get("QKNIT_DROP_PHASES", "1") == "0":
        return prog
    later: set = set()  # qubits some later op acts on non-diagonally
    keep = []
    for op in reversed(prog.ops):
        qs = set(op.qubits)
        if op.kind != "slot" and op.mat is not None and _diag_qubits(op) >= qs and not (qs & later) \
                and np.all(np.abs(np.abs(np.diag(op.mat)) - 1.0) <= 1e-15):
            continue
        later |= qs if op.kind == "slot" else op_need(op)
        keep.append(op)
    if len(keep) == len(prog.ops):
        return prog
    return dataclasses.replace(prog, ops=keep[::-1])


# ----------------------------------------------------------------------------- passes
@dataclass
class Pass:
    tile: list  # sorted state bits resident in the tile (SPLIT); all bits (PACKED)
    ops: list  # HostOps in order


def _greedy_passes(ops: list, tile_bits: int, first_tile: set | None = None,
                   needs: list | None = None) -> list[Pass] | None:
    """Greedy schedule: each pass takes ops in order while their non-diagonal qubits fit the tile
    (an op touching a qubit of a deferred op is deferred too). ``first_tile`` fixes the first
    pass's tile instead of growing it (None when that pass could take nothing)."""
    # each op's (qubits, non-diagonal qubits), computed once per call (schedule_passes passes them in
    # for its up to 200 candidate first tiles)
    if needs is None:
        needs = [(set(op.qubits), op_need(op)) for op in ops]
    remaining = list(range(len(ops)))
    passes: list[Pass] = []
    fixed = first_tile
    while remaining:
        tile = set(fixed) if fixed is not None else set(range(LOW_BITS))
        taken, blocked, rest = [], set(), []
        for k in remaining:
            op = ops[k]
            qs, need = needs[k]
            if qs & blocked:
                blocked |= qs
                rest.append(k)
                continue
            if need <= tile or (fixed is None and len(tile | need) <= tile_bits):
                tile |= need
                taken.append(op)
            else:
                blocked |= qs
                rest.append(k)
        if not taken:
            if fixed is not None:
                return None
            raise RuntimeError("pass scheduler made no progress")  # first op always fits
        fixed = None
        passes.append(Pass(sorted(tile), taken))
        remaining = rest
    return passes


def schedule_passes(prog: FragmentProgram, tile_bits: int = TILE_BITS) -> list[Pass]:
    """Pass schedule for SPLIT programs with ``tile_bits``-bit tiles (PACKED: one pass).

    Greedy in op order; when that needs more than two passes, every choice of the first pass's
    tile (the low bits plus ``tile_bits - LOW_BITS`` of the others, at most 200 choices) is tried
    with the greedy after it, and the schedule with the fewest passes is kept (first found)."""
    n = prog.n
    if n <= TILE_BITS:
        return [Pass(list(range(n)), list(prog.ops))]
    traced = set(range(prog.m, n))
    if len(traced) > tile_bits - LOW_BITS:
        raise NotImplementedError("more traced qubits than a tile can hold")
    needs = [(set(op.qubits), op_need(op)) for op in prog.ops]
    passes = _greedy_passes(prog.ops, tile_bits, needs=needs)
    free = list(range(LOW_BITS, n))
    extra = tile_bits - LOW_BITS
    if len(passes) > 2 and 0 < extra < len(free) and math.comb(len(free), extra) <= 200:
        for combo in itertools.combinations(free, extra):
            cand = _greedy_passes(prog.ops, tile_bits, set(range(LOW_BITS)) | set(combo), needs=needs)
            if cand is not None and len(cand) < len(passes):
                passes = cand
                if len(passes) <= 2:
                    break
    if not passes:
        passes.append(Pass(sorted(set(range(LOW_BITS))), []))
    # final pass must hold every traced qubit; prefer swapping in unused bits
    last = passes[-1]
    tile = set(last.tile)
    used = set(range(LOW_BITS))
    for op in last.ops:
        used |= op_need(op)
    for q in traced - tile:
        if len(tile) < tile_bits:
            tile.add(q)
            continue
        spare = sorted(tile - used - traced)
        if spare:
            tile.discard(spare[-1])
            tile.add(q)
        else:
            passes.append(Pass([], []))
            tile = set(range(LOW_BITS)) | traced
            break
    passes[-1].tile = sorted(tile)
    # fill every tile to exactly TILE_BITS bits (lowest unused first)
    for p in passes:
        t = set(p.tile)
        for q in range(n):
            if len(t) >= tile_bits:
                break
            t.add(q)
        p.tile = sorted(t)
    return passes


# ----------------------------------------------------------------------------- encoding
@dataclass
class EncodedProgram:
    n: int  # fragment qubits
    n_eff: int  # padded width (>= FIBER_BITS)
    m: int
    n_slots: int
    packed: bool
    ops: np.ndarray  # OP_DTYPE
    groups: np.ndarray  # GROUP_DTYPE
    passes: np.ndarray  # PASS_DTYPE
    mats: np.ndarray  # float64, interleaved complex
    n_host_ops: int
    tile_bits: int = TILE_BITS  # SPLIT: state bits per tile (12 interpreter; 13 compiled kernels)

    @property
    def jobs_per_tile(self) -> int:
        return 1 << (TILE_BITS - self.n_eff) if self.packed else 1

    @property
    def tiles_per_job(self) -> int:
        return 1 if self.packed else 1 << (self.n - self.tile_bits)

    def pass_tile_bits(self, ip: int) -> int:
        """State bits of pass ``ip``'s tile (the FINAL pass's may be narrower: narrow_final_tile)."""
        return self.n_eff if self.packed else bin(int(self.passes[ip]["tile_mask"])).count("1")


class _Mats:
    def __init__(self):
        self.buf: list = []

    def add(self, *mats) -> int:
        off = len(self.buf)
        for m in mats:
            for z in np.asarray(m, dtype=np.complex128).ravel():
                self.buf.extend((float(z.real), float(z.imag)))
        return off

    def add_real(self, vals) -> int:
        off = len(self.buf)
        self.buf.extend(float(v) for v in np.asarray(vals, dtype=np.float64).ravel())
        return off


def _swap_order4(m: np.ndarray) -> np.ndarray:
    """Re-express a 4x4 (q0,q1) matrix in (q1,q0) order."""
    p = [0, 2, 1, 3]
    return m[np.ix_(p, p)]


def _is_cx(m: np.ndarray) -> bool:
    ref = np.array([[1, 0, 0, 0], [0, 0, 0, 1], [0, 0, 1, 0], [0, 1, 0, 0]], dtype=np.complex128)
    return bool(np.array_equal(m, ref))


def _is_swap(m: np.ndarray) -> bool:
    ref = np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.complex128)
    return bool(np.array_equal(m, ref))


def _block(m: np.ndarray, ctrl_pos: int, bit: int) -> np.ndarray:
    """2x2 block acting on the other qubit when qubit ``ctrl_pos`` (0/1) has value ``bit``."""
    if ctrl_pos == 0:
        idx = [bit, bit + 2]  # b0 fixed, b1 varies
    else:
        idx = [2 * bit, 2 * bit + 1]
    return m[np.ix_(idx, idx)]


def _d1(rec, mats: _Mats, a: int, e1: int, variants: list):
    """Diagonal on fiber position ``a``, variant chosen by external bit ``e1``."""
    v = [np.asarray(x, dtype=np.complex128) for x in variants]
    if all(np.all(x.imag == 0) for x in v):
        return rec(K_D1R, a=a, e1=e1, mat=mats.add_real(np.concatenate([x.real for x in v])))
    return rec(K_D1, a=a, e1=e1, mat=mats.add(*v))


def _scale(rec, mats: _Mats, e1: int, e2: int, vals):
    """Whole-fiber scalar chosen by external bits (index e1bit + 2*e2bit)."""
    vals = np.asarray(vals, dtype=np.complex128)
    if np.all(vals.imag == 0):
        return rec(K_SCALER, e1=e1, e2=e2, mat=mats.add_real(vals.real))
    return rec(K_SCALE, e1=e1, e2=e2, mat=mats.add(vals))


def _emit(op: HostOp, fib: dict, mats: _Mats) -> list:
    """Encode one host op given the group fiber map (state bit -> fiber index)."""
    rec = lambda kind, a=-1, b=-1, e1=-1, e2=-1, slot=-1, mat=-1: (kind, a, b, e1, e2, slot, mat, 0)
    if op.kind == "slot":
        return [rec(K_SLOT, a=fib[op.qubits[0]], slot=op.slot)]
    if op.kind == "u1":
        q = op.qubits[0]
        m = op.mat
        if _is_diag(m):
            d = np.diag(m)
            if q in fib:
                if np.all(d.imag == 0):
                    return [rec(K_D1R, a=fib[q], mat=mats.add_real(d.real))]
                return [rec(K_D1, a=fib[q], mat=mats.add(d))]
            return [_scale(rec, mats, q, -1, [d[0], d[1], d[0], d[1]])]
        if np.all(m.imag == 0):
            return [rec(K_U1R, a=fib[q], mat=mats.add_real(m.real.ravel()))]
        if np.all(np.diag(m).imag == 0) and m[0, 1].real == 0 and m[1, 0].real == 0:
            return [rec(K_U1X, a=fib[q], mat=mats.add_real([m[0, 0].real, m[0, 1].imag,
                                                            m[1, 0].imag, m[1, 1].real]))]
        return [rec(K_U1, a=fib[q], mat=mats.add(m))]
    # two-qubit
    q0, q1 = op.qubits
    m = op.mat
    diag = _diag_qubits(op)
    if _is_diag(m):
        d = np.diag(m)  # index b0 + 2 b1
        if q0 in fib and q1 in fib:
            a, b = fib[q0], fib[q1]
            if a > b:
                a, b, d = b, a, d[[0, 2, 1, 3]]
            if np.all(d.imag == 0):
                return [rec(K_D2R, a=a, b=b, mat=mats.add_real(d.real))]
            return [rec(K_D2, a=a, b=b, mat=mats.add(d))]
        if q0 in fib:  # q1 external: variants by b1
            return [_d1(rec, mats, fib[q0], q1, [d[[0, 1]], d[[2, 3]]])]
        if q1 in fib:  # q0 external: variants by b0
            return [_d1(rec, mats, fib[q1], q0, [d[[0, 2]], d[[1, 3]]])]
        # both external: scalar selected by (b0, b1) -> index e1bit + 2 e2bit
        return [_scale(rec, mats, q0, q1, d)]
    if q0 in diag or q1 in diag:
        c_pos = 0 if q0 in diag else 1
        ctrl, tgt = (q0, q1) if c_pos == 0 else (q1, q0)
        if ctrl in fib:
            a, b = fib[ctrl], fib[tgt]
            mm = m if c_pos == 0 else _swap_order4(m)  # now ctrl = first
            if _is_cx(mm):
                return [rec(K_CX, a=a, b=b)]
            if a > b:
                a, b, mm = b, a, _swap_order4(mm)
            return [rec(K_U2, a=a, b=b, mat=mats.add(mm))]
        m0, m1 = _block(m, c_pos, 0), _block(m, c_pos, 1)
        if _is_diag(m0) and _is_diag(m1):
            return [_d1(rec, mats, fib[tgt], ctrl, [np.diag(m0), np.diag(m1)])]
        return [rec(K_U1, a=fib[tgt], e1=ctrl, mat=mats.add(m0, m1))]
    a, b = fib[q0], fib[q1]
    if _is_swap(m):
        return [rec(K_SWAP, a=min(a, b), b=max(a, b))]
    mm = m
    if a > b:
        a, b, mm = b, a, _swap_order4(m)
    return [rec(K_U2, a=a, b=b, mat=mats.add(mm))]


def fiber_groups(ops: list) -> list:
    """Cut a pass's ops into fiber groups of <= FIBER_BITS non-diagonal qubits, with lookahead: a
    group takes, in program order, every op whose qubits it can hold and that depends on no op left
    behind (an op sharing a qubit with a skipped one is skipped too), so independent later ops join
    an earlier group instead of opening a new one. Each group costs an LDS round trip of the tile in
    the sweep kernels; ops on disjoint qubits commute, so the result is the same state (fp64
    rounding aside). Returns [(ops, needed qubits)] in execution order."""
    remaining = list(ops)
    out = []
    while remaining:
        need_all: set = set()
        taken, rest, blocked = [], [], set()
        for op in remaining:
            qs = set(op.qubits)
            need = op_need(op)
            if not (qs & blocked) and len(need_all | need) <= FIBER_BITS:
                need_all |= need
                taken.append(op)
            else:
                blocked |= qs
                rest.append(op)
        if not taken:  # cannot happen (the first remaining op always fits an empty fiber)
            raise RuntimeError("fiber grouping made no progress")
        out.append((taken, need_all))
        remaining = rest
    return out


def narrow_final_tile(prog: FragmentProgram, passes: list, final_tile_bits: int) -> None:
    """Shrink the FINAL pass's tile (in place) to ``final_tile_bits`` state bits when its
    non-diagonal and traced qubits fit: those plus the lowest other state bits. The pass then runs
    on more, smaller workgroups (per-program kernels: 2^(bits - 4) threads, 2^bits x 16 B of LDS),
    several per CU, so one workgroup's barrier and LDS phases overlap another's arithmetic instead of
    stalling the CU; its ops are the same (diagonal action on the bits that leave the tile comes from
    the tile index). syc 32 5: the FINAL passes need 6 and 9 of the 13 tile bits."""
    if len(passes) < 2 or prog.n <= TILE_BITS:
        return
    last = passes[-1]
    need = set(range(prog.m, prog.n))
    for op in last.ops:
        need |= op_need(op)
    if not (FIBER_BITS + 6 <= final_tile_bits < len(last.tile)) or len(need) > final_tile_bits:
        return
    tile = set(need)
    for q in range(prog.n):
        if len(tile) >= final_tile_bits:
            break
        tile.add(q)
    last.tile = sorted(tile)


def final_need_bits(prog: FragmentProgram, tile_bits: int) -> int:
    """State bits the FINAL pass's tile must hold (its non-diagonal and traced qubits), or
    ``tile_bits`` when the program has a single pass."""
    if prog.n <= TILE_BITS:
        return tile_bits
    prog = drop_trailing_phases(prog)
    passes = schedule_passes(prog, tile_bits)
    if len(passes) < 2:
        return tile_bits
    need = set(range(prog.m, prog.n))
    for op in passes[-1].ops:
        need |= op_need(op)
    return len(need)


def encode(prog: FragmentProgram, tile_bits: int = TILE_BITS, final_tile_bits: int | None = None) -> EncodedProgram:
    """``tile_bits`` (SPLIT programs only; PACKED programs always use 12-bit tiles): 12 for the
    interpreter kernel, 13 for per-program kernels (128 KiB LDS, 512 threads). ``final_tile_bits``
    (per-program kernels only): narrower FINAL-pass tile (:func:`narrow_final_tile`)."""
    prog = drop_trailing_phases(prog)
    n = prog.n
    packed = n <= TILE_BITS
    n_eff = max(n, FIBER_BITS) if packed else n
    if packed or tile_bits >= n:
        tile_bits = TILE_BITS
    passes = schedule_passes(prog, tile_bits)
    if final_tile_bits and not packed:
        narrow_final_tile(prog, passes, final_tile_bits)
    mats = _Mats()
    ops_out, groups_out, passes_out = [], [], []
    for pi, p in enumerate(passes):
        tile = list(range(n_eff)) if packed else p.tile
        local = {q: i for i, q in enumerate(tile)}  # state bit -> local position
        n_local = n_eff if packed else len(tile)
        g_begin = len(groups_out)
        for cur, cur_need in fiber_groups(p.ops):
            pos = sorted(local[q] for q in cur_need)
            for cand in range(n_local):  # pad the fiber to 4 positions
                if len(pos) >= FIBER_BITS:
                    break
                if cand not in pos:
                    pos.append(cand)
            pos = sorted(pos)
            fib = {tile[p_]: i for i, p_ in enumerate(pos)}
            ob = len(ops_out)
            for op in cur:
                ops_out.extend(_emit(op, fib, mats))
            groups_out.append((pos, ob, len(ops_out), (0, 0)))
        flags = (PASS_INIT if pi == 0 else 0) | (PASS_FINAL if pi == len(passes) - 1 else 0)
        traced = 0
        if flags & PASS_FINAL:
            for q in range(prog.m, n_eff):
                traced |= 1 << local[q]
        tile_mask = 0
        for q in tile:
            tile_mask |= 1 << q
        passes_out.append((tile_mask, g_begin, len(groups_out), flags, traced))
    ops_arr = np.array(ops_out, dtype=OP_DTYPE) if ops_out else np.zeros(0, OP_DTYPE)
    grp_arr = np.zeros(len(groups_out), GROUP_DTYPE)
    for i, (pos, ob, oe, _) in enumerate(groups_out):
        grp_arr[i]["pos"] = pos
        grp_arr[i]["op_begin"] = ob
        grp_arr[i]["op_end"] = oe
    pass_arr = np.array(passes_out, dtype=PASS_DTYPE)
    mat_arr = np.asarray(mats.buf if mats.buf else [0.0], dtype=np.float64)
    return EncodedProgram(n=n, n_eff=n_eff, m=prog.m, n_slots=prog.num_slots, packed=packed,
                          ops=ops_arr, groups=grp_arr, passes=pass_arr, mats=mat_arr,
                          n_host_ops=len(prog.ops), tile_bits=tile_bits)
