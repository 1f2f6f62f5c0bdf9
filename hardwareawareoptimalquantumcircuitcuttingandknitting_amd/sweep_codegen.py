"""Per-program sweep kernels: HIP source specialised to one encoded fragment program.

The interpreter kernel (``csrc/qknit.hip``, ``qk_sweep_pass_kernel``) executes an encoded
program (``sweep_plan.encode``) by loading every op descriptor and matrix at run time and
dispatching on its kind and fiber positions. For SPLIT programs (``n > 12``: the syc
fragments) that dispatch and the generic index arithmetic dominate: on syc 32 5 only 12% of
its VALU instructions are f64 FMAs and waves wait 49% of their time.

:func:`generate` emits, for each pass of a SPLIT program, one ``extern "C"`` kernel with the
same semantics as the interpreter on that pass — sparse INIT tile, known-zero state bits,
fiber groups, the FINAL trace over unmeasured qubits — but with the tile layout, the bit
deposits, the fiber positions, the op sequence and every gate matrix as compile-time
constants (hex float literals: exact). The per-op arithmetic is the interpreter's own
(``csrc/sweep_ops.h``, inlined into the source), so results agree with it. The source is
compiled at plan time with hiprtc (``qk_module_compile``) and run by ``qk_sweep_compiled``.
"""
from __future__ import annotations

import hashlib
import os
import re

from . import sweep_plan as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
OPS_HEADER = os.path.join(_HERE, "csrc", "sweep_ops.h")
PER = 16  # amplitudes per thread (4 fiber bits); threads per workgroup = 2^(tile_bits - 4)


def _prologue() -> str:
    """Compiler options line (qk_module_compile) and defines ahead of the inlined sweep_ops.h.

    The kernels only ever hold finite amplitudes and the sign of a zero never reaches a result
    (probabilities are |z|^2), so they are compiled with -fno-signed-zeros -ffinite-math-only:
    with those, 0 * x, x + 0 and fma(x, 0, y) fold, and the FINAL pass's first fiber — 14 of its
    16 amplitudes are known zeros of the sparse INIT tile on syc 32 5 — skips the ops on zeros
    (tools/sweep_isa.py). QKNIT_SWEEP_FOLD_ZEROS=0 compiles without (same results up to signed
    zeros)."""
    if os.environ.get("QKNIT_SWEEP_FOLD_ZEROS", "1") == "0":
        return ""
    return "// qk-options: -fno-signed-zeros -ffinite-math-only\n"


def _lit(x: float) -> str:
    x = float(x)
    return x.hex() if x != 0.0 else ("-0.0" if str(x).startswith("-") else "0.0")


def _deposit(src: str, src_bits: list, dst_bits: list) -> str:
    """Expression moving bit src_bits[i] of ``src`` to bit dst_bits[i] (runs merged)."""
    terms = []
    i = 0
    while i < len(src_bits):
        j = i
        while (j + 1 < len(src_bits) and src_bits[j + 1] == src_bits[j] + 1
               and dst_bits[j + 1] == dst_bits[j] + 1):
            j += 1
        width = j - i + 1
        mask = (1 << width) - 1
        sb, db = src_bits[i], dst_bits[i]
        terms.append(f"((({src}) >> {sb}) & 0x{mask:x}ull) << {db}")
        i = j + 1
    return "(" + " | ".join(terms) + ")" if terms else "0ull"


def _bits(mask: int) -> list:
    return [b for b in range(64) if (mask >> b) & 1]


def _swz(t: int) -> int:
    return t ^ (((t >> 4) ^ (t >> 8)) & 15)


def _lds_at(f: dict, r: int) -> str:
    """LDS index of a fiber's amplitude r: swz(base | cst) = swz(base) ^ swz(cst) — swz is linear over
    GF(2) and the base (thread bits) and cst (fiber positions) bits are disjoint — so the thread part
    is swizzled once per group (``sb``) and each access is one XOR with a constant (round 3: the
    per-access swizzle was ~20% of the FINAL pass's VALU instructions)."""
    c = int(f["cst"][r])
    # byte offsets (sbb = 16 sb): the XOR lands on the address itself, no shift per access
    off = f"(sbb ^ {16 * _swz(c)}u)" if c else "sbb"
    return f"*reinterpret_cast<double2*>(reinterpret_cast<char*>(lds) + {off})"


class _Emitter:
    def __init__(self):
        self.lines: list[str] = []

    def __call__(self, s: str = "", ind: int = 1) -> None:
        self.lines.append("    " * ind + s)


def _variant(vals: list, ebits: list, lit=None) -> list:
    """select_variant4 semantics: vals holds up to 4 variants of length N; ebits = [b1 expr or
    None, b2 expr or None]. Returns per-element C expressions (``lit`` formats a value)."""
    lit = lit or _lit
    b1, b2 = ebits
    N = len(vals[0])

    def pick(lo_v, hi_v, cond):
        return [f"({cond} ? {lit(h)} : {lit(l)})" if h != l else lit(l) for l, h in zip(lo_v, hi_v)]

    low = pick(vals[0], vals[1], b1) if b1 is not None else [lit(x) for x in vals[0]]
    if b2 is None:
        return low
    high = pick(vals[2], vals[3], b1) if b1 is not None else [lit(x) for x in vals[2]]
    return [f"({b2} ? {h} : {l})" if h != l else l for l, h in zip(low, high)][:N]


def _sign_lit(x: float) -> str:
    """+-1 as the XOR mask of the high dword of a double (sign flip: no multiply)."""
    return "0x80000000u" if x < 0 else "0u"


def _all_unit(vals: list) -> bool:
    return all(x in (1.0, -1.0) for v in vals for x in v)


# doubles of compile-time matrix data per op kind (variants included: see _emit_op)
def _op_values(op, mats) -> list:
    """Every compile-time matrix value an op reads (all variants), as floats; [] for ops without
    a compile-time matrix (slot matrices come per job at run time; CX / SWAP are permutations)."""
    kind, e1, e2, mat = int(op["kind"]), int(op["e1"]), int(op["e2"]), int(op["mat"])
    nvar = 2 if e1 >= 0 else 1
    size = {sp.K_U1: 8 * nvar, sp.K_D1: 4 * nvar, sp.K_U2: 32, sp.K_D2: 8, sp.K_U1R: 4, sp.K_U1X: 4,
            sp.K_D1R: 2 * nvar, sp.K_D2R: 4}.get(kind)
    if kind in (sp.K_SCALE, sp.K_SCALER):
        size = (2 if kind == sp.K_SCALE else 1) * (4 if e2 >= 0 else 2)
    if size is None:
        return []
    return [float(x) for x in mats[mat: mat + size]]


def op_scale(op, mats) -> float:
    """Positive scalar divided out of an op's compile-time matrix (all its variants alike, so the
    op times the scalar is the original op for every amplitude). The largest |entry| (complex
    modulus) becomes 1: the Sycamore / Hadamard-type gates (entries +-1/sqrt2, +-i/sqrt2) turn into
    +-1 / +-i entries whose multiplies the compiler folds away (x*1 = x, fma(1, a, b) = a + b are
    exact), and diagonal +-sqrt2 phases into sign flips. 1.0 for ops without a constant matrix."""
    vals = _op_values(op, mats)
    if not vals:
        return 1.0
    kind = int(op["kind"])
    if kind in (sp.K_U1, sp.K_D1, sp.K_U2, sp.K_D2, sp.K_SCALE):  # interleaved complex
        mags = [abs(complex(vals[i], vals[i + 1])) for i in range(0, len(vals), 2)]
    else:  # real entries (U1X: [m00, Im m01, Im m10, m11], each one an entry's modulus)
        mags = [abs(v) for v in vals]
    c = max(mags)
    return c if c > 0 else 1.0


SNAP = 4e-16  # normalised entries this close to 0 / +-1 are those values (cos/sin(pi/4) differ by an ulp)


def _snap(x: float) -> float:
    """Normalised matrix entry, snapped to an exact 0 or +-1 within SNAP (a relative change of
    < 4e-16 of the entry, below fp64 rounding of the op itself) so its multiply folds away."""
    for t in (0.0, 1.0, -1.0):
        if abs(x - t) <= SNAP:
            return t
    return x


def program_scale(enc) -> float:
    """Product of :func:`op_scale` over every op of every pass: the true amplitudes are this times
    the ones the normalised kernels compute (probabilities: its square)."""
    out = 1.0
    for op in enc.ops:
        out *= op_scale(op, enc.mats)
    return out


def _emit_op(e: _Emitter, op, mats, ext, n_slots: int) -> None:
    kind, a, b, e1, e2, slot, mat = (int(op["kind"]), int(op["a"]), int(op["b"]), int(op["e1"]),
                                     int(op["e2"]), int(op["slot"]), int(op["mat"]))
    b1 = ext(e1) if e1 >= 0 else None
    b2 = ext(e2) if e2 >= 0 else None
    inv = 1.0 / op_scale(op, mats)

    def arr(n, off=0):
        return [_snap(float(x) * inv) for x in mats[mat + off: mat + off + n]]

    def const_arr(name, exprs):
        e(f"const double {name}[{len(exprs)}] = {{{', '.join(exprs)}}};", 2)

    e("{", 1)
    if kind == sp.K_U1:
        vals = [arr(8), arr(8, 8)] if b1 is not None else [arr(8)]
        const_arr("m", _variant(vals, [b1, None]))
        e(f"ap_u1<{a}>(v, m);", 2)
    elif kind == sp.K_D1:
        vals = [arr(4), arr(4, 4)] if b1 is not None else [arr(4)]
        const_arr("d", _variant(vals, [b1, None]))
        e(f"ap_d1<{a}>(v, d);", 2)
    elif kind == sp.K_SLOT:
        e(f"ap_u1<{a}>(v, job_slots + (job * {n_slots} + {slot}) * 8);", 2)
    elif kind == sp.K_U2:
        const_arr("m", [_lit(x) for x in arr(32)])
        e(f"ap_u2<{a}, {b}>(v, m);", 2)
    elif kind == sp.K_D2:
        const_arr("d", [_lit(x) for x in arr(8)])
        e(f"ap_d2<{a}, {b}>(v, d);", 2)
    elif kind == sp.K_CX:
        e(f"ap_cx<{a}, {b}>(v);", 2)
    elif kind == sp.K_SWAP:
        e(f"ap_swap<{a}, {b}>(v);", 2)
    elif kind in (sp.K_SCALE, sp.K_SCALER):
        N = 2 if kind == sp.K_SCALE else 1
        nv = 4 if b2 is not None else 2 if b1 is not None else 1
        # select_variant4 reads p[0:2N) for the b1 pair and p[2N:4N) when h2
        vals = [arr(N, k * N) for k in range(4)] if b2 is not None else [arr(N, k * N) for k in range(2)]
        if b1 is None:  # variant pair collapses to its first entry
            vals = [vals[0], vals[0]] + ([vals[2], vals[2]] if b2 is not None else [])
        del nv
        s = _variant(vals, [b1, b2])
        if kind == sp.K_SCALE:
            e(f"const double sr = {s[0]}, si = {s[1]};", 2)
            e("#pragma unroll", 0)
            e(f"for (int r = 0; r < {PER}; ++r) v[r] = cmul(sr, si, v[r]);", 2)
        elif _all_unit(vals):  # +-1 chosen by external bits: flip the sign bits
            e(f"const unsigned sg = {_variant(vals, [b1, b2], _sign_lit)[0]};", 2)
            e("#pragma unroll", 0)
            e(f"for (int r = 0; r < {PER}; ++r) v[r] = flip_sign(v[r], sg);", 2)
        else:
            e(f"const double sr = {s[0]};", 2)
            e("#pragma unroll", 0)
            e(f"for (int r = 0; r < {PER}; ++r) v[r] = make_double2(sr * v[r].x, sr * v[r].y);", 2)
    elif kind == sp.K_U1R:
        const_arr("m", [_lit(x) for x in arr(4)])
        e(f"ap_u1r<{a}>(v, m);", 2)
    elif kind == sp.K_U1X:
        const_arr("m", [_lit(x) for x in arr(4)])
        e(f"ap_u1x<{a}>(v, m);", 2)
    elif kind == sp.K_D1R:
        vals = [arr(2), arr(2, 2)] if b1 is not None else [arr(2)]
        if _all_unit(vals):  # diag(+-1, +-1): sign flips, selected by the external bit
            sg = _variant(vals, [b1, None], _sign_lit)
            e(f"const unsigned sg0 = {sg[0]}, sg1 = {sg[1]};", 2)
            e(f"ap_d1s<{a}>(v, sg0, sg1);", 2)
        else:
            const_arr("d", _variant(vals, [b1, None]))
            e(f"ap_d1r<{a}>(v, d);", 2)
    elif kind == sp.K_D2R:
        const_arr("d", [_lit(x) for x in arr(4)])
        e(f"ap_d2r<{a}, {b}>(v, d);", 2)
    else:
        raise ValueError(f"unknown op kind {kind}")
    e("}", 1)


def _pass_kernel(enc: sp.EncodedProgram, ip: int, name: str, device_fn: bool = False) -> list:
    """Pass ``ip`` of ``enc`` as an ``extern "C"`` kernel, or (``device_fn``) as a device function
    of the workgroup's block index within the pass and the shared tile (multi-fragment launches)."""
    n, m = enc.n, enc.m
    TB = enc.pass_tile_bits(ip)
    NT = 1 << (TB - 4)
    P = len(enc.passes)
    ps = enc.passes[ip]
    flags = int(ps["flags"])
    init, final = bool(flags & sp.PASS_INIT), bool(flags & sp.PASS_FINAL)
    tile_mask = int(ps["tile_mask"])
    bitpos = _bits(tile_mask)
    assert len(bitpos) == TB
    nmask = (1 << n) - 1
    outside = _bits(nmask & ~tile_mask)
    init_sparse = ip == 0 and P > 1
    zero_mask = (nmask & ~int(enc.passes[0]["tile_mask"])) if ip == 1 else 0
    tpj_log = 0 if init_sparse else n - TB
    traced = int(ps["traced_local"])
    mmask = (1 << m) - 1
    hi = [sum(((i >> k) & 1) << bitpos[TB - 4 + k] for k in range(4)) for i in range(PER)]

    e = _Emitter()
    if device_fn:
        e(f"__device__ __forceinline__ void {name}(double2* __restrict__ lds, const unsigned blk,", 0)
    else:
        e(f'extern "C" __global__ __launch_bounds__({NT}) void {name}(', 0)
    e("const double* __restrict__ job_slots, const double* __restrict__ job_sign,", 2)
    e("double2* __restrict__ state, double* __restrict__ pjob, long long n_jobs,", 2)
    e("const long long* __restrict__ label_off" + (", const int* __restrict__ pfx) {" if device_fn else ") {"), 2)
    e("using namespace qk_sweep_ops;")
    if not device_fn:
        e("const int* pfx = nullptr;")
        e(f"__shared__ double2 lds[{1 << TB}];")
        e("const unsigned blk = blockIdx.x;")
    e("const unsigned tid = threadIdx.x;")
    # FINAL: grp is a label when label_off is given (its branch jobs are summed in registers,
    # qk_sweep_compiled_labels), else a job
    e(f"const long long grp = (long long)(blk >> {tpj_log});")
    if tpj_log:
        e(f"const unsigned long long tj = blk & {(1 << tpj_log) - 1}u;")
        e(f"const unsigned long long tbase = {_deposit('tj', list(range(len(outside))), outside)};")
    else:
        e("const unsigned long long tbase = 0ull;")
    e(f"const unsigned long long lo = {_deposit('(unsigned long long)tid', list(range(TB - 4)), bitpos[:TB - 4])};")
    e("(void)n_jobs; (void)job_slots; (void)lo; (void)label_off; (void)pfx;")
    keep = [i for i in range(PER) if not ((NT * i) & traced)]
    gids = list(range(int(ps["group_begin"]), int(ps["group_end"])))
    zero_tile = init and not init_sparse and tpj_log > 0
    if zero_tile and not final:
        raise ValueError("SPLIT INIT pass that is not FINAL must be sparse")
    # direct form: the first group's fiber comes straight from HBM (or the |0..0> start) into registers
    # and the last group's fiber goes straight to HBM (or into the FINAL pass's per-thread probability
    # sums, at that fiber's positions): two LDS round trips and two barriers fewer per (job, tile) than
    # staging the whole tile through LDS at both ends. Not for FINAL passes that trace qubits out (the
    # trace sums amplitudes across threads) or passes without groups.
    if gids and not (final and traced):
        return _pass_body_direct(e, enc, ps, gids, TB, NT, n, m, bitpos, init, final, zero_tile, zero_mask)
    if final:
        e("long long j0 = grp, j1 = grp + 1;")
        e("if (label_off) { j0 = label_off[grp]; j1 = label_off[grp + 1]; }")
        for i in keep:
            e(f"double out{i} = 0.0;")
        e("for (long long job = j0; job < j1; ++job) {")
    else:
        e("const long long job = grp;")
    e(_state_ptr(enc, ps))
    e("(void)st;")
    if init:
        e("lds[swz(tid)] = make_double2((tid == 0 && tbase == 0ull) ? 1.0 : 0.0, 0.0);")
        for i in range(1, PER):
            e(f"lds[swz(tid + {NT * i})] = make_double2(0.0, 0.0);")
    else:
        for i in range(PER):
            s = f"(tbase | lo | 0x{hi[i]:x}ull)"
            if zero_mask:
                e(f"{{ const unsigned long long s = {s}; lds[swz(tid + {NT * i})] = "
                  f"(s & 0x{zero_mask:x}ull) ? make_double2(0.0, 0.0) : st[s]; }}")
            else:
                e(f"lds[swz(tid + {NT * i})] = st[{s}];")
    e("__syncthreads();")
    if zero_tile:
        e("if (tbase == 0ull) {")
    for gi in gids:
        f = _fiber(enc, gi, TB, bitpos)
        e("{")
        e(f"const unsigned sbb = 16u * swz({f['base']});", 2)
        e("double2 v[16];", 2)
        for r in range(PER):
            e(f"v[{r}] = {_lds_at(f, r)};", 2)
        _emit_group_ops(e, enc, gi, f, bitpos)
        for r in range(PER):
            e(f"{_lds_at(f, r)} = v[{r}];", 2)
        e("__syncthreads();", 2)
        e("}")
    if zero_tile:
        e("}")
    if final:
        subs = []
        sub = 0
        while True:
            subs.append(sub)
            sub = (sub - traced) & traced
            if sub == 0:
                break
        # the ops ran with op_scale divided out: probabilities carry program_scale^2
        e(f"const double sgn = job_sign[job] * {_lit(program_scale(enc) ** 2)};")
        cond = traced & (NT - 1)
        for i in keep:
            e(f"if (!(tid & {cond}u)) {{" if cond else "{")
            e("double acc = 0.0;", 2)
            for sb in subs:
                e(f"{{ const double2 z = lds[swz((tid + {NT * i}) | {sb}u)]; "
                  f"acc = fma(z.x, z.x, fma(z.y, z.y, acc)); }}", 2)
            e(f"out{i} += sgn * acc;", 2)
            e("}")
        e("__syncthreads();  // the next branch job of the label reuses the tile")
        e("}")
        for i in keep:
            e(f"if (!(tid & {cond}u)) {{" if cond else "{")
            e(f"const unsigned long long x = (tbase | lo | 0x{hi[i]:x}ull) & 0x{mmask:x}ull;", 2)
            e(f"pjob[(grp << {m}) + (long long)x] = out{i};", 2)
            e("}")
    else:
        for i in range(PER):
            e(f"st[tbase | lo | 0x{hi[i]:x}ull] = lds[swz(tid + {NT * i})];")
    e("}", 0)
    return e.lines


def _state_ptr(enc, ps) -> str:
    """Job state of a pass: the FINAL pass of a two-pass program may start from a shared INIT
    prefix's state (``pfx``: job -> prefix slot, qk_sweep_compiled_multi_shared)."""
    n = enc.n
    if len(enc.passes) == 2 and bool(int(ps["flags"]) & sp.PASS_FINAL):
        return f"double2* st = state + (pfx ? (long long)pfx[job] : job) * {1 << n}ll;"
    return f"double2* st = state + job * {1 << n}ll;"


def _fiber(enc, gi: int, TB: int, bitpos: list) -> dict:
    """Layout of group ``gi``'s fiber: tile positions (``pos``), the thread's base tile position
    (``base`` expression of tid), per-register offsets (``cst``), and the same in state bits:
    ``lo`` (expression of tid) and ``hi`` (constants), so amplitude r sits at state index
    ``tbase | lo | hi[r]``."""
    pos = [int(x) for x in enc.groups[gi]["pos"]]
    return _layout(pos, [p for p in range(TB) if p not in pos], TB, bitpos)


def _layout(pos: list, nonfib: list, TB: int, bitpos: list) -> dict:
    """A register / lane layout of the tile: register bit k holds tile position ``pos[k]``, thread-index
    bit j tile position ``nonfib[j]`` (any order: a cross-lane exchange leaves the lanes permuted)."""
    return {
        "pos": pos,
        "nonfib": nonfib,
        "base": _deposit("tid", list(range(TB - 4)), nonfib),
        "cst": [sum(((r >> k) & 1) << pos[k] for k in range(4)) for r in range(PER)],
        "lo": _deposit("(unsigned long long)tid", list(range(TB - 4)), [bitpos[p] for p in nonfib]),
        "hi": [sum(((r >> k) & 1) << bitpos[pos[k]] for k in range(4)) for r in range(PER)],
    }


_ONE_Q = (sp.K_U1, sp.K_D1, sp.K_SLOT, sp.K_U1R, sp.K_U1X, sp.K_D1R)
_TWO_Q = (sp.K_U2, sp.K_D2, sp.K_CX, sp.K_SWAP, sp.K_D2R)


def _group_used(enc, gi: int) -> list:
    """Tile positions the ops of group ``gi`` act on (a group's fiber may hold unused positions)."""
    gpos = [int(x) for x in enc.groups[gi]["pos"]]
    used = []
    gr = enc.groups[gi]
    for oi in range(int(gr["op_begin"]), int(gr["op_end"])):
        op = enc.ops[oi]
        kind = int(op["kind"])
        idx = [int(op["a"])] if kind in _ONE_Q else [int(op["a"]), int(op["b"])] if kind in _TWO_Q else []
        for a in idx:
            if gpos[a] not in used:
                used.append(gpos[a])
    return used


def _group_ext_positions(enc, gi: int, bitpos: list) -> set:
    """Tile positions of the state bits that select the variants of group ``gi``'s ops (e1 / e2):
    they must stay thread bits (a register bit would make the op's matrix differ per register)."""
    out = set()
    gr = enc.groups[gi]
    for oi in range(int(gr["op_begin"]), int(gr["op_end"])):
        for fld in ("e1", "e2"):
            eb = int(enc.ops[oi][fld])
            if eb >= 0 and eb in bitpos:
                out.add(bitpos.index(eb))
    return out


def lane_exchange_mode() -> int:
    """QKNIT_SWEEP_LANE_XCHG: 0 = every fiber-group boundary through LDS (round 5's kernels); 1 = lane
    bits 4 / 5 by permlane swaps where at most two positions change (default); 2 = also the other lane
    bits of a single-wave tile (shuffles), so that FINAL passes never touch LDS. Same box, interleaved,
    bit-identical rows (profiles/r06f_sweep_ab_variants.json): bench-plan sweep 0.0482 / 0.0474 / 0.0505
    ms and full sweep 0.349 / 0.347 / 0.351 ms for modes 0 / 1 / 2 — the shuffles for lane bits 0-3 cost
    three selects per dword and their LDS-free FINAL pass gains nothing: it is VALU-issue bound."""
    return int(os.environ.get("QKNIT_SWEEP_LANE_XCHG", "1"))


def opaque_tid() -> bool:
    """QKNIT_SWEEP_OPAQUE_TID=1: the FINAL pass's branch-job loop takes the thread index through an
    opaque zero (172 -> 128 VGPRs on syc 32 5). Measured and not the default: the sweep took 0.0483 vs
    0.0474 ms (bench plan) and 0.354 vs 0.347 ms (full plan) — recomputing the index arithmetic per job
    costs more than the occupancy gains (profiles/r06f_sweep_ab_variants.json)."""
    return os.environ.get("QKNIT_SWEEP_OPAQUE_TID", "0") == "1"


def lane_exchange_enabled() -> bool:
    return lane_exchange_mode() != 0


def _plan_layouts(enc, gids: list, TB: int, bitpos: list, final: bool = False) -> tuple:
    """Per group of a direct-form pass: its register / lane layout and how it is reached from the
    previous group's — ``"lds"`` (the tile's round trip through LDS, any layout) or a list of
    ``(register bit, lane bit)`` cross-lane exchanges (sweep_ops.h ``xchg_lane_bit_any``). Mode 1: an
    exchange applies when the group's ops need at most two tile positions that are not in the
    previous fiber and those sit on thread bits 4 / 5 (the previous layout's lane order is chosen so
    they do, unless it came from an exchange itself): the wavefront butterfly of a 1-2-bit boundary
    (syc 32 5: the last group of each FINAL pass touches two new qubits). Mode 2, FINAL passes of
    single-wave tiles: any lane bit (bits 4 / 5 preferred), up to four positions, so the pass needs
    no LDS."""
    mode = lane_exchange_mode()
    general = mode >= 2 and final and TB - 4 == 6
    fast = (5, 4)  # lane bits the permlane swaps reach
    layouts = [_fiber(enc, gids[0], TB, bitpos)]
    trans = [None]
    free = [True]  # whether the layout's lane order may still be chosen (not fixed by an exchange)
    for k in range(1, len(gids)):
        cur = layouts[-1]
        used = _group_used(enc, gids[k])
        need = [p for p in used if p not in cur["pos"]]
        ok = mode >= 1 and TB - 4 >= 6 and 0 < len(need) <= (4 if general else 2) and len(used) <= 4
        on_fast = lambda lay: [p for p in need if lay["nonfib"].index(p) in fast]  # noqa: E731
        if ok and len(on_fast(cur)) < min(len(need), 2) and free[-1]:
            # put the needed positions on thread bits 5, 4 (then 3, 2, 1, 0), the rest ascending
            slots = list(fast) + [3, 2, 1, 0]
            order = [None] * len(cur["nonfib"])
            for p, t in zip(need, slots):
                order[t] = p
            rest = iter(p for p in sorted(cur["nonfib"]) if p not in need)
            order = [p if p is not None else next(rest) for p in order]
            cur = _layout(cur["pos"], order, TB, bitpos)
            layouts[-1] = cur
        if ok and not general and len(on_fast(cur)) < len(need):
            ok = False
        if not ok:
            layouts.append(_fiber(enc, gids[k], TB, bitpos))
            trans.append("lds")
            free.append(True)
            continue
        pos, nonfib = list(cur["pos"]), list(cur["nonfib"])
        ext = _group_ext_positions(enc, gids[k], bitpos)
        # evict variant-selecting positions first: they must end on thread bits
        evict = sorted((i for i in range(4) if pos[i] not in used), key=lambda i: pos[i] not in ext)
        steps = []
        for p in need:
            t = nonfib.index(p)
            i = evict.pop(0)
            steps.append((i, t))
            pos[i], nonfib[t] = p, pos[i]
        if ext & set(pos):
            layouts.append(_fiber(enc, gids[k], TB, bitpos))
            trans.append("lds")
            free.append(True)
            continue
        layouts.append(_layout(pos, nonfib, TB, bitpos))
        trans.append(steps)
        free.append(False)
    return layouts, trans


def _emit_group_ops(e: _Emitter, enc, gi: int, f: dict, bitpos: list) -> None:
    nonfib = f["nonfib"]
    gpos = [int(x) for x in enc.groups[gi]["pos"]]
    remap = None if list(f["pos"]) == gpos else [f["pos"].index(p) if p in f["pos"] else -1 for p in gpos]

    def ext(ebit):
        if ebit in bitpos:
            j = bitpos.index(ebit)
            if j not in nonfib:  # a fiber position: the base has it cleared
                return "false"
            return f"((tid >> {nonfib.index(j)}) & 1u)"
        return f"((tbase >> {ebit}) & 1ull)"

    gr = enc.groups[gi]
    for oi in range(int(gr["op_begin"]), int(gr["op_end"])):
        op = enc.ops[oi]
        if remap is not None:  # the group runs in an exchanged layout: its fiber indices move
            op = op.copy()
            kind = int(op["kind"])
            for fld in ("a",) if kind in _ONE_Q else ("a", "b") if kind in _TWO_Q else ():
                op[fld] = remap[int(op[fld])]
                assert op[fld] >= 0
        _emit_op(e, op, enc.mats, ext, enc.n_slots)


def _pass_body_direct(e: _Emitter, enc, ps, gids: list, TB: int, NT: int, n: int, m: int, bitpos: list,
                      init: bool, final: bool, zero_tile: bool, zero_mask: int) -> list:
    """Body of a pass kernel in the direct form (see _pass_kernel)."""
    lays, trans = _plan_layouts(enc, gids, TB, bitpos, final=final)
    first, last = lays[0], lays[-1]
    uses_lds = any(t == "lds" for t in trans)
    mmask = (1 << m) - 1
    if final:
        e(f"const unsigned long long xlo = (tbase | {last['lo']}) & 0x{mmask:x}ull;")
        for r in range(PER):
            e(f"double out{r} = 0.0;")
        e("long long j0 = grp, j1 = grp + 1;")
        e("if (label_off) { j0 = label_off[grp]; j1 = label_off[grp + 1]; }")
        e("for (long long job = j0; job < j1; ++job) {")
    else:
        e("const long long job = grp;")
    loop_start = len(e.lines)
    e(_state_ptr(enc, ps))
    e("(void)st;")
    e("double2 v[16];")
    if init:  # |0..0>: amplitude 1 at tile position 0 = register 0 of thread 0 (of the tbase == 0 tile)
        e("v[0] = make_double2((tid == 0 && tbase == 0ull) ? 1.0 : 0.0, 0.0);")
        for r in range(1, PER):
            e(f"v[{r}] = make_double2(0.0, 0.0);")
    else:
        e(f"const unsigned long long slo = tbase | {first['lo']};")
        for r in range(PER):
            if zero_mask:
                e(f"{{ const unsigned long long s = slo | 0x{first['hi'][r]:x}ull; "
                  f"v[{r}] = (s & 0x{zero_mask:x}ull) ? make_double2(0.0, 0.0) : st[s]; }}")
            else:
                e(f"v[{r}] = st[slo | 0x{first['hi'][r]:x}ull];")
    if zero_tile:
        e("if (tbase == 0ull) {")
    for k, gi in enumerate(gids):
        f = lays[k]
        e("{")
        if k > 0 and trans[k] == "lds":
            e(f"const unsigned sbb = 16u * swz({f['base']});", 2)
            for r in range(PER):
                e(f"v[{r}] = {_lds_at(f, r)};", 2)
        elif k > 0:  # cross-lane butterfly: register bit i <-> lane bit t
            for i, t in trans[k]:
                e(f"xchg_lane_bit_any<{i}, {t}>(v);", 2)
        _emit_group_ops(e, enc, gi, f, bitpos)
        if k < len(gids) - 1 and trans[k + 1] == "lds":
            if k == 0 or trans[k] != "lds":
                e(f"const unsigned sbb = 16u * swz({f['base']});", 2)
            for r in range(PER):
                e(f"{_lds_at(f, r)} = v[{r}];", 2)
            e("__syncthreads();", 2)
        e("}")
    if zero_tile:
        e("}")
    if final:
        # the ops ran with op_scale divided out: probabilities carry program_scale^2
        e(f"const double sgn = job_sign[job] * {_lit(program_scale(enc) ** 2)};")
        for r in range(PER):
            e(f"out{r} = fma(sgn, fma(v[{r}].x, v[{r}].x, v[{r}].y * v[{r}].y), out{r});")
        if uses_lds:
            e("__syncthreads();  // the next branch job's first LDS writes follow this job's last reads")
        if opaque_tid():
            # the thread index enters each branch job through an opaque zero, so the compiler cannot
            # hoist the job's index arithmetic out of the loop and keep it live across the whole body
            # (the FINAL multi kernel of syc 32 5: 172 -> 128 VGPRs, tools/sweep_vgpr.py)
            e.lines[loop_start:] = [re.sub(r"\btid\b", "tidq", ln) for ln in e.lines[loop_start:]]
            e.lines.insert(loop_start, "    unsigned qz; asm volatile(\"v_mov_b32 %0, 0\" : \"=v\"(qz)); "
                                       "const unsigned tidq = tid + qz;")
        e("}")
        for r in range(PER):
            e(f"pjob[(grp << {m}) + (long long)(xlo | 0x{last['hi'][r] & mmask:x}ull)] = out{r};")
    else:
        e(f"const unsigned long long slo2 = tbase | {last['lo']};")
        for r in range(PER):
            e(f"st[slo2 | 0x{last['hi'][r]:x}ull] = v[{r}];")
    e("}", 0)
    return e.lines


def generate(enc: sp.EncodedProgram) -> tuple[str, list]:
    """HIP source (sweep_ops.h inlined) and kernel names, one kernel per pass."""
    if enc.packed:
        raise ValueError("per-program kernels are generated for SPLIT programs (n > 12) only")
    body = []
    names = []
    key = hashlib.sha1(enc.ops.tobytes() + enc.groups.tobytes() + enc.passes.tobytes()
                       + enc.mats.tobytes() + bytes([enc.n, enc.m, enc.n_slots])).hexdigest()[:12]
    for ip in range(len(enc.passes)):
        name = f"qk_sweep_{key}_p{ip}"
        names.append(name)
        body += _pass_kernel(enc, ip, name) + [""]
    src = _prologue() + open(OPS_HEADER).read() + "\n" + "\n".join(body) + "\n"
    return src, names


MULTI_MAX = 4  # fragments per multi-fragment launch (qknit_jit.hip QK_MULTI_MAX)
_MULTI_STRUCT = """struct qk_multi_args {
    const double* slots[4];
    const double* sign[4];
    void* state[4];
    double* out[4];
    const long long* label_off[4];
    long long n_jobs[4];
    long long begin[4];
    long long end[4];
    const unsigned long long* map;
    const double* islots[4];
    const int* pfx[4];
};
"""


def generate_multi(encs: list) -> tuple[str, list]:
    """Several SPLIT programs of one tile width swept together: one kernel per pass round ``r``,
    in which fragment ``f`` (if it has a pass ``r``) owns the blocks ``[begin[f], end[f])`` and runs
    its pass ``r`` body on them (``qk_sweep_compiled_multi``). Independent fragments then share
    each launch instead of queueing behind each other."""
    if not 1 <= len(encs) <= MULTI_MAX:
        raise ValueError(f"1..{MULTI_MAX} programs per multi-fragment module")
    if any(e.packed for e in encs):
        raise ValueError("multi-fragment kernels need SPLIT programs")
    for r in range(max(len(e.passes) for e in encs)):
        if len({e.pass_tile_bits(r) for e in encs if len(e.passes) > r}) != 1:
            raise ValueError("multi-fragment kernels need one tile width per pass round")
    h = hashlib.sha1()
    for e in encs:
        h.update(e.ops.tobytes() + e.groups.tobytes() + e.passes.tobytes() + e.mats.tobytes()
                 + bytes([e.n, e.m, e.n_slots]))
    key = h.hexdigest()[:12]
    body, names = [_MULTI_STRUCT], []
    shares = [len(e.passes) == 2 for e in encs]
    for r in range(max(len(e.passes) for e in encs)):
        members = [f for f, e in enumerate(encs) if len(e.passes) > r]
        for f in members:
            body += _pass_kernel(encs[f], r, f"qk_mb_{key}_f{f}_p{r}", device_fn=True) + [""]
        name = f"qk_sweepm_{key}_r{r}"
        names.append(name)
        tb = encs[members[0]].pass_tile_bits(r)
        # QKNIT_SWEEP_WAVES_PER_EU: minimum waves per SIMD the compiler must fit (register budget)
        wpe = os.environ.get("QKNIT_SWEEP_WAVES_PER_EU")
        lb = f"{1 << (tb - 4)}, {int(wpe)}" if wpe else f"{1 << (tb - 4)}"
        body.append(f'extern "C" __global__ __launch_bounds__({lb}) void {name}(qk_multi_args a) {{')
        body.append(f"    __shared__ double2 lds[{1 << tb}];")
        body.append("    const long long b = blockIdx.x;")
        # caller-ordered blocks (qk_sweep_compiled_multi block_maps): program << 56 | block in its range;
        # otherwise the programs' block ranges in order
        body.append("    int f = -1;")
        body.append("    long long lb = 0;")
        body.append("    if (a.map) {")
        body.append("        const unsigned long long m = a.map[b];")
        body.append("        f = (int)(m >> 56);")
        body.append("        lb = (long long)(m & 0x00ffffffffffffffull);")
        body.append("    } else {")
        for f in members:
            body.append(f"        if (b >= a.begin[{f}] && b < a.end[{f}]) {{ f = {f}; lb = b - a.begin[{f}]; }}")
        body.append("    }")
        for f in members:
            body.append(f"    if (f == {f} && lb >= 0 && lb < a.end[{f}] - a.begin[{f}]) {{")
            # shared INIT prefixes (qk_sweep_compiled_multi_shared): the INIT round reads the prefixes'
            # slot rows, the FINAL round of a two-pass program maps each job to its prefix's state
            slots = f"(a.islots[{f}] ? a.islots[{f}] : a.slots[{f}])" if (r == 0 and shares[f]) else f"a.slots[{f}]"
            pfx = f"a.pfx[{f}]" if (r == 1 and shares[f]) else "nullptr"
            body.append(f"        qk_mb_{key}_f{f}_p{r}(lds, (unsigned)lb, {slots}, a.sign[{f}],")
            body.append(f"            (double2*)a.state[{f}], a.out[{f}], a.n_jobs[{f}], a.label_off[{f}], {pfx});")
            body.append("        return;")
            body.append("    }")
        body.append("}")
        body.append("")
    src = _prologue() + open(OPS_HEADER).read() + "\n" + "\n".join(body) + "\n"
    return src, names
