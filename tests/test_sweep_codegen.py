"""Cross-lane butterflies of the per-program sweep kernels (sweep_codegen._plan_layouts, sweep_ops.h
xchg_lane_bit): a CPU model of where every amplitude of a tile sits — (thread, register) -> tile
position — run through each pass's layout transitions (an LDS round trip re-gathers by the next
layout; an exchange applies the v_permlane16_swap / v_permlane32_swap semantics to register pairs),
checked against the layout the generator then uses for the group's ops and the final stores. The
arithmetic itself is checked on the GPU against the interpreter and the oracle (test_gpu.py)."""
import numpy as np
import pytest

from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, cutting, engine
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import sweep_codegen as sc
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import sweep_plan as sp


def _where(lay: dict, TB: int) -> np.ndarray:
    """[threads, 16] tile position held by (thread, register) in a layout."""
    nt = 1 << (TB - 4)
    out = np.zeros((nt, 16), dtype=np.int64)
    for t in range(nt):
        base = sum(((t >> j) & 1) << p for j, p in enumerate(lay["nonfib"]))
        for r in range(16):
            out[t, r] = base | sum(((r >> k) & 1) << p for k, p in enumerate(lay["pos"]))
    return out


def _permlane_swap(A: np.ndarray, B: np.ndarray, bit: int):
    """v_permlane{16,32}_swap on one register pair, per 64-lane wave: lanes with lane bit ``bit`` set
    of A trade with the lanes of B that have it clear (same other bits)."""
    A, B = A.copy(), B.copy()
    for lane in range(A.shape[0]):
        if (lane & 63) >> bit & 1:
            lo = lane - (1 << bit)
            A[lane], B[lo] = B[lo], A[lane]
    return A, B


def _programs():
    out = []
    for key in ("syc_32_5_p2", "syc_32_1_p2", "syc_32_1_p2_forced", "qft_16_1_p3"):
        name, n, d, p, var = cutting.BASELINE_CONFIGS[key]
        cut = cutting.config_cut_circuit(name, n, d, p, var)[1]
        for fs in engine.prepare_fragments(VirtualCircuit(cut), upload=False, basis=True):
            want, tb, ftb = fs.jit
            if fs.prog.n <= 12:
                continue
            dprog = engine._device_program(fs.prog)[0]
            out.append((key, sp.encode(dprog, tile_bits=tb, final_tile_bits=ftb)))
    return out


@pytest.mark.parametrize("lane_xchg", ["2", "1", "0"])
def test_lane_exchange_layouts_track_every_amplitude(monkeypatch, lane_xchg):
    monkeypatch.setenv("QKNIT_SWEEP_LANE_XCHG", lane_xchg)
    exchanges = 0
    final_lds = 0
    for key, enc in _programs():
        for ip, ps in enumerate(enc.passes):
            TB = enc.pass_tile_bits(ip)
            bitpos = sc._bits(int(ps["tile_mask"]))
            gids = list(range(int(ps["group_begin"]), int(ps["group_end"])))
            if not gids:
                continue
            final = bool(int(ps["flags"]) & sp.PASS_FINAL)
            lays, trans = sc._plan_layouts(enc, gids, TB, bitpos, final=final)
            if final and TB == 10:
                final_lds += sum(t == "lds" for t in trans)
            held = _where(lays[0], TB)
            for k, gi in enumerate(gids):
                if k > 0 and trans[k] == "lds":
                    held = _where(lays[k], TB)  # written by the previous layout, read by this one
                elif k > 0:
                    for i, t in trans[k]:
                        exchanges += 1
                        for r in range(16):
                            if not r >> i & 1:
                                held[:, r], held[:, r | 1 << i] = _permlane_swap(held[:, r], held[:, r | 1 << i], t)
                np.testing.assert_array_equal(held, _where(lays[k], TB), err_msg=f"{key} pass {ip} group {gi}")
                # the group's ops act on register bits, their variant bits on thread bits
                assert set(sc._group_used(enc, gi)) <= set(lays[k]["pos"])
                assert not sc._group_ext_positions(enc, gi, bitpos) & set(lays[k]["pos"])
                # a layout is a bijection onto the tile
                assert sorted(lays[k]["pos"] + lays[k]["nonfib"]) == list(range(TB))
    if lane_xchg == "2":
        assert final_lds == 0  # no FINAL pass of a 10-bit tile touches LDS
    if lane_xchg == "1":
        assert exchanges >= 4  # syc 32 5: both FINAL passes end in a two-bit butterfly
    if lane_xchg == "0":
        assert exchanges == 0


def test_generated_kernels_use_lane_exchanges_only_when_enabled(monkeypatch):
    key, enc = _programs()[0]
    src_on, _ = sc.generate(enc)
    monkeypatch.setenv("QKNIT_SWEEP_LANE_XCHG", "0")
    src_off, _ = sc.generate(enc)
    body = lambda src: src.split("}  // namespace qk_sweep_ops")[-1]  # noqa: E731
    assert "xchg_lane_bit_any<" in body(src_on) and "xchg_lane_bit_any<" not in body(src_off)
