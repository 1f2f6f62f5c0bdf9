#!/usr/bin/env python3
"""Per-pass sweep counters (rocpd_summary.py pmc outputs of the INIT / FINAL pass kernels) -> the
profiles/*_sweep_pmc.json record bench.py reads (sweep_counters).

  python tools/sweep_pmc_json.py WORKLOAD OUT.json r0=pmc_r0.json r1=pmc_r1.json

Derived per kernel: HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB (FETCH_SIZE doubled: gfx950
counts half of the wide streaming reads, MI355X_MICROARCH.md), fp64 flops = 64 x (ADD + MUL + 2 FMA)
wave-instructions, f64 issue fraction = f64 wave-instructions x 4 cycles / (1024 SIMDs x cycles),
wait / active fractions of SQ_WAVE_CYCLES, LDS bank-conflict cycles / LDS cycles, effective clock =
GRBM_GUI_ACTIVE / 8 XCDs / duration.
"""
import json
import sys


def derive(raw: dict) -> dict:
    ms = raw["mean_ms"]
    dur = ms * 1e-3
    clk = raw["GRBM_GUI_ACTIVE"] / 8 / dur
    hbm = (2 * raw["FETCH_SIZE"] + raw["WRITE_SIZE"]) * 1024.0
    f64 = raw["SQ_INSTS_VALU_ADD_F64"] + raw["SQ_INSTS_VALU_MUL_F64"] + raw["SQ_INSTS_VALU_FMA_F64"]
    flops = 64.0 * (raw["SQ_INSTS_VALU_ADD_F64"] + raw["SQ_INSTS_VALU_MUL_F64"] + 2 * raw["SQ_INSTS_VALU_FMA_F64"])
    wc = raw["SQ_WAVE_CYCLES"]
    return {
        "mean_ms": ms, "hbm_bytes": hbm, "hbm_GBs": hbm / dur / 1e9, "fp64_flops": flops,
        "fp64_TFs": flops / dur / 1e12, "f64_wave_instructions": f64,
        "f64_issue_frac": f64 * 4 / (1024 * dur * clk), "valu_wave_instructions": raw["SQ_INSTS_VALU"],
        "valu_busy_frac": raw["SQ_INSTS_VALU"] * 4 / (1024 * dur * clk),
        "wait_any_frac": raw["SQ_WAIT_ANY"] / wc, "wait_inst_frac": raw["SQ_WAIT_INST_ANY"] / wc,
        "active_frac": raw["SQ_ACTIVE_INST_ANY"] / wc,
        "lds_bank_conflict_frac": raw["SQ_LDS_BANK_CONFLICT"] / max(raw["SQ_LDS_IDX_ACTIVE"], 1.0),
        "waves": raw["SQ_WAVES"], "effective_clock_GHz": clk / 1e9, "raw": raw,
    }


def main():
    workload, out, *parts = sys.argv[1:]
    kernels = {}
    for part in parts:
        tag, _, path = part.partition("=")
        raw = json.load(open(path))
        label = {"r0": "INIT pass", "r1": "FINAL pass"}.get(tag, tag)
        kernels[f"qk_sweepm_*_{tag} ({label})"] = derive(raw)
    ms = sum(k["mean_ms"] for k in kernels.values())
    hbm = sum(k["hbm_bytes"] for k in kernels.values())
    flops = sum(k["fp64_flops"] for k in kernels.values())
    # issue fractions over the step: each kernel's SIMD-cycles of (f64 / all) VALU issue (4 cycles per
    # wave64 instruction) over the step's SIMD-cycles at that kernel's clock
    simd_cyc = sum(1024 * k["mean_ms"] * 1e-3 * k["effective_clock_GHz"] * 1e9 for k in kernels.values())
    f64_issue = sum(4 * k["f64_wave_instructions"] for k in kernels.values()) / simd_cyc
    valu_busy = sum(4 * k["valu_wave_instructions"] for k in kernels.values()) / simd_cyc
    lds = sum(k["raw"].get("SQ_LDS_IDX_ACTIVE", 0.0) for k in kernels.values())
    conf = sum(k["raw"].get("SQ_LDS_BANK_CONFLICT", 0.0) for k in kernels.values())
    rec = {
        "workload": workload, "kernels": kernels,
        "note": "rocprofv3 --pmc, four passes (FETCH_SIZE; WRITE_SIZE; 8 SQ; 7 SQ + GRBM) over tools/sweep_bench.py "
                "or tools/sweep_run.py; derivations in tools/sweep_pmc_json.py",
        "per_step": {"ms": ms, "hbm_bytes": hbm, "hbm_frac_of_8TBs": hbm / (ms * 1e-3) / 8e12, "fp64_flops": flops,
                     "fp64_frac_of_78.6TF": flops / (ms * 1e-3) / 78.6e12, "f64_issue_frac": f64_issue,
                     "valu_busy_frac": valu_busy, "lds_bank_conflict_frac": conf / lds if lds else None,
                     "per_kernel": {name: {"ms": k["mean_ms"], "hbm_GBs": k["hbm_GBs"], "valu_busy_frac": k["valu_busy_frac"],
                                           "f64_issue_frac": k["f64_issue_frac"],
                                           "lds_bank_conflict_frac": k["lds_bank_conflict_frac"],
                                           "wait_any_frac": k["wait_any_frac"], "waves": k["waves"]}
                                    for name, k in kernels.items()}},
    }
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec["per_step"]))


if __name__ == "__main__":
    main()
