#!/usr/bin/env python3
"""MFMA counters of the exact K-term contraction (bench.py knit_general) -> profiles/*_gemm_k64_pmc.json.

  python tools/gemm_pmc_json.py OUT.json RAW.json M N K

RAW.json: tools/rocpd_summary.py pmc output over rocprofv3 --pmc passes of tools/step_run.py
--no-data-rank (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64
SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE). Derived:
flops = 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 (checked against 2 M N K); effective clock =
GRBM_GUI_ACTIVE / 8 XCDs / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
(v_mfma_f64_16x16x4_f64 holds its SIMD 64 cycles); HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB.
"""
import json
import sys


def main():
    out, raw_path, M, N, K = sys.argv[1], sys.argv[2], *map(int, sys.argv[3:6])
    raw = json.load(open(raw_path))
    dur = raw["mean_ms"] * 1e-3
    clk = raw["GRBM_GUI_ACTIVE"] / 8 / dur
    flops = 512.0 * raw["SQ_INSTS_VALU_MFMA_MOPS_F64"]
    alg = 2.0 * M * N * K
    busy = raw["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * dur)
    hbm = (2 * raw["FETCH_SIZE"] + raw["WRITE_SIZE"]) * 1024.0
    rec = {"kernel": raw.get("kernel"), "gemm_mnk": [M, N, K], "mean_ms": raw["mean_ms"],
           "dispatches": raw.get("dispatches"), "flops_counted": flops, "flops_algorithmic": alg,
           "achieved_TFs": flops / dur / 1e12, "frac_of_78.6TF": flops / dur / 78.6e12,
           "effective_clock_GHz": clk / 1e9,
           "frac_of_clock_peak": flops / dur / (1024 * 32 * clk),  # 2048 flops per 64-cycle MFMA per SIMD
           "mfma_busy_frac": busy, "mfma_cycles_per_instruction": raw["SQ_VALU_MFMA_BUSY_CYCLES"] / raw["SQ_INSTS_VALU_MFMA_F64"],
           "hbm_bytes_per_launch": hbm, "output_bytes": 8.0 * M * N, "raw": raw,
           "note": "rocprofv3 --pmc over tools/step_run.py --no-data-rank; derivations in tools/gemm_pmc_json.py"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "raw"}))


if __name__ == "__main__":
    main()
