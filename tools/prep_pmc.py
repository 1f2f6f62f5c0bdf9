#!/usr/bin/env python3
"""Per-kernel counters of the data-rank preparation chain from rocprofv3 --pmc passes over
tools/step_run.py (one pass per counter group: the TCC block holds FETCH_SIZE or WRITE_SIZE, not
both). Writes a JSON summary (profiles/r03_prep_pmc.json).

    python tools/prep_pmc.py --out profiles/r03_prep_pmc.json DIR [DIR ...]

Per kernel: mean duration over its dispatches, HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB; FETCH
doubled for gfx950's half count of wide streaming reads, MI355X_MICROARCH.md HBM section) and their
fraction of 8 TB/s, VALU issue (4 cycles per wave-instruction) and MFMA busy cycles as fractions of
the chip's 1024 SIMDs x the dispatch's cycles (GRBM_GUI_ACTIVE / 8 XCDs, else 2.4 GHz), LDS
bank-conflict cycles per LDS-active cycle.
"""
import argparse
import collections
import csv
import glob
import json
import os

CHAIN = ("qk_prep_operands_kernel", "qk_prep_reduce_kernel", "qk_rank_factors_kernel", "qk_compress_cols_kernel",
         "qk_compress_kernel", "qk_gemm_glds_kernel", "qk_gemm_wave_kernel",
         "qk_probe_v_kernel", "qk_probe_d_kernel", "qk_probe_accept_kernel",
         "qk_knit_outer_blocked_kernel", "qk_select")


def collect(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            acc = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                name = next((k for k in CHAIN if k in r["Kernel_Name"]), None)
                if name is None:
                    continue
                key = (f, r["Dispatch_Id"])
                acc[(name, key, r["Counter_Name"])] += float(r["Counter_Value"])
                durs[name][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for (name, key, cn), v in acc.items():
                per[name][cn].append(v)
    return per, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    args = ap.parse_args()
    per, durs = collect(args.dirs)
    out = {"workload": "syc 32 5 p=2 bench step (tools/step_run.py)", "note": args.note, "kernels": {}}
    for name in CHAIN:
        if name not in per:
            continue
        c = {k: sum(v) / len(v) for k, v in per[name].items()}
        ms = sum(durs[name].values()) / len(durs[name])
        rec = {"mean_ms": ms, "dispatches": len(durs[name]), "raw": c}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            b = 2 * 1024 * c.get("FETCH_SIZE", 0.0) + 1024 * c.get("WRITE_SIZE", 0.0)
            rec.update(hbm_bytes=b, hbm_GBs=b / (ms * 1e-3) / 1e9, hbm_frac=b / (ms * 1e-3) / 8e12)
        # clock cycles of the dispatch: GRBM_GUI_ACTIVE / 8 XCDs when counted, else 2.4 GHz nominal
        cycles = c["GRBM_GUI_ACTIVE"] / 8 if "GRBM_GUI_ACTIVE" in c else ms * 1e-3 * 2.4e9
        if "GRBM_GUI_ACTIVE" in c:
            rec["effective_clock_GHz"] = cycles / (ms * 1e-3) / 1e9
        simd_cycles = 1024 * cycles  # 256 CUs x 4 SIMDs
        if "SQ_INSTS_VALU" in c:
            rec["valu_busy_frac"] = 4 * c["SQ_INSTS_VALU"] / simd_cycles  # a wave-instruction: 4 cycles
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            rec["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        if c.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        out["kernels"][name] = rec
    chain = [k for k in out["kernels"] if k not in ("qk_knit_outer_blocked_kernel", "qk_select")]
    out["chain_ms"] = sum(out["kernels"][k]["mean_ms"] for k in chain)
    json.dump(out, open(args.out, "w"), indent=1)
    for k, r in out["kernels"].items():
        print(k, {a: (round(b, 4) if isinstance(b, float) else b) for a, b in r.items() if a != "raw"})
    print("chain_ms", out["chain_ms"])


if __name__ == "__main__":
    main()
