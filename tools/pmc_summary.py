#!/usr/bin/env python3
"""Counter values of the longest dispatches of one kernel from rocprofv3 --pmc output dirs.

  python tools/pmc_summary.py KERNEL_SUBSTR DIR [DIR ...]
Prints, per counter, the mean over the kernel's long dispatches (>= half the longest), plus the
dispatch duration; with GRBM_GUI_ACTIVE present also the effective clock (GUI_ACTIVE / 8 XCDs /
duration, MI355X_MICROARCH.md DVFS note).
"""
import collections
import csv
import glob
import os
import sys


def main():
    kern, dirs = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(list)
    durs = []
    for d in dirs:
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
        if not rows:
            continue
        dur = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows}
        tmax = max(dur.values())
        keep = {k for k, v in dur.items() if v >= 0.5 * tmax}
        durs += [dur[k] for k in keep]
        per = collections.defaultdict(float)
        for r in rows:
            if r["Dispatch_Id"] in keep:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (did, name), v in per.items():
            vals[name].append(v)
    ms = sum(durs) / max(len(durs), 1)
    print(f"kernel~{kern}: {len(durs)} long dispatches, mean {ms:.3f} ms")
    for name in sorted(vals):
        v = sum(vals[name]) / len(vals[name])
        print(f"  {name:36s} {v:18.4g}")
    if "GRBM_GUI_ACTIVE" in vals:
        g = sum(vals["GRBM_GUI_ACTIVE"]) / len(vals["GRBM_GUI_ACTIVE"])
        print(f"  effective clock ~ {g / 8 / (ms * 1e-3) / 1e9:.3f} GHz")


if __name__ == "__main__":
    main()
