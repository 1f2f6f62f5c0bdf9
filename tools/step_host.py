#!/usr/bin/env python3
"""Host launch time vs GPU start of every kernel of one mid-run step (rocprofv3 --kernel-trace
--hip-trace CSVs): which kernels waited for the host, which for other streams.

  python tools/step_host.py DIR/run_kernel_trace.csv DIR/run_hip_api_trace.csv
"""
import csv
import sys


def main():
    kt, at = sys.argv[1], sys.argv[2]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"],
                 int(r["Correlation_Id"])) for r in csv.DictReader(open(kt)))
    api = {int(r["Correlation_Id"]): int(r["Start_Timestamp"]) for r in csv.DictReader(open(at))}
    writes = [k for k in ks if "qk_knit_outer" in k[2]]
    mid = len(writes) // 2
    t0, t1 = writes[mid][0], writes[mid + 1][0]
    print(f"step interval {(t1 - t0) / 1e3:.1f} us")
    for s, e, name, st, cid in ks:
        if t0 <= s < t1:
            h = api.get(cid)
            hs = f"{(h - t0) / 1e3:8.1f}" if h else "     n/a"
            print(f"  st {st:>2} gpu +{(s - t0) / 1e3:7.1f} dur {(e - s) / 1e3:6.1f} host +{hs}  {name[:60]}")


if __name__ == "__main__":
    main()
