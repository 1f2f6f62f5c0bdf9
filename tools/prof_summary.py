#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max µs) from a rocprofv3 .db or kernel_stats.csv."""
import collections
import csv
import glob
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    acc = collections.defaultdict(list)
    for kid, s, e, gx in c.execute("select kernel_id, start, end, grid_size_x from rocpd_kernel_dispatch"):
        acc[names.get(kid, str(kid))].append((e - s) / 1e3)
    return acc


def main():
    path = sys.argv[1]
    if path.endswith(".db"):
        acc = from_db(path)
    else:
        acc = collections.defaultdict(list)
        for f in glob.glob(path):
            for row in csv.DictReader(open(f)):
                acc[row["Kernel_Name"]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in acc.values())
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>12s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'%':>6s}")
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:70]:70s} {len(v):6d} {sum(v):12.1f} {sum(v)/len(v):10.1f} {min(v):10.1f} {max(v):10.1f} {100*sum(v)/total:6.2f}")
    # one kernel symbol serves several problem shapes (the knit contraction and the small operand
    # transforms share qk_gemm_glds_kernel): split each kernel's dispatches at half its longest
    print("\nlong dispatches (>= 50% of the kernel's longest), per kernel:")
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        big = [x for x in v if x >= 0.5 * max(v)]
        if len(big) < len(v):
            print(f"{k[:70]:70s} {len(big):6d} {sum(big):12.1f} {sum(big)/len(big):10.1f} {min(big):10.1f} "
                  f"{max(big):10.1f}")


if __name__ == "__main__":
    main()
