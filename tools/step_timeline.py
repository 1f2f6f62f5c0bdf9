#!/usr/bin/env python3
"""One pipelined step's kernels from a rocprofv3 --kernel-trace CSV, by stream, in time order.

  python tools/step_timeline.py run_kernel_trace.csv [--steps N]

Takes the write kernel launches (qk_knit_outer_*) as step markers and prints, for the step
interval in the middle of the run, every kernel that started in it: its stream, start
offset from the interval start, duration, and the gaps on each stream (time no kernel of that
stream ran). Used for the 8-rank rank_sim step."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], r["Queue_Id"]) for r in rows]
    ks.sort()
    writes = [k for k in ks if "qk_knit_outer" in k[2]]
    if len(writes) < 3:
        sys.exit("fewer than 3 write kernels in the trace")
    mid = len(writes) // 2  # a step in the middle of the run (the last ones have no next preparation)
    t0, t1 = writes[mid][0], writes[mid + 1][0]
    print(f"step interval {(t1 - t0) / 1e3:.1f} us (write start to write start)")
    busy = defaultdict(float)
    for s, e, name, st, q in ks:
        if t0 <= s < t1:
            busy[st] += (e - s) / 1e3
            print(f"  stream {st:>3} q{q:>2} +{(s - t0) / 1e3:8.1f} us {(e - s) / 1e3:8.1f} us  {name[:90]}")
    for st, b in sorted(busy.items()):
        print(f"stream {st}: kernels {b:.1f} us of {(t1 - t0) / 1e3:.1f}")


if __name__ == "__main__":
    main()
