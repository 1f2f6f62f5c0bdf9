#!/usr/bin/env python3
"""One pipelined step's kernels from a rocprofv3 --kernel-trace CSV, by stream, in time order.

  python tools/step_timeline.py run_kernel_trace.csv|run_results.db [--steps N]

Takes the write kernel launches (qk_knit_outer_*) as step markers and prints, for the step
interval in the middle of the run, every kernel that started in it: its stream, start
offset from the interval start, duration, and the gaps on each stream (time no kernel of that
stream ran); then the time with 0, 1, 2, ... writes in flight over the middle half of the run. Used for the 8-rank rank_sim step."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    if path.endswith(".db"):  # rocprofv3's default rocpd database (its kernels view)
        import sqlite3

        con = sqlite3.connect(path)
        ks = [(int(a), int(b), n, str(s), str(q)) for a, b, n, s, q in
              con.execute("select start, end, name, stream_id, queue_id from kernels")]
    else:
        rows = list(csv.DictReader(open(path)))
        ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], r["Queue_Id"])
              for r in rows]
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
    # write concurrency over the middle half of the run (write launches n/4 .. 3n/4): the time with
    # 0, 1, 2, ... write kernels in flight
    a, b = writes[len(writes) // 4][0], writes[3 * len(writes) // 4][0]
    ev = sorted([(max(s, a), 1) for s, e, *_ in writes if e > a and s < b] +
                [(min(e, b), -1) for s, e, *_ in writes if e > a and s < b])
    depth, last, hist = 0, a, defaultdict(float)
    for t, d in ev:
        hist[depth] += (t - last) / 1e3
        depth, last = depth + d, t
    hist[depth] += (b - last) / 1e3
    n_w = 3 * len(writes) // 4 - len(writes) // 4
    print(f"write concurrency over {n_w} writes ({(b - a) / 1e3:.1f} us, {(b - a) / 1e3 / n_w:.1f} us per write): " +
          ", ".join(f"{k} in flight {v:.1f} us" for k, v in sorted(hist.items())))


if __name__ == "__main__":
    main()
