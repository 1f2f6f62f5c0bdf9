#!/usr/bin/env python3
"""Per-kernel summaries from rocprofv3's default rocpd (SQLite) output.

  python tools/rocpd_summary.py trace DB [--top 30]              kernel-trace stats (calls, avg/min/max us)
  python tools/rocpd_summary.py pmc KERNEL_SUBSTR DB [DB ...]    counter means over the kernel's dispatches

rocprofv3 on ROCm 7.2 writes ``<dir>/<host>/<pid>_results.db`` (or ``-o NAME``: ``NAME_results.db``)
unless ``--output-format csv`` is given; this reads the ``kernels`` and ``counters_collection``
views of that database. PMC: values are summed over the counter's per-SE/per-instance rows of
one dispatch, then averaged over dispatches; with ``--long`` only dispatches at least half as long
as the kernel's longest are kept (drops the short warm-up/operand launches of a shared kernel).
Durations are in ns in the database.
"""
import argparse
import collections
import sqlite3


def trace(db: str, top: int):
    con = sqlite3.connect(db)
    rows = con.execute("select name, duration from kernels").fetchall()
    agg = collections.defaultdict(list)
    for name, dur in rows:
        agg[name].append(dur / 1e3)
    total = sum(sum(v) for v in agg.values())
    lines = [f"{'kernel':72s} {'calls':>6s} {'total_us':>11s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}"]
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        lines.append(f"{name[:72]:72s} {len(v):6d} {sum(v):11.1f} {sum(v) / len(v):10.1f} {min(v):9.1f} "
                     f"{max(v):9.1f} {100 * sum(v) / total:6.2f}")
    print("\n".join(lines))
    return lines


def timeline(db: str, last: int, around: str | None = None):
    """The last ``last`` kernels in start order (with ``around``: the ``last`` kernels up to and
    including the last one whose name contains it): start / end relative to the first of them (us),
    duration, queue and stream ids (which kernels overlapped, on which queues)."""
    con = sqlite3.connect(db)
    cols = [d[0] for d in con.execute("select * from kernels limit 1").description]
    extra = [c for c in ("queue_id", "stream_id", "queue", "stream") if c in cols]
    rows = con.execute(f"select name, start, end{''.join(', ' + c for c in extra)} from kernels "
                       "order by start").fetchall()
    if around:
        hits = [i for i, r in enumerate(rows) if around in r[0]]
        if hits:
            rows = rows[:hits[-1] + 1]
    rows = rows[-last:]
    t0 = rows[0][1] if rows else 0
    lines = [f"columns: {cols}", f"{'start_us':>10s} {'end_us':>10s} {'dur_us':>9s} " + " ".join(f"{c:>9s}" for c in extra)
             + "  kernel"]
    for r in rows:
        lines.append(f"{(r[1] - t0) / 1e3:10.1f} {(r[2] - t0) / 1e3:10.1f} {(r[2] - r[1]) / 1e3:9.1f} "
                     + " ".join(f"{str(x):>9s}" for x in r[3:]) + "  " + r[0][:70])
    print("\n".join(lines))
    return lines


def pmc(kern: str, dbs: list, long_only: bool):
    vals = collections.defaultdict(list)
    durs = {}
    for db in dbs:
        con = sqlite3.connect(db)
        # instr(): case-sensitive plain substring (LIKE is case-insensitive and '_' is a wildcard)
        rows = con.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection "
                           "where instr(kernel_name, ?) > 0", (kern,)).fetchall()
        per = collections.defaultdict(float)
        dd = {}
        for did, _, cname, v, dur in rows:
            per[(did, cname)] += v
            dd[did] = dur
        if long_only and dd:
            tmax = max(dd.values())
            dd = {k: v for k, v in dd.items() if v >= 0.5 * tmax}
        for (did, cname), v in per.items():
            if did in dd:
                vals[cname].append(v)
        durs.update({(db, k): v for k, v in dd.items()})
    if not durs:
        print(f"no dispatches of *{kern}*")
        return {}
    ms = sum(durs.values()) / len(durs) / 1e6
    print(f"kernel~{kern}: {len(durs)} dispatches, mean {ms:.4f} ms")
    out = {"dispatches": len(durs), "mean_ms": ms}
    for name in sorted(vals):
        v = sum(vals[name]) / len(vals[name])
        out[name] = v
        print(f"  {name:36s} {v:18.6g}")
    return out


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("trace")
    t.add_argument("db")
    t.add_argument("--top", type=int, default=30)
    tl = sub.add_parser("timeline")
    tl.add_argument("db")
    tl.add_argument("--last", type=int, default=120)
    tl.add_argument("--around", default=None)
    p = sub.add_parser("pmc")
    p.add_argument("kernel")
    p.add_argument("dbs", nargs="+")
    p.add_argument("--long", action="store_true")
    for q in (t, tl, p):
        q.add_argument("--out", default=None, help="also write the result here (trace: text, pmc: JSON)")
    a = ap.parse_args()
    if a.cmd in ("trace", "timeline"):
        lines = trace(a.db, a.top) if a.cmd == "trace" else timeline(a.db, a.last, a.around)
        if a.out:
            open(a.out, "w").write("\n".join(lines) + "\n")
    else:
        import json

        res = pmc(a.kernel, a.dbs, a.long)
        if a.out:
            json.dump({"kernel": a.kernel, **res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
