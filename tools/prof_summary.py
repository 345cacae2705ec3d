#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace into a per-step markdown table.

Accepts the ``--stats`` CSV (``*_kernel_stats.csv``; totals divided by ``--steps``) or the rocpd
SQLite database (``*_results.db``, the default output format). For the database, the timed window
is cut at the per-step optimizer launches (one ``sgd_kernel`` per step): only the last ``--steps``
steps are summarised, so warmup and set-up kernels are excluded.

  python tools/prof_summary.py gpurun_out/prof/run_results.db --steps 20 > profiles/x.md
"""
import argparse
import collections
import csv
import sqlite3


def rows_from_csv(path, steps):
    rows = list(csv.DictReader(open(path)))
    return [(r["Name"], float(r["TotalDurationNs"]), int(r["Calls"])) for r in rows], steps, None


def rows_from_db(path, steps, marker):
    c = sqlite3.connect(path)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [k for k in ks if marker in k[0]]
    if len(marks) > steps:
        t0 = marks[-steps - 1][2]
        t1 = marks[-1][2]
        ks = [k for k in ks if k[1] >= t0 and k[2] <= t1]
        wall = (t1 - t0) / 1e6 / steps
    else:
        wall = None
    agg = collections.defaultdict(lambda: [0.0, 0])
    for n, s, e in ks:
        agg[n][0] += e - s
        agg[n][1] += 1
    return [(n, v[0], v[1]) for n, v in agg.items()], steps, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1, help="number of (final) steps to summarise")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    ap.add_argument("--marker", default="sgd_kernel", help="kernel launched once per step")
    a = ap.parse_args()
    if a.path.endswith(".db"):
        rows, steps, wall = rows_from_db(a.path, a.steps, a.marker)
    else:
        rows, steps, wall = rows_from_csv(a.path, a.steps)
    tot = sum(r[1] for r in rows)
    if a.title:
        print(f"### {a.title}\n")
    print(f"GPU kernel time per step: **{tot / 1e6 / steps:.3f} ms** ({len(rows)} distinct kernels)"
          + (f"; wall time per step in the trace window: {wall:.3f} ms" if wall else "") + "\n")
    print("| ms/step | % | calls/step | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for n, t, calls in sorted(rows, key=lambda r: -r[1])[: a.top]:
        name = n.replace("|", "/")[:120]
        print(f"| {t / 1e6 / steps:.3f} | {100 * t / tot:.1f} | {calls / steps:.1f} | "
              f"{t / calls / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
