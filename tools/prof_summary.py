#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a markdown table.

  python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 13 > profiles/x.md
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if a.title:
        print(f"### {a.title}\n")
    print(f"GPU kernel time per step: **{tot / 1e6 / a.steps:.3f} ms** ({len(rows)} distinct kernels)\n")
    print("| ms/step | % | calls/step | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        name = r["Name"].replace("|", "/")[:110]
        print(f"| {float(r['TotalDurationNs']) / 1e6 / a.steps:.3f} | {float(r['Percentage']):.1f} | "
              f"{int(r['Calls']) / a.steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
