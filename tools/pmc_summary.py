#!/usr/bin/env python3
"""Average rocprofv3 --pmc CSV counters per kernel (skips the first dispatch = warm-up).

  python tools/pmc_summary.py gpurun_out/pmc/<tag>_p1 gpurun_out/pmc/<tag>_p2
"""
import collections
import csv
import glob
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                vals[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        if "conv" not in k and "wgrad" not in k and "stem" not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            v = v[1:] if len(v) > 1 else v
            print(f"  {c:28s} {sum(v) / len(v):16.0f}")


if __name__ == "__main__":
    main()
