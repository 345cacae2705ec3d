#!/usr/bin/env python3
"""Per-kernel PMC table of ONE eager training step (derived MFMA-busy % and HBM GB/s).

Input: the directories of several ``rocprofv3 --pmc <set> --kernel-trace --output-format csv``
runs of ``bench.py --graph 0`` (tools/gpu/pmc_step.sh), one counter set per run. For every run
the last complete step is cut at the optimizer launch (``sgd_kernel``: dispatches after the
second-to-last one up to and including the last one), counters are joined to durations by
Dispatch_Id, and kernels of the same name are summed over the step.

Derived columns (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE sums the 8 XCDs; 256 CUs x 4 SIMDs):
* MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
* HBM GB/s   = (2 * FETCH_SIZE + WRITE_SIZE) KiB / duration  (FETCH_SIZE reads half the bytes
  of a wide coalesced stream on gfx950, so it is doubled; the absolute is an estimate)

  python tools/pmc_step.py gpurun_out/pmc_step/b1024_p* [--top 12] [--md]
"""
import argparse
import collections
import csv
import glob
import re


def short(name, n=70):
    grid = name[name.rfind(" @grid"):] if " @grid" in name else ""
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("pca::", "")
    return name[:n] + grid


def load_run(d):
    trace = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            g = r.get("Grid_Size") or (int(r.get("Grid_Size_X", 1)) * int(r.get("Grid_Size_Y", 1))
                                       * int(r.get("Grid_Size_Z", 1)))
            trace[int(r["Dispatch_Id"])] = (f'{r["Kernel_Name"]} @grid{g}', int(r["Start_Timestamp"]),
                                            int(r["End_Timestamp"]))
    counters = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            counters[did][r["Counter_Name"]] = counters[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if did not in trace:
                trace[did] = (f'{r["Kernel_Name"]} @grid{r.get("Grid_Size", "?")}', 0, 0)
    ids = sorted(trace)
    sgd = [i for i in ids if "sgd_kernel" in trace[i][0]]
    if len(sgd) >= 2:
        lo, hi = sgd[-2], sgd[-1]
        ids = [i for i in ids if lo < i <= hi]
    return [(trace[i][0], (trace[i][2] - trace[i][1]) / 1e3, counters.get(i, {})) for i in ids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: {"us": [], "n": 0, "c": collections.Counter()})
    for d in a.dirs:
        per = collections.defaultdict(lambda: [0.0, 0, collections.Counter()])
        for name, us, cs in load_run(d):
            e = per[name]
            e[0] += us
            e[1] += 1
            e[2].update(cs)
        for name, (us, n, cs) in per.items():
            agg[name]["us"].append(us)
            agg[name]["n"] = max(agg[name]["n"], n)
            agg[name]["c"].update(cs)
    rows = []
    for name, e in agg.items():
        us = min(e["us"]) if e["us"] else 0.0
        c = e["c"]
        mfma = None
        if c.get("GRBM_GUI_ACTIVE"):
            mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        gbs = None
        if us > 0 and ("FETCH_SIZE" in c or "WRITE_SIZE" in c):
            gbs = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024 / (us * 1e3)
        rows.append((us, e["n"], mfma, gbs, c.get("SQ_LDS_BANK_CONFLICT"), c.get("SQ_INSTS_LDS"), name))
    rows.sort(key=lambda r: -r[0])
    total = sum(r[0] for r in rows)
    hdr = f"{'us/step':>9} {'n':>3} {'MFMA%':>6} {'HBM GB/s':>9} {'LDSconf%':>8}  kernel"
    print(f"step kernels: {total:.1f} us (min over passes per kernel), {len(rows)} distinct kernels")
    print(hdr)
    for us, n, mfma, gbs, conf, lds, name in rows[: a.top if a.top > 0 else None]:
        cp = f"{100.0 * conf / lds:8.1f}" if conf is not None and lds else f"{'-':>8}"
        print(f"{us:9.1f} {n:3d} {mfma if mfma is not None else float('nan'):6.1f} "
              f"{gbs if gbs is not None else float('nan'):9.0f} {cp}  {short(name)}")


if __name__ == "__main__":
    main()
