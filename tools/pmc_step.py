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


def _grid(r):
    g = r.get("Grid_Size")
    if g:
        return int(g)
    return int(r.get("Grid_Size_X", 1)) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1))


def _window(rows):
    """rows (dispatch_id, ...) sorted; keep the last complete step (after the second-to-last
    sgd_kernel up to and including the last one)."""
    sgd = [r[0] for r in rows if "sgd_kernel" in r[1] or "sgd_prep_kernel" in r[1]]
    if len(sgd) >= 2:
        lo, hi = sgd[-2], sgd[-1]
        rows = [r for r in rows if lo < r[0] <= hi]
    return rows


def load_run(d):
    """{key: [us, launches, Counter]} of one run's last step. Counters and durations are windowed
    and keyed (kernel name @ grid) separately: the counter and trace CSVs number dispatches
    independently."""
    out = collections.defaultdict(lambda: [0.0, 0, collections.Counter()])
    trace = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            trace.append((int(r["Dispatch_Id"]), r["Kernel_Name"], _grid(r),
                          (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    trace.sort()
    for _, name, g, us in _window(trace):
        e = out[f"{name} @grid{g}"]
        e[0] += us
        e[1] += 1
    per = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            ent = per.setdefault(did, [did, r["Kernel_Name"], _grid(r), collections.Counter()])
            ent[3][r["Counter_Name"]] += float(r["Counter_Value"])
    for _, name, g, cs in _window(sorted(per.values(), key=lambda x: x[0])):
        key = f"{name} @grid{g}"
        if key not in out:
            # grid reported differently by the two CSVs: fall back to a unique same-name entry
            same = [k for k in out if k.rsplit(" @grid", 1)[0] == name]
            if len(same) == 1:
                key = same[0]
        out[key][2].update(cs)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: {"us": [], "n": 0, "c": collections.Counter()})
    for d in a.dirs:
        for name, (us, n, cs) in load_run(d).items():
            if n:
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
    # whole-step traffic past L2 (the same FETCH/WRITE estimate as the per-kernel column)
    tb = sum((2 * e["c"].get("FETCH_SIZE", 0.0) + e["c"].get("WRITE_SIZE", 0.0)) * 1024
             for e in agg.values())
    if tb > 0 and total > 0:
        print(f"step traffic past L2: {tb / 1e9:.2f} GB -> {tb / (total * 1e3):.0f} GB/s averaged over "
              f"the step's kernel time")
    print(hdr)
    for us, n, mfma, gbs, conf, lds, name in rows[: a.top if a.top > 0 else None]:
        cp = f"{100.0 * conf / lds:8.1f}" if conf is not None and lds else f"{'-':>8}"
        print(f"{us:9.1f} {n:3d} {mfma if mfma is not None else float('nan'):6.1f} "
              f"{gbs if gbs is not None else float('nan'):9.0f} {cp}  {short(name)}")


if __name__ == "__main__":
    main()
