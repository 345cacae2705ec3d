#!/usr/bin/env python3
"""profiles/zoo_bs256_r3.md from the native zoo pass (tools/gpu/zoo_r3.sh) next to round 2."""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
r2 = {}
for ln in open(os.path.join(ROOT, "profiles/zoo_bs256_r2.md")):
    m = re.match(r"\| (\S+) \| ([\d,]+) \| ([\d.]+) \| [\d.]+ \| ([\d,]+) \| ([\d.]+) \|", ln)
    if m:
        r2[m.group(1)] = (float(m.group(3)), int(m.group(4).replace(",", "")))
rows = []
d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out/zoo3")
for f in sorted(glob.glob(f"{d}/*.json")):
    name = os.path.basename(f)[:-5]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        rows.append((name, None, None))
        continue
    rows.append((name, j["ms_per_step"], j["value"]))
print("# Whole-zoo training throughput, bs=256, 1x MI355X (round 3, native path)\n")
print("`bash tools/gpu/zoo_r3.sh` (native `bench.py --model M --batch 256 --steps 10 --warmup 3`, one process per "
      "model; raw lines `profiles/bench/zoo_bs256_r3/`). Round-2 native and stock columns from "
      "`profiles/zoo_bs256_r2.md` (a different box: expect a few % box-to-box spread). The odd-width grouped nets "
      "(ShuffleNetG2/G3, DPN26, ResNeXt29_32x4d, PNASNet, LeNet, densenet_cifar) now pad / slice / shuffle their "
      "channels with native remap kernels.\n")
print("| model | native img/s | native ms/step | round-2 native ms | stock img/s (r2) | speed-up vs stock |")
print("|---|---:|---:|---:|---:|---:|")
for name, ms, v in rows:
    if ms is None:
        print(f"| {name} | failed | | | | |")
        continue
    p = r2.get(name)
    sp = f"{v / p[1]:.2f}x" if p else "—"
    print(f"| {name} | {v:,.0f} | {ms:.3f} | {p[0] if p else '—'} | {f'{p[1]:,}' if p else '—'} | {sp} |")
