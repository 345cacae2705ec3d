#!/usr/bin/env python3
"""Per-kernel timeline of ONE training step from a rocprofv3 kernel trace.

Reads ``*_kernel_trace.csv`` (``rocprofv3 --kernel-trace --output-format csv``), cuts the last
complete step at the per-step optimizer launch (``--marker``, default ``sgd_``: the fused or plain SGD kernel) and prints,
in dispatch order, each kernel's start offset, duration and the idle gap before it, plus totals:
busy time (union of kernel intervals), summed kernel time, and idle time. With hipGraph replay or
a side stream, overlapping kernels show as negative gaps.

  python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv [--step -2] [--md]
"""
import argparse
import collections
import csv
import re

# kernel -> phase of the training step (pytorch_cifar_amd kernel names)
CATEGORIES = [
    ("conv fwd", r"conv_igemm_(ph_)?kernel<[^>]*, 0, |conv3x3_c64_kernel<false|splitk_reduce_kernel<true>|dw_fwd|direct_fwd"),
    ("conv dgrad", r"conv_igemm_(ph_)?kernel<[^>]*, [12], |conv3x3_c64_kernel<true|splitk_reduce_kernel<false>|dw_dgrad|direct_dgrad"),
    ("conv wgrad", r"wgrad|slab_reduce|dw_w"),
    ("batchnorm fwd", r"bn_apply|bn_finalize|bn_stats|colsum"),
    ("batchnorm bwd", r"bn_bwd"),
    ("optimizer / weight prep", r"sgd_kernel|weight_prep"),
    ("squeeze-excite", r"se_scale|se_"),
    ("head (pool, linear, CE)", r"head_|gap_|Cijk|ce_fused|scale_by_scalar|reduce_kernel"),
    ("data (augment, gather)", r"augment|scatter_gather|copyBuffer"),
]


def category(name):
    for cat, rx in CATEGORIES:
        if re.search(rx, name):
            return cat
    return "other (fills, elementwise)"


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        s = int(r.get("Start_Timestamp") or r.get("BeginNs") or r.get("start"))
        e = int(r.get("End_Timestamp") or r.get("EndNs") or r.get("end"))
        out.append((s, e, name))
    out.sort()
    return out


def short(name, n=90):
    name = re.sub(r"\(.*", "", name) if "(" in name else name
    name = name.replace("void ", "").replace("pca::", "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="sgd_")
    ap.add_argument("--step", type=int, default=-2, help="which step window (python index over windows)")
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--categories", action="store_true", help="print only per-phase totals")
    a = ap.parse_args()
    ks = load(a.path)
    marks = [i for i, k in enumerate(ks) if a.marker in k[2]]
    if len(marks) < 2:
        raise SystemExit("need at least two marker kernels")
    wins = list(zip(marks[:-1], marks[1:]))
    i0, i1 = wins[a.step]
    step = ks[i0 + 1: i1 + 1]
    t0 = ks[i0][1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = step[-1][1] - t0
    ksum = sum(e - s for s, e, _ in step)
    print(f"kernels: {len(step)}; step wall (marker to marker): {wall / 1e3:.1f} us; "
          f"busy (union): {busy / 1e3:.1f} us; summed kernel time: {ksum / 1e3:.1f} us; "
          f"idle: {(wall - busy) / 1e3:.1f} us\n")
    if a.categories:
        agg = collections.defaultdict(lambda: [0.0, 0])
        for s_, e_, n_ in step:
            agg[category(n_)][0] += (e_ - s_) / 1e3
            agg[category(n_)][1] += 1
        print("| phase | us / step | % | kernels |\n|---|---:|---:|---:|")
        for cat, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
            print(f"| {cat} | {t:.1f} | {100 * t * 1e3 / ksum:.1f} | {c} |")
        return
    if a.md:
        print("| # | start us | dur us | gap us | kernel |\n|---:|---:|---:|---:|---|")
    prev_e = t0
    for j, (s, e, n) in enumerate(step):
        gap = (s - prev_e) / 1e3
        if a.md:
            print(f"| {j} | {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {gap:.1f} | `{short(n)}` |")
        else:
            print(f"{j:4d} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap:6.1f}  {short(n)}")
        prev_e = max(prev_e, e)


if __name__ == "__main__":
    main()
