#!/usr/bin/env python3
"""Whole-zoo throughput: native step vs the stock PyTorch-ROCm comparator, one subprocess each.

Runs ``bench.py --model M --batch B`` and ``bench.py --model M --batch B --baseline`` for every
model given (default: one representative per family) and prints one JSON line per model with
both img/s and the ratio, so a family where the native path loses to stock kernels stands out.

  python tools/zoo_bench.py [--batch 256] [--steps 10] [--warmup 3] [--timeout 150] [M ...]
"""
import argparse
import json
import os
import subprocess
import sys

FAMILIES = ["LeNet", "VGG16", "ResNet18", "ResNet50", "PreActResNet18", "GoogLeNet", "DenseNet121",
            "ResNeXt29_2x64d", "MobileNet", "MobileNetV2", "DPN26", "ShuffleNetG2",
            "ShuffleNetV2_1", "SENet18", "EfficientNetB0", "RegNetX_200MF", "RegNetY_400MF",
            "SimpleDLA", "DLA", "PNASNetA"]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(model, batch, steps, warmup, timeout, baseline):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", model, "--batch", str(batch),
           "--steps", str(steps), "--warmup", str(warmup)]
    if baseline:
        cmd.append("--baseline")
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return None, "timeout"
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            return json.loads(line), None
    return None, (p.stderr.strip().splitlines() or ["no output"])[-1][:200]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=150)
    ap.add_argument("--native-only", action="store_true", help="skip the stock comparator runs")
    ap.add_argument("models", nargs="*")
    args = ap.parse_args()
    for m in args.models or FAMILIES:
        nat, e1 = run(m, args.batch, args.steps, args.warmup, args.timeout, False)
        ref, e2 = (None, None) if args.native_only else run(m, args.batch, args.steps, args.warmup,
                                                             args.timeout, True)
        out = {"model": m, "batch": args.batch,
               "native_img_s": nat["value"] if nat else None,
               "native_ms": nat["ms_per_step"] if nat else None,
               "stock_img_s": ref["value"] if ref else None,
               "stock_ms": ref["ms_per_step"] if ref else None}
        if nat and ref:
            out["speedup"] = round(nat["value"] / ref["value"], 2)
        if e1 or e2:
            out["errors"] = [e1, e2]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
