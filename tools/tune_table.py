#!/usr/bin/env python3
"""Measure and write the shipped kernel-selection table (pytorch_cifar_amd/tune/mi355x.json).

Runs each BASELINE configuration's bench step once with the table disabled and a fresh tune cache
(every conv geometry autotuned on this box), then writes the union of the selections, stamped with
the extension's candidate-set version (engine/tuning.py ignores a table of another version).

  python tools/tune_table.py [--out pytorch_cifar_amd/tune/mi355x.json]     # on a GPU box
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CONFIGS = [("ResNet18", 1024), ("ResNet18", 512), ("ResNet18", 256), ("ResNet18", 128),
           ("MobileNetV2", 1024), ("EfficientNetB0", 1024), ("EfficientNetB0", 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "pytorch_cifar_amd", "tune", "mi355x.json"))
    ap.add_argument("--configs", default="",
                    help="Model:batch,... to measure instead of the BASELINE set")
    ap.add_argument("--merge", nargs="*", default=None,
                    help="keep the rows of --out and add only geometries it lacks: from these "
                         "PCA_TUNE_CACHE files if given (no GPU needed), else measured")
    args = ap.parse_args()
    configs = ([(c.split(":")[0], int(c.split(":")[1])) for c in args.configs.split(",")]
               if args.configs else CONFIGS)
    rows, runs = {}, []
    old = None
    if args.merge is not None:
        with open(args.out) as fh:
            old = json.load(fh)
        for r in old["rows"]:
            rows[tuple(r[:14])] = r
        runs = list(old.get("configs", []))
        if args.merge:
            added = 0
            for path in args.merge:
                with open(path) as fh:
                    for r in json.load(fh):
                        if tuple(r[:14]) not in rows:
                            rows[tuple(r[:14])] = r
                            added += 1
                runs.append({"cache": os.path.basename(path)})
            from pytorch_cifar_amd.engine.tuning import selection_hash

            old.update(rows=sorted(rows.values()), configs=runs,
                       hash=selection_hash(rows.values()))
            with open(args.out, "w") as fh:
                json.dump(old, fh, indent=0)
            print("merged", added, "rows ->", len(rows), "hash", old["hash"])
            return
    for model, batch in configs:
        with tempfile.TemporaryDirectory() as d:
            cache = os.path.join(d, "tune.json")
            env = dict(os.environ, PCA_TUNE_TABLE="0", PCA_TUNE_CACHE=cache)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", model, "--batch", str(batch),
                   "--steps", "3", "--warmup", "2"]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                sys.exit(f"{model} bs{batch} failed:\n{p.stderr[-2000:]}")
            with open(cache) as fh:
                got = json.load(fh)
            for r in got:
                if old is None or tuple(r[:14]) not in rows:
                    rows[tuple(r[:14])] = r
            runs.append({"model": model, "batch": batch, "rows": len(got)})
            print(model, batch, len(got), flush=True)
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.engine.tuning import selection_hash

    lib = _native.lib()
    import torch

    props = torch.cuda.get_device_properties(0)
    out = {"version": lib.tune_version(), "arch": "gfx950", "cus": props.multi_processor_count,
           "configs": runs,
           "rows": sorted(rows.values()), "hash": selection_hash(rows.values())}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=0)
    print("wrote", args.out, len(rows), "rows, hash", out["hash"])


if __name__ == "__main__":
    main()
