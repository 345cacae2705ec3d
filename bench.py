#!/usr/bin/env python3
"""Headline benchmark: ResNet-18 training throughput (images/sec, whole node) at global batch 1024.

Metric/config from BASELINE.json: "images/sec (whole node) ResNet-18 bs=1024 at 1/2/4/8 MI355X".
One process per GPU (torchrun env: RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), RCCL data parallelism,
bf16 compute, synthetic 32x32x3 uint8 images through the GPU augmentation kernel (crop+flip+
normalize, main.py's train transform), random-init weights, full step timed: augment, forward,
cross-entropy, backward, gradient all-reduce, SGD(momentum 0.9, wd 5e-4) update.

The global batch is fixed at 1024 and split across ranks (main_dist.py:111: batch_size/world), so
scaling is "strong". Prints exactly one JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--model ResNet18] [--batch 1024]

--gpus N > 1 works both under torchrun (the driver's form) and stand-alone: without a WORLD_SIZE
in the environment bench.py starts the N rank processes itself (parallel/launcher.py
spawn_local_ranks, one fresh interpreter per GPU with the torchrun env on 127.0.0.1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REF_NAME = "aqualovers/pytorch-cifar"


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="ResNet18")
    ap.add_argument("--batch", type=int, default=1024, help="global batch")
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a hipGraph (1/0)")
    # 4 MiB buckets (not DDP's 25): only the last bucket's all-reduce is exposed after the
    # backward; arithmetic in parallel/ddp.py (25 MiB: ~11 MB exposed, 4 MiB: ~4 MB)
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--grad-compress", default="none", choices=["none", "bf16", "bf16_tail"],
                    help="opt-in bf16 gradient all-reduce (off: exact fp32 DDP semantics)")
    ap.add_argument("--baseline", action="store_true",
                    help="run the stock PyTorch-ROCm comparator step instead (MIOpen/hipBLASLt, autocast bf16)")
    ap.add_argument("--profile-steps", type=int, default=0)
    return ap.parse_args()


def main():
    args = parse()
    from pytorch_cifar_amd.parallel import launcher

    if args.gpus > 1 and launcher.spawned_world() == 0:
        # `python bench.py --gpus N` without torchrun: start the N rank processes ourselves (the
        # reference's main_dist.py:51-60 mp.spawn), before anything here touches the GPU; rank 0
        # of the children prints the JSON line.
        ngpu = torch.cuda.device_count()      # counts devices without initialising HIP
        if 0 < ngpu < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but only {ngpu} GPU(s) visible")
        sys.exit(launcher.spawn_local_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))

    ctx = launcher.init_from_env(backend="nccl")
    rank, world = ctx.rank, ctx.world
    if world != args.gpus and rank == 0:
        # n_gpus / parallelism below report the ranks actually timed (WORLD_SIZE)
        print(f"bench.py: warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    device = ctx.device
    per_rank = args.batch // world

    from pytorch_cifar_amd.engine.trainer import build_bench_step

    step, meta = build_bench_step(args.model, per_rank, device, ctx, graph=bool(args.graph),
                                  baseline=args.baseline, bucket_mb=args.bucket_mb,
                                  grad_compress=args.grad_compress)

    # (CPU runs — the gloo contract test in tests/test_cli_cpu.py — have nothing to synchronize)
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    for _ in range(args.warmup):
        step()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    ctx.barrier()
    t1 = time.perf_counter()
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    dt = ctx.all_reduce_max(dt)
    elapsed = float(dt.item())
    ms = elapsed / args.steps * 1e3
    img_s = per_rank * world * args.steps / elapsed
    base = None
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")) as f:
            pub = json.load(f).get("published") or {}
        base = pub.get("value") if isinstance(pub, dict) else None
    except Exception:
        base = None
    if hasattr(step, "info"):
        meta.update(step.info())
    if rank == 0:
        out = {
            "metric": ("images/sec (whole node) ResNet-18 bs=1024 at 1/2/4/8 MI355X" if args.model == "ResNet18"
                       else f"images/sec (whole node) {args.model} bs={args.batch}"),
            "value": round(img_s, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (img_s / base) if base else None,
            "dtype": "bf16",
            "data": "synthetic (uint8 32x32x3 images, random labels; GPU crop+flip+normalize); random-init weights",
            "config": {
                "model": args.model,
                "global_batch": per_rank * world,
                "seq_len": None,
                "image": "32x32x3",
                "parallelism": f"dp{world}",
                "graph": bool(args.graph) and not args.baseline,
                "impl": "stock-pytorch-rocm" if args.baseline else "pytorch_cifar_amd",
                **meta,
            },
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
