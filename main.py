#!/usr/bin/env python3
'''Train CIFAR10 on MI355X (single process) — CLI parity with the reference main.py.

Reference flags: --lr (0.1), --resume/-r. Additive flags: --model (default SimpleDLA, the
reference's main.py:71 choice), --epochs (200), --batch_size (128), --test_batch_size (100),
--data_dir, --synthetic, --seed, --graph, --max_steps, --log_every, --checkpoint_dir, --cpu.

Semantics kept: RandomCrop(32, pad 4) + HFlip + Normalize train transform, SGD(momentum 0.9,
wd 5e-4), CosineAnnealingLR(T_max=200) stepped per epoch, CE loss, best-accuracy checkpoint
``./checkpoint/ckpt.pth`` = {'net', 'acc', 'epoch'} with the wrapped net's ``module.`` keys.
'''
import argparse
import os
import sys

import torch

from pytorch_cifar_amd import models
from pytorch_cifar_amd.data.factory import build_loaders
from pytorch_cifar_amd.engine.arena import ParamArena
from pytorch_cifar_amd.engine.checkpoint import load_checkpoint, save_checkpoint
from pytorch_cifar_amd.engine.optim import SGD
from pytorch_cifar_amd.engine.trainer import Trainer
from pytorch_cifar_amd.parallel import launcher
from pytorch_cifar_amd.parallel.data_parallel import DataParallel
from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel
from pytorch_cifar_amd.parallel.launcher import DistContext
from utils import progress_bar

parser = argparse.ArgumentParser(description='PyTorch CIFAR10 Training (MI355X-native)')
parser.add_argument('--lr', default=0.1, type=float, help='learning rate')
parser.add_argument('--resume', '-r', action='store_true', help='resume from checkpoint')
parser.add_argument('--model', default='SimpleDLA', help='model constructor name (see models.MODEL_REGISTRY)')
parser.add_argument('--epochs', default=200, type=int, help='number of epochs')
parser.add_argument('--batch_size', default=128, type=int)
parser.add_argument('--test_batch_size', default=100, type=int)
parser.add_argument('--data_dir', default='./data')
parser.add_argument('--synthetic', action='store_true', help='synthetic CIFAR-shaped data (no dataset files)')
parser.add_argument('--synthetic_size', default=None, type=int)
parser.add_argument('--seed', default=0, type=int)
parser.add_argument('--graph', default=1, type=int, help='capture the train step in a hipGraph (GPU)')
parser.add_argument('--max_steps', default=None, type=int, help='cap steps per epoch (smoke runs)')
parser.add_argument('--log_every', default=20, type=int)
parser.add_argument('--checkpoint_dir', default='./checkpoint')
parser.add_argument('--cpu', action='store_true', help='force the CPU reference path')
parser.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'],
                    help='bf16: native MI355X kernels; fp32: stock PyTorch fp32 kernels on the GPU')
parser.add_argument('--deterministic', action='store_true', help='bitwise-reproducible weight gradients')
parser.add_argument('--debug_sync', action='store_true',
                    help='sync + error-check after every native op (locates async GPU faults; disables graphs)')
parser.add_argument('--profile', default=None, metavar='TRACE.json',
                    help='torch.profiler Chrome trace of the first training steps')
parser.add_argument('--no_nan_guard', action='store_true', help='do not stop on a non-finite loss')
parser.add_argument('--t_max', default=200, type=int, help='cosine schedule length (reference: 200)')
parser.add_argument('--nproc', default=None, type=int,
                    help='data-parallel ranks (default: every visible GPU, one process each; '
                         'the reference main.py:74 DataParallel used all GPUs too)')
parser.add_argument('--bucket_mb', default=4.0, type=float, help='gradient all-reduce bucket size (MiB)')



def _apply_runtime_flags(args, loaders):
    """--deterministic / --debug_sync / --dtype fp32 (aux subsystems)."""
    import pytorch_cifar_amd
    from pytorch_cifar_amd.ops import functional as PF

    on_gpu = torch.cuda.is_available() and not args.cpu
    if args.deterministic and on_gpu:
        pytorch_cifar_amd.set_deterministic(True)
    if args.debug_sync:
        pytorch_cifar_amd.set_debug_sync(True)
        args.graph = 0
    if args.dtype == 'fp32' and on_gpu:
        PF.set_reference_mode(True)
        args.graph = 0
        for ld in loaders:
            ld.fp32 = True

def _data_parallel_ranks(args):
    # The launcher parent must stay off the GPU (it spawns the per-GPU ranks): --nproc or the
    # visible-device list decide first; otherwise the devices are counted in a short-lived child
    # process, since torch.cuda.device_count() may fall back to hipGetDeviceCount (a HIP
    # initialisation) when amdsmi is unavailable.
    if args.nproc:
        return args.nproc
    if args.cpu:
        return 1
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            # an empty list hides every GPU: one process (it runs on the CPU)
            return max(1, len([d for d in v.split(",") if d.strip()]))
    import subprocess
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=180)
    except subprocess.TimeoutExpired:
        sys.exit("main.py: counting GPUs timed out (HIP runtime hung?); pass --nproc N")
    if r.returncode != 0:
        sys.exit(f"main.py: counting GPUs failed (rc {r.returncode}): {r.stderr.strip()[-300:]}; "
                 "pass --nproc N")
    try:
        return max(1, int(r.stdout.strip().splitlines()[-1]))
    except (ValueError, IndexError):
        return 1


def main(argv=None):
    args = parser.parse_args(argv)
    nranks = _data_parallel_ranks(args)
    if nranks > 1 and launcher.spawned_world() == 0:
        # Reference main.py:73-74 wraps the net in nn.DataParallel over every visible GPU. Here each
        # GPU gets its own rank process (started fresh, the parent never touches the GPU) running
        # the native RCCL bucket engine; the batch is split across ranks like DataParallel's
        # scatter, and rank 0 writes the same module.-prefixed checkpoint.
        argv = list(sys.argv[1:] if argv is None else argv)
        rc = launcher.spawn_local_ranks(nranks, [os.path.abspath(__file__)] + argv)
        if rc:
            raise SystemExit(rc)
        return 0.0
    if launcher.spawned_world() > 1:
        ctx = launcher.init_from_env(backend='gloo' if args.cpu else 'nccl')
    else:
        dev = torch.device('cuda', 0) if torch.cuda.is_available() and not args.cpu else torch.device('cpu')
        if dev.type == 'cuda':
            torch.cuda.set_device(dev)
        ctx = DistContext(device=dev)
    device = ctx.device
    is_main = ctx.rank == 0
    torch.manual_seed(args.seed)
    best_acc = 0  # best test accuracy
    start_epoch = 0  # start from epoch 0 or last checkpoint epoch

    say = print if is_main else (lambda *a, **k: None)
    say('==> Preparing data..')
    batch_size = max(1, args.batch_size // ctx.world)
    test_batch_size = max(1, args.test_batch_size // ctx.world)
    trainloader, testloader = build_loaders(args.data_dir, args.synthetic, batch_size,
                                            test_batch_size, device, world=ctx.world, rank=ctx.rank,
                                            seed=args.seed, synthetic_size=args.synthetic_size,
                                            test_synthetic_size=(args.synthetic_size // 5 if args.synthetic_size else None))
    _apply_runtime_flags(args, (trainloader, testloader))

    say('==> Building model..')
    model = models.build_model(args.model).to(device)
    net = model
    arena = None
    ddp = None
    if ctx.world > 1:
        arena = ParamArena(model.parameters())
        ddp = net = DistributedDataParallel(model, ctx, bucket_cap_mb=args.bucket_mb, arena=arena)
    elif device.type == 'cuda':
        arena = ParamArena(model.parameters())
        net = DataParallel(model, device_ids=[device.index])

    ckpt_path = os.path.join(args.checkpoint_dir, 'ckpt.pth')
    optimizer = SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-4)
    if arena is not None:
        optimizer.attach_arena(arena)
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=args.t_max)
    if args.resume:
        say('==> Resuming from checkpoint..')
        assert os.path.isdir(args.checkpoint_dir), 'Error: no checkpoint directory found!'
        best_acc, start_epoch = load_checkpoint(ckpt_path, net, optimizer, scheduler, map_location=device)
        start_epoch += 1

    trainer = Trainer(net, optimizer, trainloader, testloader, ctx, ddp=ddp,
                      graph=bool(args.graph) and device.type == 'cuda', log_every=args.log_every,
                      progress=progress_bar if is_main else None, max_steps=args.max_steps,
                      nan_guard=not args.no_nan_guard, is_main=is_main)
    prof_cm = None
    if args.profile and is_main:
        from pytorch_cifar_amd.utils.profiling import torch_profile
        prof_cm = torch_profile(args.profile)
        trainer.profiler = prof_cm.__enter__()

    for epoch in range(start_epoch, start_epoch + args.epochs):
        say('\nEpoch: %d' % epoch)
        trainer.train_epoch(epoch)
        _, acc, _, _ = trainer.test_epoch(epoch)
        if trainer.images_per_sec:
            say('Throughput: %.1f img/s' % trainer.images_per_sec)
        if acc > best_acc:
            say('Saving..')
            if is_main:
                save_checkpoint(ckpt_path, net, acc, epoch, optimizer, scheduler)
            best_acc = acc
        scheduler.step()
    if prof_cm is not None:
        prof_cm.__exit__(None, None, None)
        print('Profile trace written to %s' % args.profile)
    ctx.barrier()
    ctx.shutdown()
    return best_acc


if __name__ == '__main__':
    sys.exit(0 if main() is not None else 1)
