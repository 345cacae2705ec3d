#!/usr/bin/env python3
'''Distributed CIFAR10 training on MI355X — CLI parity with the reference main_dist.py.

Reference flags (main_dist.py:25-46): --lr 0.1, --batch_size 512 (global), --epochs 100,
--output_dir (required), --resume/-r, --workers 4, --world_size -1, --rank -1, --dist_url,
--dist, --amp. Additive: --model (default ResNet152 as main_dist.py:136), --t_max (200),
--data_dir, --synthetic, --seed, --graph, --max_steps, --bucket_mb, --log_every, --no_broadcast_buffers.

Launch modes:
  torchrun --nproc-per-node N main_dist.py ...      one process per GPU (RANK/WORLD_SIZE env)
  python main_dist.py --dist ...                    spawns one process per visible GPU
                                                    (nodes = --world_size, node rank = --rank;
                                                    both default to 1/0 instead of -1)
  python main_dist.py ...                           one rank per visible GPU, spawned here
                                                    (reference: single-process DataParallel)

Per-rank batch = batch_size / world_size (main_dist.py:111). Gradients are averaged with bucketed
RCCL all-reduces overlapped with backward; BN buffers follow DDP's broadcast_buffers semantics;
EfficientNet-B0's unused parameters are handled (the reference's DDP crashed on them).
--amp is accepted for parity: the GPU path always computes in bf16 (no loss scaling needed).
'''
import argparse
import logging
import os
import sys

import torch
import torch.multiprocessing as mp

from pytorch_cifar_amd import models
from pytorch_cifar_amd.data.factory import build_loaders
from pytorch_cifar_amd.engine.arena import ParamArena
from pytorch_cifar_amd.engine.checkpoint import load_checkpoint, save_checkpoint
from pytorch_cifar_amd.engine.optim import SGD
from pytorch_cifar_amd.engine.trainer import Trainer
from pytorch_cifar_amd.parallel import launcher
from pytorch_cifar_amd.parallel.data_parallel import DataParallel
from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel
from utils import set_logger

parser = argparse.ArgumentParser(description='PyTorch CIFAR10 Training (MI355X-native, distributed)')
parser.add_argument('--lr', default=0.1, type=float, help='learning rate')
parser.add_argument('--batch_size', default=512, type=int, help='batch size')
parser.add_argument('--epochs', default=100, type=int, help='number of training epochs')
parser.add_argument('--output_dir', required=True, type=str, help='output directory')
parser.add_argument('--resume', '-r', action='store_true', help='resume from checkpoint')
parser.add_argument('--workers', default=4, type=int, help='accepted for parity (data is GPU-resident)')
parser.add_argument('--world_size', default=-1, type=int, help='number of nodes for distributed training')
parser.add_argument('--rank', default=-1, type=int, help='node rank for distributed training')
parser.add_argument('--dist_url', default='tcp://127.0.0.1:23456', type=str,
                    help='url used to set up distributed training')
parser.add_argument('--dist', action='store_true',
                    help='launch one process per GPU on this node (mp.spawn)')
parser.add_argument('--amp', action='store_true', default=False)
parser.add_argument('--model', default='ResNet152')
parser.add_argument('--t_max', default=200, type=int)
parser.add_argument('--data_dir', default='./data')
parser.add_argument('--synthetic', action='store_true')
parser.add_argument('--synthetic_size', default=None, type=int)
parser.add_argument('--seed', default=0, type=int)
parser.add_argument('--graph', default=1, type=int)
parser.add_argument('--max_steps', default=None, type=int)
parser.add_argument('--bucket_mb', default=4.0, type=float,
                    help='gradient all-reduce bucket size (MiB); small buckets overlap backward on xGMI')
parser.add_argument('--grad_compress', default='none', choices=['none', 'bf16', 'bf16_tail'],
                    help='opt-in bf16 gradient all-reduce (every bucket, or only the exposed last one)')
parser.add_argument('--log_every', default=20, type=int)
parser.add_argument('--no_broadcast_buffers', action='store_true')
parser.add_argument('--cpu', action='store_true', help='gloo/CPU ranks (tests)')
parser.add_argument('--nproc', default=None, type=int,
                    help='ranks for the non---dist path (default: every visible GPU, one process each)')
parser.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'],
                    help='bf16: native MI355X kernels; fp32: stock PyTorch fp32 kernels on the GPU')
parser.add_argument('--deterministic', action='store_true', help='bitwise-reproducible weight gradients')
parser.add_argument('--debug_sync', action='store_true',
                    help='sync + error-check after every native op (locates async GPU faults; disables graphs)')
parser.add_argument('--profile', default=None, metavar='TRACE.json',
                    help='torch.profiler Chrome trace of the first training steps')
parser.add_argument('--no_nan_guard', action='store_true', help='do not stop on a non-finite loss')

best_acc = 0



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

def main(argv=None):
    args = parser.parse_args(argv)
    if launcher.spawned_world() > 1 and not args.dist:
        ctx = launcher.init_from_env(backend='gloo' if args.cpu else 'nccl')
        return main_worker(ctx, args)
    if args.dist:
        ngpus = 1 if args.cpu else torch.cuda.device_count()
        nodes = args.world_size if args.world_size > 0 else 1
        args.world_size = ngpus * nodes
        args.node_rank = args.rank if args.rank >= 0 else 0
        mp.spawn(_spawn_entry, nprocs=ngpus, args=(ngpus, args))
        return 0
    nranks = args.nproc if args.nproc else (0 if args.cpu else torch.cuda.device_count())
    if nranks > 1:
        # reference non---dist path (README / train.sh): nn.DataParallel over every visible GPU
        # (main_dist.py:145-147) with the global batch split across them. Here: one rank process
        # per GPU on the native RCCL bucket engine, started fresh (never an exec of this process).
        argv = list(sys.argv[1:] if argv is None else argv)
        rc = launcher.spawn_local_ranks(nranks, [os.path.abspath(__file__)] + argv)
        if rc:
            raise SystemExit(rc)
        return 0.0
    ctx = launcher.DistContext(device=torch.device('cuda' if torch.cuda.is_available() and not args.cpu else 'cpu'))
    if ctx.device.type == 'cuda':
        torch.cuda.set_device(0)
        ctx.device = torch.device('cuda', 0)
    return main_worker(ctx, args)


def _spawn_entry(gpu, ngpus, args):
    rank = args.node_rank * ngpus + gpu
    ctx = launcher.init_distributed(rank, args.world_size, gpu, backend='gloo' if args.cpu else 'nccl',
                                    init_method=args.dist_url)
    main_worker(ctx, args)


def main_worker(ctx, args):
    global best_acc
    start_epoch = 0
    device = ctx.device
    torch.manual_seed(args.seed)
    if ctx.rank == 0 and not os.path.isdir(args.output_dir):
        os.makedirs(args.output_dir, exist_ok=True)
    ctx.barrier()
    set_logger(os.path.join(args.output_dir, 'train.log'), rank=ctx.rank)

    print('==> Preparing data..')
    batch_size = args.batch_size // ctx.world
    if args.batch_size % ctx.world:
        logging.info('Batch size {} is not a multiple of number of total GPUS {}.'.format(args.batch_size, ctx.world))
        logging.info('Batch size {} per GPU and total {} will be applied instead.'.format(batch_size, batch_size * ctx.world))
    trainloader, testloader = build_loaders(args.data_dir, args.synthetic, batch_size, batch_size, device,
                                            world=ctx.world, rank=ctx.rank, crop_pad=0, flip=True,
                                            seed=args.seed, synthetic_size=args.synthetic_size,
                                            test_synthetic_size=(args.synthetic_size // 5 if args.synthetic_size else None))
    _apply_runtime_flags(args, (trainloader, testloader))

    print('==> Building model..')
    model = models.build_model(args.model).to(device)
    ddp = None
    arena = None
    if ctx.world > 1:
        arena = ParamArena(model.parameters())
        ddp = DistributedDataParallel(model, ctx, bucket_cap_mb=args.bucket_mb, arena=arena,
                                      broadcast_buffers=not args.no_broadcast_buffers,
                                      grad_compress=args.grad_compress)
        net = ddp
    else:
        if device.type == 'cuda':
            arena = ParamArena(model.parameters())
        net = DataParallel(model, device_ids=[device.index] if device.type == 'cuda' else [])

    optimizer = SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-4)
    if arena is not None:
        optimizer.attach_arena(arena)
    scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=args.t_max)

    ckpt = os.path.join(args.output_dir, 'ckpt.pth')
    if args.resume:
        print('==> Resuming from checkpoint..')
        legacy = os.path.join('checkpoint', 'ckpt.pth')
        path = ckpt if os.path.exists(ckpt) else legacy
        assert os.path.exists(path), 'Error: no checkpoint found!'
        best_acc, start_epoch = load_checkpoint(path, net, optimizer, scheduler, map_location=device)
        start_epoch += 1

    tqdm_progress = None
    if ctx.rank == 0:
        from utils import progress_bar
        tqdm_progress = progress_bar
    trainer = Trainer(net, optimizer, trainloader, testloader, ctx, ddp=ddp,
                      graph=bool(args.graph) and device.type == 'cuda', log_every=args.log_every,
                      progress=tqdm_progress, max_steps=args.max_steps, nan_guard=not args.no_nan_guard)
    prof_cm = None
    if args.profile and ctx.rank == 0:
        from pytorch_cifar_amd.utils.profiling import torch_profile
        prof_cm = torch_profile(args.profile)
        trainer.profiler = prof_cm.__enter__()

    logging.info("Start training...")
    for epoch in range(start_epoch, args.epochs):
        print('\nEpoch: %d' % epoch)
        logging.info('Epoch: %d' % epoch)
        loss, acc, correct, total = trainer.train_epoch(epoch)
        logging.info('Train Loss: %.3f | Acc: %.3f%% (%d/%d)' % (loss, acc, correct, total))
        if trainer.images_per_sec:
            logging.info('Throughput: %.1f img/s (all ranks)' % trainer.images_per_sec)
        loss, acc, correct, total = trainer.test_epoch(epoch)
        logging.info('Eval Loss: %.3f | Acc: %.3f%% (%d/%d)' % (loss, acc, correct, total))
        if acc > best_acc:
            logging.info("- Found new best accuracy")
            if ctx.rank == 0:
                print('Saving..')
                save_checkpoint(ckpt, net, acc, epoch, optimizer, scheduler)
            best_acc = acc
        scheduler.step()
    if prof_cm is not None:
        prof_cm.__exit__(None, None, None)
        logging.info('Profile trace written to %s' % args.profile)
    ctx.barrier()
    ctx.shutdown()
    return best_acc


if __name__ == '__main__':
    sys.exit(0 if main() is not None else 1)
