"""Data-parallel engine on CPU ranks (gloo, world_size 2) — the fake-comm-backend strategy of
SURVEY §4 item 3: bucketing, gradient averaging, unused parameters (EfficientNet-B0), rank-0
state/buffer broadcast and DistributedSampler-equivalent sharding, without GPUs."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    from pytorch_cifar_amd.parallel.launcher import init_distributed

    ctx = init_distributed(rank, world, rank, backend="gloo")
    try:
        res = fn(ctx)
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        ctx.shutdown()


def run_ranks(fn, world=2):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, fn, d), nprocs=world, join=True)
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]


# ---------------------------------------------------------------------------- scenarios
def _grad_avg(ctx):
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import cross_entropy
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(100 + ctx.rank)  # different init per rank: DDP must broadcast rank 0's
    model = models.LeNet()
    ddp = DistributedDataParallel(model, ctx, bucket_cap_mb=0.01, first_bucket_mb=0.01)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    xs, ys = x[ctx.rank * 4:(ctx.rank + 1) * 4], y[ctx.rank * 4:(ctx.rank + 1) * 4]
    loss = cross_entropy(ddp(xs), ys)
    loss.backward()
    return {"params": {n: p.detach().clone() for n, p in model.named_parameters()},
            "grads": {n: p.grad.detach().clone() for n, p in model.named_parameters()},
            "buckets": ddp.bucket_sizes_mib(), "x": x, "y": y}


def test_ddp_broadcast_and_gradient_average():
    r0, r1 = run_ranks(_grad_avg)
    for n in r0["params"]:
        torch.testing.assert_close(r0["params"][n], r1["params"][n])  # C3 initial broadcast
        torch.testing.assert_close(r0["grads"][n], r1["grads"][n])    # all-reduced (avg)
    assert len(r0["buckets"]) > 1
    # oracle: mean of the two half-batch gradients computed in one process with rank 0's weights
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import cross_entropy

    m = models.LeNet()
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(r0["params"][n])
    acc = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
    for r in range(2):
        m.zero_grad()
        cross_entropy(m(r0["x"][r * 4:(r + 1) * 4]), r0["y"][r * 4:(r + 1) * 4]).backward()
        for n, p in m.named_parameters():
            acc[n] += p.grad / 2
    for n in acc:
        torch.testing.assert_close(r0["grads"][n], acc[n], rtol=1e-4, atol=1e-6)


def _unused(ctx):
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import cross_entropy
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    model = models.EfficientNetB0()
    ddp = DistributedDataParallel(model, ctx)
    x = torch.randn(2, 3, 32, 32)
    y = torch.randint(0, 10, (2,))
    for _ in range(2):  # the reference's default DDP crashed on the 2nd iteration
        model.zero_grad(set_to_none=False)
        cross_entropy(ddp(x), y).backward()
    unused = sorted(n for n, p in model.named_parameters() if any(p is q for q in ddp.last_unused))
    return {"unused": unused,
            "g": model.layers[0].conv1.weight.grad.abs().max().item(),
            "bn_buf": model.bn1.running_mean.clone()}


def test_ddp_unused_parameters_efficientnet():
    r0, r1 = run_ranks(_unused)
    assert r0["unused"] == ["layers.0.bn1.bias", "layers.0.bn1.weight", "layers.0.conv1.weight"]
    assert r0["g"] == 0.0 and r1["g"] == 0.0


def _buffers(ctx):
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    model = models.ResNet18()
    ddp = DistributedDataParallel(model, ctx)
    x = torch.randn(2, 3, 32, 32) * (1 + ctx.rank)  # different data -> different local BN stats
    ddp(x).sum().backward()
    after_first = model.bn1.running_mean.clone()
    model.eval()  # eval forward: no local running-stat update after the broadcast
    with torch.no_grad():
        ddp(x)  # grad-enabled previous forward -> rank 0's buffers are broadcast first (C4)
    return {"after_first": after_first, "synced": model.bn1.running_mean.clone()}


def test_ddp_broadcast_buffers():
    r0, r1 = run_ranks(_buffers)
    assert not torch.allclose(r0["after_first"], r1["after_first"])  # no SyncBN: local stats
    torch.testing.assert_close(r1["synced"], r0["after_first"])      # rank 0's buffers won


def test_bucket_layout_resnet18():
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.parallel.launcher import DistContext
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    m = models.ResNet18()
    ddp = DistributedDataParallel(m, DistContext())
    sizes = ddp.bucket_sizes_mib()
    assert sizes[0] <= 1.0  # small first bucket: the reduction pipeline starts early in backward
    assert abs(sum(sizes) - sum(p.numel() for p in m.parameters()) * 4 / 2 ** 20) < 0.5
    assert all(s <= 25 for s in sizes)


def test_shard_sampler_matches_torch_distributed_sampler():
    from torch.utils.data.distributed import DistributedSampler

    from pytorch_cifar_amd.data.loader import ShardSampler

    ds = list(range(1003))
    for world in (1, 2, 3, 8):
        for rank in range(world):
            for epoch in (0, 5):
                a = ShardSampler(len(ds), world, rank, shuffle=True, seed=0)
                b = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=0)
                a.set_epoch(epoch)
                b.set_epoch(epoch)
                assert a.indices().tolist() == list(iter(b))


def _train_steps(ctx, compress=None, steps=5):
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.ops.functional import cross_entropy
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(100 + ctx.rank)   # rank 0's initial state must win (C3)
    model = models.LeNet()
    ddp = DistributedDataParallel(model, ctx, bucket_cap_mb=0.01, first_bucket_mb=0.01,
                                  grad_compress=compress)
    opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    g = torch.Generator().manual_seed(11)
    init = {n: p.detach().clone() for n, p in model.named_parameters()}
    batches = []
    for _ in range(steps):
        x = torch.randn(8, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (8,), generator=g)
        batches.append((x, y))
        opt.zero_grad()
        cross_entropy(ddp(x[ctx.rank * 4:(ctx.rank + 1) * 4]), y[ctx.rank * 4:(ctx.rank + 1) * 4]).backward()
        opt.step()
    return {"init": init, "params": {n: p.detach().clone() for n, p in model.named_parameters()},
            "batches": batches}


def _train_steps_bf16(ctx):
    return _train_steps(ctx, compress="bf16")


def test_ddp_steps_bitwise_equal_across_ranks_and_match_single_process():
    """N optimizer steps of 2-rank DDP (LeNet, no BatchNorm): both ranks hold bitwise-identical
    parameters (every rank applies the same averaged gradient), and they match one process
    training on the concatenated batch (reference main_dist.py:140-144 DDP semantics)."""
    r0, r1 = run_ranks(_train_steps)
    for n in r0["params"]:
        assert torch.equal(r0["params"][n], r1["params"][n]), n
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.ops.functional import cross_entropy

    m = models.LeNet()
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(r0["init"][n])
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    for x, y in r0["batches"]:
        opt.zero_grad()
        cross_entropy(m(x), y).backward()
        opt.step()
    for n, p in m.named_parameters():
        torch.testing.assert_close(r0["params"][n], p.detach(), rtol=2e-5, atol=1e-6)


def test_ddp_bf16_compressed_buckets():
    """Opt-in bf16 bucket all-reduce: ranks stay bitwise identical, and the trajectory stays within
    bf16 rounding of the exact fp32 one."""
    c0, c1 = run_ranks(_train_steps_bf16)
    e0, _ = run_ranks(_train_steps)
    ds = []
    for n in c0["params"]:
        assert torch.equal(c0["params"][n], c1["params"][n]), n
        d = ((c0["params"][n] - e0["params"][n]).norm() / e0["params"][n].norm()).item()
        assert d < 1e-2, (n, d)
        ds.append(d)
    assert max(ds) > 0, "the bf16 path was not taken"


def _train_one_step_tail(ctx):
    r = _train_steps(ctx, compress="bf16_tail", steps=1)
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel

    # which parameters the tail bucket (the one whose all-reduce is launched last) holds
    torch.manual_seed(0)
    m = models.LeNet()
    ddp = DistributedDataParallel(m, ctx, bucket_cap_mb=0.01, first_bucket_mb=0.01, grad_compress="bf16_tail")
    names = {id(p): n for n, p in m.named_parameters()}
    r["tail"] = sorted(names[id(p)] for p in ddp.buckets[-1].params)
    r["n_buckets"] = len(ddp.buckets)
    r["low"] = [b.low is not None for b in ddp.buckets]
    return r


def _train_one_step_exact(ctx):
    return _train_steps(ctx, compress=None, steps=1)


def test_ddp_bf16_tail_bucket_only():
    """--grad_compress bf16_tail: only the last bucket (the last all-reduce of the backward, the
    one exposed after it) travels in bf16. After one step, parameters of every other bucket are
    bitwise equal to the exact fp32 run; the tail bucket's differ, by at most bf16 rounding."""
    t0, t1 = run_ranks(_train_one_step_tail)
    e0, _ = run_ranks(_train_one_step_exact)
    assert t0["n_buckets"] > 1
    assert t0["low"] == [False] * (t0["n_buckets"] - 1) + [True]
    for n in t0["params"]:
        assert torch.equal(t0["params"][n], t1["params"][n]), n
    diff_tail = []
    for n in t0["params"]:
        if n in t0["tail"]:
            d = (t0["params"][n] - e0["params"][n]).abs().max().item()
            step = (e0["params"][n] - e0["init"][n]).abs().max().item()
            assert d <= 2 ** -7 * step + 1e-7, (n, d, step)
            diff_tail.append(d)
        else:
            assert torch.equal(t0["params"][n], e0["params"][n]), n
    assert max(diff_tail) > 0, "the tail bucket was not rounded to bf16"


def _tune_sync(ctx):
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.engine.tuning import selection_rows, sync_selection

    lib = _native.lib()
    lib.conv_clear_tuned()
    # each rank "tuned" differently: same geometries, rank-dependent tile / split choices, plus a
    # geometry only rank 1 saw
    rows = [[0] + [64, 32, 32, 64, 128, 3, 3, 1, 1, 1, 32, 32, 0] + [3 + ctx.rank, 1 + ctx.rank],
            [1] + [64, 16, 16, 128, 128, 3, 3, 1, 1, 1, 16, 16, 0] + [35, 8 * (ctx.rank + 1)]]
    if ctx.rank == 1:
        rows.append([0] + [64, 8, 8, 256, 256, 3, 3, 1, 1, 1, 8, 8, 0] + [12, 1])
    lib.tune_import(rows)
    before = selection_rows(lib)
    h = sync_selection(ctx, lib)
    return {"before": before, "after": selection_rows(lib), "hash": h}


def test_rank_consistent_kernel_selection():
    """Ranks that autotuned to different kernel choices adopt rank 0's selection (engine/tuning.py
    sync_selection): identical tables and selection hashes afterwards (reference main_dist.py:
    140-147, replicated model under cudnn.benchmark)."""
    r0, r1 = run_ranks(_tune_sync)
    assert r0["before"] != r1["before"]
    assert r0["after"] == r1["after"] == r0["before"]
    assert r0["hash"] == r1["hash"]
