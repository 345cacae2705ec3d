"""Entry points on the GPU: main.py (single process, hipGraph step) and main_dist.py under
torchrun with one rank over RCCL, plus the native RCCL communicator on a 1-rank clique."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, timeout=400):
    env = dict(os.environ, PYTHONPATH=ROOT, PCA_NO_AUTOBUILD="1")
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout + r.stderr


def test_main_py_gpu(tmp_path):
    out = _run([os.path.join(ROOT, "main.py"), "--model", "ResNet18", "--epochs", "1",
                "--synthetic", "--synthetic_size", "4096", "--max_steps", "8",
                "--checkpoint_dir", str(tmp_path / "ck")], cwd=str(tmp_path))
    assert "Saving.." in out, out[-2000:]


def test_main_dist_one_rank_rccl(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    _run(["-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
          "--master-addr", "127.0.0.1", "--master-port", str(port),
          os.path.join(ROOT, "main_dist.py"), "--model", "ResNet18", "--epochs", "1",
          "--synthetic", "--synthetic_size", "4096", "--max_steps", "8", "--batch_size", "512",
          "--output_dir", str(tmp_path / "o")], cwd=str(tmp_path))
    assert os.path.exists(tmp_path / "o" / "ckpt.pth")
    assert "Eval Loss" in open(tmp_path / "o" / "train.log").read()


def test_native_rccl_single_rank():
    from pytorch_cifar_amd import _native

    C = _native.lib()
    uid = C.rccl_unique_id()
    comm = C.RcclComm(uid, 1, 0, 0)  # (unique_id, world, rank, device)
    t = torch.arange(1000, device="cuda", dtype=torch.float32)
    ref = t.clone()
    comm.all_reduce(t, "sum", torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(t, ref)
    comm.all_reduce(t, "avg", torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(t, ref)
    comm.destroy()


def test_main_py_gpu_fp32_and_deterministic(tmp_path):
    out = _run([os.path.join(ROOT, "main.py"), "--model", "ResNet18", "--epochs", "1",
                "--synthetic", "--synthetic_size", "2048", "--max_steps", "4", "--dtype", "fp32",
                "--checkpoint_dir", str(tmp_path / "a")], cwd=str(tmp_path))
    assert "Saving.." in out, out[-2000:]
    out = _run([os.path.join(ROOT, "main.py"), "--model", "ResNet18", "--epochs", "1",
                "--synthetic", "--synthetic_size", "2048", "--max_steps", "4", "--deterministic",
                "--debug_sync", "--checkpoint_dir", str(tmp_path / "b")], cwd=str(tmp_path))
    assert "Saving.." in out, out[-2000:]


def test_ddp_rccl_inside_hipgraph_matches_eager():
    """The multi-GPU step path on a 1-rank RCCL clique: bucketed all-reduces issued from the
    gradient-ready hooks on the comm stream, captured into the step's hipGraph together with the
    backward, must leave parameters identical to the same steps without the data-parallel engine
    (a world-1 average is the identity). This is the code the 8-GPU bench replays."""
    from pytorch_cifar_amd import _native, models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep
    from pytorch_cifar_amd.parallel.ddp import DistributedDataParallel
    from pytorch_cifar_amd.parallel.launcher import DistContext

    import pytorch_cifar_amd

    C = _native.lib()
    pytorch_cifar_amd.set_deterministic(True)   # bitwise-comparable weight gradients
    comm = C.RcclComm(C.rccl_unique_id(), 1, 0, 0)
    ctx = DistContext(rank=0, world=1, local_rank=0, device=torch.device("cuda", 0),
                      backend="nccl", comm=comm)
    imgs, labs = synthetic_cifar10(256, seed=5)
    finals = []
    for use_ddp in (False, True):
        torch.manual_seed(0)
        model = models.ResNet18().cuda()
        arena = ParamArena(model.parameters())
        opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
        net, ddp = model, None
        if use_ddp:
            ddp = DistributedDataParallel(model, ctx, bucket_cap_mb=4.0, arena=arena,
                                          force_collectives=True)
            net = ddp
            assert len(ddp.buckets) > 2
        loader = DeviceLoader(imgs, labs, 64, "cuda", crop_pad=4, flip=True, drop_last=True, seed=0)
        step = TrainStep(net, opt, loader, 64, ddp=ddp, graph=True)
        loader.set_epoch(0)
        for idx in loader.batch_indices():
            step(idx)
        torch.cuda.synchronize()
        assert step.graph is not None, f"graph capture failed: {step.graph_error!r}"
        finals.append(arena.param_flat.detach().clone())
    comm.destroy()
    pytorch_cifar_amd.set_deterministic(False)
    # same seeds -> same batches and augmentation draws; deterministic wgrad and a world-1 average
    # (sum / 1) make the two runs bitwise comparable
    torch.testing.assert_close(finals[1], finals[0], rtol=0, atol=0)


def test_graph_steps_equal_eager_steps():
    """the hipGraph warm-up bodies must not leak into training state. N captured
    steps leave parameters, momenta, BN running stats and the metrics buffer where N eager
    steps leave them (no augmentation randomness: crop 0, flip off)."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep

    import pytorch_cifar_amd

    pytorch_cifar_amd.set_deterministic(True)
    imgs, labs = synthetic_cifar10(256, seed=7)
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        model = models.ResNet18().cuda()
        arena = ParamArena(model.parameters())
        opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
        loader = DeviceLoader(imgs, labs, 64, "cuda", crop_pad=0, flip=False, drop_last=True, seed=0)
        step = TrainStep(model, opt, loader, 64, graph=graph)
        loader.set_epoch(0)
        for idx in loader.batch_indices():
            step(idx)
        torch.cuda.synchronize()
        if graph:
            assert step.graph is not None, f"graph capture failed: {step.graph_error!r}"
        runs.append((arena.param_flat.clone(), arena.mom_flat.clone(),
                     model.bn1.running_mean.clone(), int(model.bn1.num_batches_tracked),
                     step.metrics.clone()))
    pytorch_cifar_amd.set_deterministic(False)
    (p0, m0, r0, n0, k0), (p1, m1, r1, n1, k1) = runs
    assert n0 == n1 == 4
    torch.testing.assert_close(k1, k0, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(r1, r0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(p1, p0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m1, m0, rtol=1e-5, atol=1e-6)
