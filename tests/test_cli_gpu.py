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
