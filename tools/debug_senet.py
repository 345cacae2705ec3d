"""SENet18 native-vs-stock gradient check (GPU): per-parameter relative error against the fp32
CPU oracle for the native and the stock-bf16 paths, over a few seeds, in the zoo-test settings
(static tile heuristic, deterministic reductions). Prints every parameter whose native error is
above 2x stock's, in backward order, so the first layer where the native path drifts shows up."""
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import test_ops_gpu as T  # noqa: E402
from pytorch_cifar_amd import _native, models  # noqa: E402

C = _native.lib()
C.conv_autotune(False)
C.conv_clear_tuned()
C.set_deterministic(os.environ.get("DBG_DET", "1") == "1")
name = sys.argv[1] if len(sys.argv) > 1 else "SENet18"
for seed in range(int(os.environ.get("DBG_SEEDS", "3"))):
    torch.manual_seed(seed)
    ref = models.MODEL_REGISTRY[name]()
    native = copy.deepcopy(ref).cuda()
    stock = copy.deepcopy(ref).cuda()
    x = torch.randn(32, 3, 32, 32)
    y = torch.randint(0, 10, (32,))
    o_r = T._run(ref, x, y, "cpu")
    o_n = T._run(native, x, y, "cuda")
    o_s = T._run(stock, x, y, "cuda", stock=True)
    print(f"seed {seed}: logits native {T.rel(o_n, o_r):.4f} stock {T.rel(o_s, o_r):.4f}", flush=True)
    gr, gn, gs = T._grads(ref), T._grads(native), T._grads(stock)
    rows = []
    for n, g in gr.items():
        if g is None:
            continue
        en, es = T.rel(gn[n], g), T.rel(gs[n], g)
        rows.append((n, en, es))
    for n, en, es in reversed(rows):
        flag = " <<" if en > 2 * es + 0.01 else ""
        if "fc" in n or flag:
            print(f"  {n:32s} native {en:.4f} stock {es:.4f}{flag}", flush=True)
