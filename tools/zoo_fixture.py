#!/usr/bin/env python3
"""Write tests/fixtures/zoo_contract.json: the model zoo's state_dict contract and fp64 digests.

For every constructor in MODEL_REGISTRY the fixture pins
  * the ordered state_dict keys with their shapes (the reference's checkpoint contract,
    /root/reference/models/*.py attribute names; ckpt.pth['net'] layout, main.py:137-148), and
  * an fp64 digest of one seeded forward/backward on the CPU path (logits, input-gradient norm,
    per-parameter gradient norms) as a regression pin.

Provenance: the fixture was generated from this repo's models at a commit whose test suite
asserted, model by model, identical keys/shapes with the reference package and fp64 forward /
backward agreement to 1e-12 / 1e-10 (round-4 tests/test_models_cpu.py, which imported the
reference read-only). The test suite itself no longer executes any reference code.

  python tools/zoo_fixture.py            # regenerate (only after an intended contract change)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "fixtures", "zoo_contract.json")

# models whose fp64 digest is pinned (the CPU suite runs one fp64 step of each)
DIGEST = [
    "VGG11", "LeNet", "ResNet18", "PreActResNet18", "GoogLeNet", "densenet_cifar",
    "ResNeXt29_32x4d", "MobileNet", "MobileNetV2", "DPN26", "SENet18", "EfficientNetB0",
    "RegNetX_200MF", "RegNetY_400MF", "SimpleDLA", "DLA", "PNASNetA", "PNASNetB",
    "ShuffleNetV2_0.5", "ShuffleNetG2",
]

HEAVY = ["ResNet101", "ResNet152", "PreActResNet34", "PreActResNet101", "PreActResNet152",
         "DenseNet169", "DenseNet201", "DenseNet161", "ResNeXt29_4x64d", "ResNeXt29_8x64d",
         "DPN92", "ShuffleNetV2_1.5", "ShuffleNetV2_2"]


def digest(name: str) -> dict:
    from pytorch_cifar_amd import models

    torch.manual_seed(0)
    m = models.MODEL_REGISTRY[name]().double().train()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(3, 3, 32, 32, generator=g, dtype=torch.float64).requires_grad_(True)
    gy = torch.randn(3, 10, generator=g, dtype=torch.float64)
    torch.manual_seed(2)   # dropout masks (EfficientNet-B0)
    y = m(x)
    y.backward(gy)
    return {
        "logits": [float(v) for v in y.detach().flatten()],
        "gx_norm": float(x.grad.norm()),
        "gp_norm": {n: float(p.grad.norm()) for n, p in m.named_parameters() if p.grad is not None},
    }


def main():
    from pytorch_cifar_amd import models

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    out = {}
    for name in models.MODEL_REGISTRY:
        torch.manual_seed(0)
        sd = models.MODEL_REGISTRY[name]().state_dict()
        keys = [f"{k}:{'x'.join(map(str, v.shape))}" for k, v in sd.items()]
        # deep variants (ResNet152, DenseNet201, ...) pin a hash of the list; the rest list it
        ent = ({"keys_sha256": hashlib.sha256("\n".join(keys).encode()).hexdigest(), "n_keys": len(keys)}
               if name in HEAVY else {"keys": keys})
        if name in DIGEST:
            ent["fp64"] = digest(name)
        out[name] = ent
        print(name, len(sd), flush=True)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
