"""Bisect helper: SENet18 native-vs-stock gradient check under env toggles (GPU)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import test_ops_gpu as T  # noqa: E402
from pytorch_cifar_amd import models  # noqa: E402

for name in sys.argv[1:] or ["SENet18"]:
    try:
        T.compare_model(models.MODEL_REGISTRY[name])
        print(name, "OK", os.environ.get("PCA_WGRAD_STREAM"), os.environ.get("PCA_CONV_AUTOTUNE"), flush=True)
    except AssertionError as e:
        print(name, "FAIL", os.environ.get("PCA_WGRAD_STREAM"), os.environ.get("PCA_CONV_AUTOTUNE"), str(e)[:300], flush=True)
