"""Reference-compatible ``models`` package: ``from models import *`` exposes the same
constructors as the reference's models/__init__.py, implemented by pytorch_cifar_amd.models."""
from pytorch_cifar_amd.models import *  # noqa: F401,F403
from pytorch_cifar_amd.models import MODEL_REGISTRY, build_model  # noqa: F401
