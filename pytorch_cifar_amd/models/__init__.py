"""CIFAR-10 model zoo (parity: reference models/__init__.py:1-18, same constructor names)."""
from .resnet import *  # noqa: F401,F403
