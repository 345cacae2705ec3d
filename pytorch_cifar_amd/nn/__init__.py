from . import functional  # noqa: F401
from .modules import AvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, Sequential  # noqa: F401
