"""CIFAR-10 model zoo (parity: reference models/__init__.py:1-18).

Same constructor names and signatures, same module/parameter/buffer names (so state_dicts
interchange with the reference's), every model mapping [N,3,32,32] -> [N,10] logits. The star
import order mirrors the reference, so shadowed helper names resolve the same way
(``Bottleneck`` -> resnet, ``BasicBlock`` -> dla, ``Block``/``SE`` -> regnet, ``cfg`` -> vgg).
"""
from .vgg import *  # noqa: F401,F403
from .dpn import *  # noqa: F401,F403
from .lenet import *  # noqa: F401,F403
from .senet import *  # noqa: F401,F403
from .pnasnet import *  # noqa: F401,F403
from .densenet import *  # noqa: F401,F403
from .googlenet import *  # noqa: F401,F403
from .shufflenet import *  # noqa: F401,F403
from .shufflenetv2 import *  # noqa: F401,F403
from .resnet import *  # noqa: F401,F403
from .resnext import *  # noqa: F401,F403
from .preact_resnet import *  # noqa: F401,F403
from .mobilenet import *  # noqa: F401,F403
from .mobilenetv2 import *  # noqa: F401,F403
from .efficientnet import *  # noqa: F401,F403
from .regnet import *  # noqa: F401,F403
from .dla_simple import *  # noqa: F401,F403
from .dla import *  # noqa: F401,F403
from .dla import BasicBlock  # noqa: F401  (reference: models.BasicBlock is dla's)

# name -> zero-arg constructor for every configuration of the zoo (44 configs)
MODEL_REGISTRY = {
    **{f"VGG{d}": (lambda d=d: VGG(f"VGG{d}")) for d in (11, 13, 16, 19)},  # noqa: F405
    "LeNet": LeNet,  # noqa: F405
    "ResNet18": ResNet18, "ResNet34": ResNet34, "ResNet50": ResNet50,  # noqa: F405
    "ResNet101": ResNet101, "ResNet152": ResNet152,  # noqa: F405
    "PreActResNet18": PreActResNet18, "PreActResNet34": PreActResNet34,  # noqa: F405
    "PreActResNet50": PreActResNet50, "PreActResNet101": PreActResNet101,  # noqa: F405
    "PreActResNet152": PreActResNet152,  # noqa: F405
    "GoogLeNet": GoogLeNet,  # noqa: F405
    "DenseNet121": DenseNet121, "DenseNet169": DenseNet169, "DenseNet201": DenseNet201,  # noqa: F405
    "DenseNet161": DenseNet161, "densenet_cifar": densenet_cifar,  # noqa: F405
    "ResNeXt29_2x64d": ResNeXt29_2x64d, "ResNeXt29_4x64d": ResNeXt29_4x64d,  # noqa: F405
    "ResNeXt29_8x64d": ResNeXt29_8x64d, "ResNeXt29_32x4d": ResNeXt29_32x4d,  # noqa: F405
    "MobileNet": MobileNet, "MobileNetV2": MobileNetV2,  # noqa: F405
    "DPN26": DPN26, "DPN92": DPN92,  # noqa: F405
    "ShuffleNetG2": ShuffleNetG2, "ShuffleNetG3": ShuffleNetG3,  # noqa: F405
    **{f"ShuffleNetV2_{s}": (lambda s=s: ShuffleNetV2(s)) for s in (0.5, 1, 1.5, 2)},  # noqa: F405
    "SENet18": SENet18, "EfficientNetB0": EfficientNetB0,  # noqa: F405
    "RegNetX_200MF": RegNetX_200MF, "RegNetX_400MF": RegNetX_400MF,  # noqa: F405
    "RegNetY_400MF": RegNetY_400MF,  # noqa: F405
    "SimpleDLA": SimpleDLA, "DLA": DLA,  # noqa: F405
    "PNASNetA": PNASNetA, "PNASNetB": PNASNetB,  # noqa: F405
}


def build_model(name: str, **kwargs):
    """Construct a zoo model by name ('ResNet18', 'VGG16', 'ShuffleNetV2_1', ...)."""
    if name in MODEL_REGISTRY and not kwargs:
        return MODEL_REGISTRY[name]()
    g = globals()
    if name.startswith("VGG") and name in ("VGG11", "VGG13", "VGG16", "VGG19"):
        return VGG(name)  # noqa: F405
    if name in g and callable(g[name]):
        return g[name](**kwargs)
    raise KeyError(f"unknown model {name!r}; known: {sorted(MODEL_REGISTRY)}")
