"""Model registry by name (reference: `dataparallel.py:36-37` builds ``--arch`` choices from every
lowercase callable in ``torchvision.models``; `:112-117` instantiates ``models.__dict__[arch]()``).

torchvision is not available offline here, so the registry is ours, with torchvision-identical
parameter names, shapes and initialisation: ResNet / ResNeXt / Wide-ResNet (native executor on GPU),
AlexNet, VGG (with and without BN), SqueezeNet, DenseNet, MobileNetV2/V3, ShuffleNetV2, MNASNet, EfficientNet-B0..B7,
GoogLeNet, Inception-v3, EfficientNetV2, RegNet-X/Y, ConvNeXt, ViT, Swin V1/V2 and MaxViT (stock-PyTorch engine).  ``pretrained=True`` loads weights
from a LOCAL torchvision-format checkpoint (``--pretrained-path`` or ``$PDT_PRETRAINED_DIR/<arch>.pth``)
with the safe ``weights_only`` loader -- the GPU box has no network.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional

import torch

from . import classic, efficient, inception, mobile, modern, resnet

_REGISTRY: Dict[str, Callable[..., torch.nn.Module]] = {
    "resnet18": resnet.resnet18,
    "resnet34": resnet.resnet34,
    "resnet50": resnet.resnet50,
    "resnet101": resnet.resnet101,
    "resnet152": resnet.resnet152,
    "resnext50_32x4d": resnet.resnext50_32x4d,
    "resnext101_32x8d": resnet.resnext101_32x8d,
    "resnext101_64x4d": resnet.resnext101_64x4d,
    "wide_resnet50_2": resnet.wide_resnet50_2,
    "wide_resnet101_2": resnet.wide_resnet101_2,
    "alexnet": classic.alexnet,
    "vgg11": classic.vgg11, "vgg11_bn": classic.vgg11_bn, "vgg13": classic.vgg13, "vgg13_bn": classic.vgg13_bn,
    "vgg16": classic.vgg16, "vgg16_bn": classic.vgg16_bn, "vgg19": classic.vgg19, "vgg19_bn": classic.vgg19_bn,
    "squeezenet1_0": classic.squeezenet1_0, "squeezenet1_1": classic.squeezenet1_1,
    "densenet121": mobile.densenet121, "densenet161": mobile.densenet161, "densenet169": mobile.densenet169,
    "densenet201": mobile.densenet201,
    "mobilenet_v2": mobile.mobilenet_v2,
    "shufflenet_v2_x0_5": mobile.shufflenet_v2_x0_5, "shufflenet_v2_x1_0": mobile.shufflenet_v2_x1_0,
    "shufflenet_v2_x1_5": mobile.shufflenet_v2_x1_5, "shufflenet_v2_x2_0": mobile.shufflenet_v2_x2_0,
    "googlenet": inception.googlenet, "inception_v3": inception.inception_v3,
    "mnasnet0_5": efficient.mnasnet0_5, "mnasnet0_75": efficient.mnasnet0_75, "mnasnet1_0": efficient.mnasnet1_0,
    "mnasnet1_3": efficient.mnasnet1_3,
    "mobilenet_v3_large": efficient.mobilenet_v3_large, "mobilenet_v3_small": efficient.mobilenet_v3_small,
    **efficient.EFFICIENTNETS,
    **modern.MODERN,
}


def register(name: str, fn: Callable[..., torch.nn.Module]) -> None:
    if not name.islower():
        raise ValueError("model names are lowercase (torchvision convention)")
    _REGISTRY[name] = fn


def model_names() -> List[str]:
    return sorted(_REGISTRY)


def resolution_kwargs(arch: str, size: int) -> dict:
    """Constructor kwargs for the fixed-resolution archs (ViT position table, MaxViT partition grid) at a
    ``size`` x ``size`` crop; empty for the resolution-agnostic CNNs."""
    if arch.startswith("vit_"):
        return {"image_size": size}
    if arch == "maxvit_t":
        # stem (stride 2) then four stride-2 stages: the block / grid partition must tile EVERY stage's map
        maps, g = [], size
        for i in range(5):
            g = (g - 1) // 2 + 1
            if i >= 1:
                maps.append(g)
        fits = [d for d in range(2, 8) if all(m % d == 0 for m in maps)]
        if not fits:
            raise ValueError(f"maxvit_t: a {size}px crop gives stage maps {maps}; no partition size in 2..7 divides "
                             f"them all (use a multiple of 32, e.g. 224)")
        return {"input_size": (size, size), "partition_size": max(fits)}
    return {}


def create(arch: str, pretrained: bool = False, pretrained_path: Optional[str] = None, **kwargs) -> torch.nn.Module:
    if arch not in _REGISTRY:
        raise KeyError(f"unknown arch {arch!r}; choices: {model_names()}")
    if pretrained and (arch.startswith("vit_") or arch == "maxvit_t"):
        # position tables / relative-position biases are sized for the 224 crop the torchvision weights use
        if kwargs.get("image_size", 224) != 224 or tuple(kwargs.get("input_size", (224, 224))) != (224, 224):
            raise ValueError(f"--pretrained {arch} weights are for 224x224 crops; got {kwargs}")
    model = _REGISTRY[arch](**kwargs)
    if pretrained:
        path = pretrained_path or os.path.join(os.environ.get("PDT_PRETRAINED_DIR", "pretrained"), f"{arch}.pth")
        if not os.path.exists(path):
            raise FileNotFoundError(f"--pretrained needs local weights (no network): {path} not found")
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd:
            sd = sd["state_dict"]
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
        model.load_state_dict(sd)
    return model
