"""ResNet family with torchvision-compatible module names, shapes and initialisation.

The reference builds its models with ``torchvision.models.__dict__[arch]()``
(`dataparallel.py:112-117`, `distributed.py:132-137`, `distributed_syncBN_amp.py:135-140`)
and saves ``model.module.state_dict()`` (`distributed.py:212-218`).  torchvision is not
installed in this image, so the architectures are defined here with the exact same
parameter/buffer names (``conv1.weight``, ``bn1.running_mean``, ``layer1.0.conv1.weight``,
``layer2.0.downsample.0.weight``, ``fc.bias`` ...) so checkpoints are interchangeable.

On a GPU the module is executed by the native ResNet executor
(:mod:`pytorch_distributed_template_amd.models.executor`), which runs our HIP kernels
(implicit-GEMM MFMA convolutions, fused BN/ReLU/residual, pooling, loss) in NHWC with
explicit forward/backward.  On the CPU the plain ``forward`` below is the reference path.
"""
from __future__ import annotations

import math
from typing import List, Optional, Type, Union

import torch
import torch.nn as nn


def conv3x3(in_planes: int, out_planes: int, stride: int = 1, groups: int = 1, dilation: int = 1) -> nn.Conv2d:
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                     groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes: int, out_planes: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 groups: int = 1, base_width: int = 64, dilation: int = 1, norm_layer=None) -> None:
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        if groups != 1 or base_width != 64:
            raise ValueError("BasicBlock only supports groups=1 and base_width=64")
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 groups: int = 1, base_width: int = 64, dilation: int = 1, norm_layer=None) -> None:
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, groups: int = 1, width_per_group: int = 64,
                 replace_stride_with_dilation: Optional[List[bool]] = None, norm_layer=None) -> None:
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.dilation = 1
        if replace_stride_with_dilation is None:
            replace_stride_with_dilation = [False, False, False]
        self.groups = groups
        self.base_width = width_per_group
        self.block_type = block.__name__
        self.layers_cfg = list(layers)
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2, dilate=replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2, dilate=replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2, dilate=replace_stride_with_dilation[2])
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck) and m.bn3.weight is not None:
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock) and m.bn2.weight is not None:
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1, dilate: bool = False) -> nn.Sequential:
        norm_layer = self._norm_layer
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width,
                        previous_dilation, norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                dilation=self.dilation, norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def forward_reference(self, x: torch.Tensor) -> torch.Tensor:
        """Plain PyTorch forward (CPU reference / numerics oracle)."""
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_reference(x)


def _resnet(block, layers, pretrained: bool = False, **kwargs) -> ResNet:
    model = ResNet(block, layers, **kwargs)
    return model


def resnet18(pretrained: bool = False, **kwargs) -> ResNet:
    return _resnet(BasicBlock, [2, 2, 2, 2], pretrained, **kwargs)


def resnet34(pretrained: bool = False, **kwargs) -> ResNet:
    return _resnet(BasicBlock, [3, 4, 6, 3], pretrained, **kwargs)


def resnet50(pretrained: bool = False, **kwargs) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 6, 3], pretrained, **kwargs)


def resnet101(pretrained: bool = False, **kwargs) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 23, 3], pretrained, **kwargs)


def resnet152(pretrained: bool = False, **kwargs) -> ResNet:
    return _resnet(Bottleneck, [3, 8, 36, 3], pretrained, **kwargs)


def resnext50_32x4d(pretrained: bool = False, **kwargs) -> ResNet:
    kwargs.update(groups=32, width_per_group=4)
    return _resnet(Bottleneck, [3, 4, 6, 3], pretrained, **kwargs)


def resnext101_32x8d(pretrained: bool = False, **kwargs) -> ResNet:
    kwargs.update(groups=32, width_per_group=8)
    return _resnet(Bottleneck, [3, 4, 23, 3], pretrained, **kwargs)


def resnext101_64x4d(pretrained: bool = False, **kwargs) -> ResNet:
    kwargs.update(groups=64, width_per_group=4)
    return _resnet(Bottleneck, [3, 4, 23, 3], pretrained, **kwargs)


def wide_resnet50_2(pretrained: bool = False, **kwargs) -> ResNet:
    kwargs.update(width_per_group=64 * 2)
    return _resnet(Bottleneck, [3, 4, 6, 3], pretrained, **kwargs)


def wide_resnet101_2(pretrained: bool = False, **kwargs) -> ResNet:
    kwargs.update(width_per_group=64 * 2)
    return _resnet(Bottleneck, [3, 4, 23, 3], pretrained, **kwargs)
