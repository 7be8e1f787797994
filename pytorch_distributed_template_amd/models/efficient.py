"""MNASNet, MobileNetV3, EfficientNet-B0..B7 and EfficientNetV2-S/M/L with torchvision-identical module names, shapes and init.

Registry members (reference C05, `dataparallel.py:36-37`); executed by the stock-PyTorch engine.
"""
from __future__ import annotations

import copy
import math
from functools import partial
from typing import Callable, List, Optional

import torch
import torch.nn as nn

# ------------------------------------------------------------------------------------------ MNASNet
_MNAS_BN_MOMENTUM = 1 - 0.9997  # TensorFlow's 0.9997 decay in PyTorch's convention


class _MnasInvertedResidual(nn.Module):
    def __init__(self, in_ch: int, out_ch: int, kernel_size: int, stride: int, expansion: int,
                 bn_momentum: float = 0.1):
        super().__init__()
        mid = in_ch * expansion
        self.apply_residual = in_ch == out_ch and stride == 1
        self.layers = nn.Sequential(
            nn.Conv2d(in_ch, mid, 1, bias=False), nn.BatchNorm2d(mid, momentum=bn_momentum), nn.ReLU(inplace=True),
            nn.Conv2d(mid, mid, kernel_size, padding=kernel_size // 2, stride=stride, groups=mid, bias=False),
            nn.BatchNorm2d(mid, momentum=bn_momentum), nn.ReLU(inplace=True),
            nn.Conv2d(mid, out_ch, 1, bias=False), nn.BatchNorm2d(out_ch, momentum=bn_momentum))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.layers(x) + x if self.apply_residual else self.layers(x)


def _mnas_stack(in_ch: int, out_ch: int, kernel_size: int, stride: int, expansion: int, repeats: int,
                bn_momentum: float) -> nn.Sequential:
    blocks = [_MnasInvertedResidual(in_ch, out_ch, kernel_size, stride, expansion, bn_momentum)]
    blocks += [_MnasInvertedResidual(out_ch, out_ch, kernel_size, 1, expansion, bn_momentum)
               for _ in range(repeats - 1)]
    return nn.Sequential(*blocks)


def _round_to_multiple_of(val: float, divisor: int, round_up_bias: float = 0.9) -> int:
    new_val = max(divisor, int(val + divisor / 2) // divisor * divisor)
    return new_val if new_val >= round_up_bias * val else new_val + divisor


class MNASNet(nn.Module):
    """MNASNet-B1 with depth multiplier ``alpha``."""

    def __init__(self, alpha: float, num_classes: int = 1000, dropout: float = 0.2):
        super().__init__()
        self.alpha = alpha
        d = [_round_to_multiple_of(c * alpha, 8) for c in (32, 16, 24, 40, 80, 96, 192, 320)]
        m = _MNAS_BN_MOMENTUM
        layers = [
            nn.Conv2d(3, d[0], 3, padding=1, stride=2, bias=False), nn.BatchNorm2d(d[0], momentum=m),
            nn.ReLU(inplace=True),
            nn.Conv2d(d[0], d[0], 3, padding=1, stride=1, groups=d[0], bias=False), nn.BatchNorm2d(d[0], momentum=m),
            nn.ReLU(inplace=True),
            nn.Conv2d(d[0], d[1], 1, padding=0, stride=1, bias=False), nn.BatchNorm2d(d[1], momentum=m),
            # (out, kernel, stride, expansion, repeats) per stage
            _mnas_stack(d[1], d[2], 3, 2, 3, 3, m), _mnas_stack(d[2], d[3], 5, 2, 3, 3, m),
            _mnas_stack(d[3], d[4], 5, 2, 6, 3, m), _mnas_stack(d[4], d[5], 3, 1, 6, 2, m),
            _mnas_stack(d[5], d[6], 5, 2, 6, 4, m), _mnas_stack(d[6], d[7], 3, 1, 6, 1, m),
            nn.Conv2d(d[7], 1280, 1, padding=0, stride=1, bias=False), nn.BatchNorm2d(1280, momentum=m),
            nn.ReLU(inplace=True),
        ]
        self.layers = nn.Sequential(*layers)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout, inplace=True), nn.Linear(1280, num_classes))
        for mod in self.modules():
            if isinstance(mod, nn.Conv2d):
                nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
                if mod.bias is not None:
                    nn.init.zeros_(mod.bias)
            elif isinstance(mod, nn.BatchNorm2d):
                nn.init.ones_(mod.weight)
                nn.init.zeros_(mod.bias)
            elif isinstance(mod, nn.Linear):
                nn.init.kaiming_uniform_(mod.weight, mode="fan_out", nonlinearity="sigmoid")
                nn.init.zeros_(mod.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(self.layers(x).mean([2, 3]))


def mnasnet0_5(**kwargs) -> MNASNet:
    return MNASNet(0.5, **kwargs)


def mnasnet0_75(**kwargs) -> MNASNet:
    return MNASNet(0.75, **kwargs)


def mnasnet1_0(**kwargs) -> MNASNet:
    return MNASNet(1.0, **kwargs)


def mnasnet1_3(**kwargs) -> MNASNet:
    return MNASNet(1.3, **kwargs)


# -------------------------------------------------------------------------------------- MobileNetV3
def _make_divisible(v: float, divisor: int = 8, min_value: Optional[int] = None) -> int:
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    return new_v + divisor if new_v < 0.9 * v else new_v


class ConvBNActivation(nn.Sequential):
    """conv -> BN -> activation as children 0, 1, 2 (torchvision's Conv2dNormActivation layout)."""

    def __init__(self, in_ch: int, out_ch: int, kernel_size: int = 3, stride: int = 1, groups: int = 1,
                 norm_layer: Callable[..., nn.Module] = nn.BatchNorm2d,
                 activation_layer: Optional[Callable[..., nn.Module]] = nn.ReLU, dilation: int = 1):
        padding = (kernel_size - 1) // 2 * dilation
        layers: List[nn.Module] = [nn.Conv2d(in_ch, out_ch, kernel_size, stride, padding, dilation=dilation,
                                             groups=groups, bias=False), norm_layer(out_ch)]
        if activation_layer is not None:
            layers.append(activation_layer(inplace=True))
        super().__init__(*layers)


class SqueezeExcitation(nn.Module):
    def __init__(self, input_channels: int, squeeze_channels: int,
                 activation: Callable[..., nn.Module] = nn.ReLU,
                 scale_activation: Callable[..., nn.Module] = nn.Hardsigmoid):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(input_channels, squeeze_channels, 1)
        self.fc2 = nn.Conv2d(squeeze_channels, input_channels, 1)
        self.activation = activation()
        self.scale_activation = scale_activation()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x))))) * x


class _V3Config:
    def __init__(self, in_ch: int, kernel: int, expanded: int, out_ch: int, use_se: bool, activation: str,
                 stride: int, dilation: int = 1, width_mult: float = 1.0):
        self.input_channels = _make_divisible(in_ch * width_mult)
        self.kernel = kernel
        self.expanded_channels = _make_divisible(expanded * width_mult)
        self.out_channels = _make_divisible(out_ch * width_mult)
        self.use_se = use_se
        self.use_hs = activation == "HS"
        self.stride = stride
        self.dilation = dilation


class _V3InvertedResidual(nn.Module):
    def __init__(self, cnf: _V3Config, norm_layer: Callable[..., nn.Module]):
        super().__init__()
        self.use_res_connect = cnf.stride == 1 and cnf.input_channels == cnf.out_channels
        act = nn.Hardswish if cnf.use_hs else nn.ReLU
        layers: List[nn.Module] = []
        if cnf.expanded_channels != cnf.input_channels:
            layers.append(ConvBNActivation(cnf.input_channels, cnf.expanded_channels, 1, norm_layer=norm_layer,
                                           activation_layer=act))
        stride = 1 if cnf.dilation > 1 else cnf.stride
        layers.append(ConvBNActivation(cnf.expanded_channels, cnf.expanded_channels, cnf.kernel, stride,
                                       groups=cnf.expanded_channels, norm_layer=norm_layer, activation_layer=act,
                                       dilation=cnf.dilation))
        if cnf.use_se:
            layers.append(SqueezeExcitation(cnf.expanded_channels, _make_divisible(cnf.expanded_channels // 4)))
        layers.append(ConvBNActivation(cnf.expanded_channels, cnf.out_channels, 1, norm_layer=norm_layer,
                                       activation_layer=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.block(x)
        return y + x if self.use_res_connect else y


class MobileNetV3(nn.Module):
    def __init__(self, setting: List[_V3Config], last_channel: int, num_classes: int = 1000, dropout: float = 0.2):
        super().__init__()
        norm = partial(nn.BatchNorm2d, eps=0.001, momentum=0.01)
        layers: List[nn.Module] = [ConvBNActivation(3, setting[0].input_channels, 3, 2, norm_layer=norm,
                                                    activation_layer=nn.Hardswish)]
        layers += [_V3InvertedResidual(c, norm) for c in setting]
        last_in = setting[-1].out_channels
        layers.append(ConvBNActivation(last_in, 6 * last_in, 1, norm_layer=norm, activation_layer=nn.Hardswish))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Linear(6 * last_in, last_channel), nn.Hardswish(inplace=True),
                                        nn.Dropout(p=dropout, inplace=True), nn.Linear(last_channel, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


def _v3_setting(arch: str, width_mult: float = 1.0):
    c = partial(_V3Config, width_mult=width_mult)
    if arch == "mobilenet_v3_large":
        rows = [(16, 3, 16, 16, False, "RE", 1), (16, 3, 64, 24, False, "RE", 2), (24, 3, 72, 24, False, "RE", 1),
                (24, 5, 72, 40, True, "RE", 2), (40, 5, 120, 40, True, "RE", 1), (40, 5, 120, 40, True, "RE", 1),
                (40, 3, 240, 80, False, "HS", 2), (80, 3, 200, 80, False, "HS", 1), (80, 3, 184, 80, False, "HS", 1),
                (80, 3, 184, 80, False, "HS", 1), (80, 3, 480, 112, True, "HS", 1),
                (112, 3, 672, 112, True, "HS", 1), (112, 5, 672, 160, True, "HS", 2),
                (160, 5, 960, 160, True, "HS", 1), (160, 5, 960, 160, True, "HS", 1)]
        last = 1280
    else:
        rows = [(16, 3, 16, 16, True, "RE", 2), (16, 3, 72, 24, False, "RE", 2), (24, 3, 88, 24, False, "RE", 1),
                (24, 5, 96, 40, True, "HS", 2), (40, 5, 240, 40, True, "HS", 1), (40, 5, 240, 40, True, "HS", 1),
                (40, 5, 120, 48, True, "HS", 1), (48, 5, 144, 48, True, "HS", 1), (48, 5, 288, 96, True, "HS", 2),
                (96, 5, 576, 96, True, "HS", 1), (96, 5, 576, 96, True, "HS", 1)]
        last = 1024
    return [c(*r) for r in rows], _make_divisible(last * width_mult)


def mobilenet_v3_large(**kwargs) -> MobileNetV3:
    setting, last = _v3_setting("mobilenet_v3_large")
    return MobileNetV3(setting, last, **kwargs)


def mobilenet_v3_small(**kwargs) -> MobileNetV3:
    setting, last = _v3_setting("mobilenet_v3_small")
    return MobileNetV3(setting, last, **kwargs)


# ------------------------------------------------------------------------------------- EfficientNet
class StochasticDepth(nn.Module):
    """Drop the whole residual branch per sample with probability ``p`` in training ("row" mode)."""

    def __init__(self, p: float):
        super().__init__()
        self.p = p

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.training or self.p == 0.0:
            return x
        survival = 1.0 - self.p
        noise = torch.empty((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype, device=x.device)
        return x * noise.bernoulli_(survival).div_(survival)


class _MBConvConfig:
    def __init__(self, expand_ratio: float, kernel: int, stride: int, in_ch: int, out_ch: int, num_layers: int,
                 width_mult: float, depth_mult: float):
        self.expand_ratio = expand_ratio
        self.kernel = kernel
        self.stride = stride
        self.input_channels = _make_divisible(in_ch * width_mult)
        self.out_channels = _make_divisible(out_ch * width_mult)
        self.num_layers = int(math.ceil(num_layers * depth_mult))


class MBConv(nn.Module):
    def __init__(self, cnf: _MBConvConfig, stochastic_depth_prob: float, norm_layer: Callable[..., nn.Module]):
        super().__init__()
        self.use_res_connect = cnf.stride == 1 and cnf.input_channels == cnf.out_channels
        expanded = _make_divisible(cnf.input_channels * cnf.expand_ratio)
        layers: List[nn.Module] = []
        if expanded != cnf.input_channels:
            layers.append(ConvBNActivation(cnf.input_channels, expanded, 1, norm_layer=norm_layer,
                                           activation_layer=nn.SiLU))
        layers.append(ConvBNActivation(expanded, expanded, cnf.kernel, cnf.stride, groups=expanded,
                                       norm_layer=norm_layer, activation_layer=nn.SiLU))
        layers.append(SqueezeExcitation(expanded, max(1, cnf.input_channels // 4),
                                        activation=partial(nn.SiLU, inplace=True), scale_activation=nn.Sigmoid))
        layers.append(ConvBNActivation(expanded, cnf.out_channels, 1, norm_layer=norm_layer, activation_layer=None))
        self.block = nn.Sequential(*layers)
        self.stochastic_depth = StochasticDepth(stochastic_depth_prob)
        self.out_channels = cnf.out_channels

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.block(x)
        return self.stochastic_depth(y) + x if self.use_res_connect else y


class _FusedMBConvConfig(_MBConvConfig):
    """EfficientNetV2 early-stage block config (no width/depth scaling)."""

    def __init__(self, expand_ratio: float, kernel: int, stride: int, in_ch: int, out_ch: int, num_layers: int):
        super().__init__(expand_ratio, kernel, stride, in_ch, out_ch, num_layers, 1.0, 1.0)


class FusedMBConv(nn.Module):
    """Fused expand (kxk conv + BN + SiLU) -> 1x1 project; a single kxk conv when the expand ratio is 1."""

    def __init__(self, cnf: _MBConvConfig, stochastic_depth_prob: float, norm_layer: Callable[..., nn.Module]):
        super().__init__()
        self.use_res_connect = cnf.stride == 1 and cnf.input_channels == cnf.out_channels
        expanded = _make_divisible(cnf.input_channels * cnf.expand_ratio)
        if expanded != cnf.input_channels:
            layers = [ConvBNActivation(cnf.input_channels, expanded, cnf.kernel, cnf.stride, norm_layer=norm_layer,
                                       activation_layer=nn.SiLU),
                      ConvBNActivation(expanded, cnf.out_channels, 1, norm_layer=norm_layer, activation_layer=None)]
        else:
            layers = [ConvBNActivation(cnf.input_channels, cnf.out_channels, cnf.kernel, cnf.stride,
                                       norm_layer=norm_layer, activation_layer=nn.SiLU)]
        self.block = nn.Sequential(*layers)
        self.stochastic_depth = StochasticDepth(stochastic_depth_prob)
        self.out_channels = cnf.out_channels

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.block(x)
        return self.stochastic_depth(y) + x if self.use_res_connect else y


class EfficientNet(nn.Module):
    def __init__(self, setting: List[_MBConvConfig], dropout: float, stochastic_depth_prob: float = 0.2,
                 num_classes: int = 1000, norm_layer: Optional[Callable[..., nn.Module]] = None,
                 last_channel: Optional[int] = None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        layers: List[nn.Module] = [ConvBNActivation(3, setting[0].input_channels, 3, 2, norm_layer=norm_layer,
                                                    activation_layer=nn.SiLU)]
        total = sum(c.num_layers for c in setting)
        block_id = 0
        for cnf in setting:
            stage: List[nn.Module] = []
            for _ in range(cnf.num_layers):
                bc = copy.copy(cnf)
                if stage:  # every block after a stage's first keeps the width and stride 1
                    bc.input_channels = bc.out_channels
                    bc.stride = 1
                block = FusedMBConv if isinstance(cnf, _FusedMBConvConfig) else MBConv
                stage.append(block(bc, stochastic_depth_prob * float(block_id) / total, norm_layer))
                block_id += 1
            layers.append(nn.Sequential(*stage))
        last_in = setting[-1].out_channels
        last_channel = last_channel or 4 * last_in
        layers.append(ConvBNActivation(last_in, last_channel, 1, norm_layer=norm_layer, activation_layer=nn.SiLU))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout, inplace=True), nn.Linear(last_channel, num_classes))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                r = 1.0 / math.sqrt(m.out_features)
                nn.init.uniform_(m.weight, -r, r)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


# (width multiplier, depth multiplier, dropout) per variant
_EFFNET = {"b0": (1.0, 1.0, 0.2), "b1": (1.0, 1.1, 0.2), "b2": (1.1, 1.2, 0.3), "b3": (1.2, 1.4, 0.3),
           "b4": (1.4, 1.8, 0.4), "b5": (1.6, 2.2, 0.4), "b6": (1.8, 2.6, 0.5), "b7": (2.0, 3.1, 0.5)}
# (expand ratio, kernel, stride, in, out, layers) per stage
_EFFNET_STAGES = [(1, 3, 1, 32, 16, 1), (6, 3, 2, 16, 24, 2), (6, 5, 2, 24, 40, 2), (6, 3, 2, 40, 80, 3),
                  (6, 5, 1, 80, 112, 3), (6, 5, 2, 112, 192, 4), (6, 3, 1, 192, 320, 1)]


def _efficientnet(variant: str, **kwargs) -> EfficientNet:
    w, d, dropout = _EFFNET[variant]
    setting = [_MBConvConfig(*st, width_mult=w, depth_mult=d) for st in _EFFNET_STAGES]
    if variant in ("b5", "b6", "b7"):
        kwargs.setdefault("norm_layer", partial(nn.BatchNorm2d, eps=0.001, momentum=0.01))
    return EfficientNet(setting, kwargs.pop("dropout", dropout), **kwargs)


def _effnet_ctor(variant: str):
    def ctor(**kwargs) -> EfficientNet:
        return _efficientnet(variant, **kwargs)
    ctor.__name__ = f"efficientnet_{variant}"
    return ctor


EFFICIENTNETS = {f"efficientnet_{v}": _effnet_ctor(v) for v in _EFFNET}


# EfficientNetV2: (fused?, expand ratio, kernel, stride, in, out, layers) per stage, dropout
_EFFNET_V2 = {
    "s": ([(1, 1, 3, 1, 24, 24, 2), (1, 4, 3, 2, 24, 48, 4), (1, 4, 3, 2, 48, 64, 4), (0, 4, 3, 2, 64, 128, 6),
           (0, 6, 3, 1, 128, 160, 9), (0, 6, 3, 2, 160, 256, 15)], 0.2),
    "m": ([(1, 1, 3, 1, 24, 24, 3), (1, 4, 3, 2, 24, 48, 5), (1, 4, 3, 2, 48, 80, 5), (0, 4, 3, 2, 80, 160, 7),
           (0, 6, 3, 1, 160, 176, 14), (0, 6, 3, 2, 176, 304, 18), (0, 6, 3, 1, 304, 512, 5)], 0.3),
    "l": ([(1, 1, 3, 1, 32, 32, 4), (1, 4, 3, 2, 32, 64, 7), (1, 4, 3, 2, 64, 96, 7), (0, 4, 3, 2, 96, 192, 10),
           (0, 6, 3, 1, 192, 224, 19), (0, 6, 3, 2, 224, 384, 25), (0, 6, 3, 1, 384, 640, 7)], 0.4),
}


def _efficientnet_v2(variant: str, **kwargs) -> EfficientNet:
    stages, dropout = _EFFNET_V2[variant]
    setting = [_FusedMBConvConfig(*st[1:]) if st[0] else _MBConvConfig(*st[1:], width_mult=1.0, depth_mult=1.0)
               for st in stages]
    kwargs.setdefault("norm_layer", partial(nn.BatchNorm2d, eps=1e-3))
    return EfficientNet(setting, kwargs.pop("dropout", dropout), last_channel=1280, **kwargs)


def _effnet_v2_ctor(variant: str):
    def ctor(**kwargs) -> EfficientNet:
        return _efficientnet_v2(variant, **kwargs)
    ctor.__name__ = f"efficientnet_v2_{variant}"
    return ctor


EFFICIENTNETS.update({f"efficientnet_v2_{v}": _effnet_v2_ctor(v) for v in _EFFNET_V2})
