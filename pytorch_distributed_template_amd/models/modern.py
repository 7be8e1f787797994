"""RegNet-X/Y, ConvNeXt and Vision Transformer with torchvision-identical module names, shapes, parameter
counts and init.

Registry members (reference C05, `dataparallel.py:36-37` exposes every lowercase torchvision constructor as an
``--arch`` choice); executed by the stock-PyTorch engine (MIOpen / hipBLASLt through PyTorch-ROCm).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from functools import partial
from typing import Callable, List, Optional

import torch
import torch.nn as nn

from .efficient import StochasticDepth, _make_divisible


def _conv_bn_act(cin: int, cout: int, k: int, stride: int = 1, groups: int = 1,
                 act: Optional[Callable[..., nn.Module]] = nn.ReLU) -> nn.Sequential:
    """torchvision ``Conv2dNormActivation`` (conv '0', BN '1', activation '2'; no conv bias)."""
    layers: List[nn.Module] = [nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
                               nn.BatchNorm2d(cout)]
    if act is not None:
        layers.append(act(inplace=True))
    return nn.Sequential(*layers)


# ------------------------------------------------------------------------------------------ RegNet
class _RegNetSE(nn.Module):
    """Squeeze-excitation with 1x1 convs (fc1/fc2), ReLU squeeze and sigmoid gate."""

    def __init__(self, channels: int, squeeze: int):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(channels, squeeze, 1)
        self.fc2 = nn.Conv2d(squeeze, channels, 1)
        self.activation = nn.ReLU()
        self.scale_activation = nn.Sigmoid()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        s = self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x)))))
        return x * s


class _RegNetBottleneck(nn.Module):
    """X block (1x1 -> grouped 3x3 -> 1x1) with an optional SE (Y block) sized off the block input width."""

    def __init__(self, cin: int, cout: int, stride: int, group_width: int, bottleneck: float,
                 se_ratio: Optional[float]):
        super().__init__()
        self.proj = _conv_bn_act(cin, cout, 1, stride, act=None) if (cin != cout or stride != 1) else None
        wb = int(round(cout * bottleneck))
        f = OrderedDict()
        f["a"] = _conv_bn_act(cin, wb, 1)
        f["b"] = _conv_bn_act(wb, wb, 3, stride, groups=wb // group_width)
        if se_ratio:
            f["se"] = _RegNetSE(wb, int(round(se_ratio * cin)))
        f["c"] = _conv_bn_act(wb, cout, 1, act=None)
        self.f = nn.Sequential(f)
        self.activation = nn.ReLU(inplace=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        sc = x if self.proj is None else self.proj(x)
        return self.activation(sc + self.f(x))


def _regnet_stages(depth: int, w0: int, wa: float, wm: float, group_width: int, bottleneck: float = 1.0):
    """Quantised linear width schedule -> per-stage (width, depth, group width) (RegNet design space)."""
    cont = torch.arange(depth) * wa + w0
    cap = torch.round(torch.log(cont / w0) / math.log(wm))
    widths = (torch.round(w0 * torch.pow(wm, cap) / 8) * 8).int().tolist()
    stage_w, stage_d = [], []
    for w in widths:
        if stage_w and stage_w[-1] == w:
            stage_d[-1] += 1
        else:
            stage_w.append(w)
            stage_d.append(1)
    wbot = [int(w * bottleneck) for w in stage_w]
    gws = [min(group_width, w) for w in wbot]
    wbot = [_make_divisible(w, g) for w, g in zip(wbot, gws)]
    stage_w = [int(w / bottleneck) for w in wbot]
    return list(zip(stage_w, stage_d, gws))


class RegNet(nn.Module):
    def __init__(self, depth: int, w0: int, wa: float, wm: float, group_width: int,
                 se_ratio: Optional[float] = None, num_classes: int = 1000, stem_width: int = 32):
        super().__init__()
        self.stem = _conv_bn_act(3, stem_width, 3, 2)
        stages = OrderedDict()
        cin = stem_width
        for i, (w, d, g) in enumerate(_regnet_stages(depth, w0, wa, wm, group_width)):
            blocks = OrderedDict()
            for j in range(d):
                blocks[f"block{i + 1}-{j}"] = _RegNetBottleneck(cin if j == 0 else w, w, 2 if j == 0 else 1,
                                                                g, 1.0, se_ratio)
            stages[f"block{i + 1}"] = nn.Sequential(blocks)
            cin = w
        self.trunk_output = nn.Sequential(stages)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                nn.init.normal_(m.weight, 0.0, math.sqrt(2.0 / fan_out))
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.avgpool(self.trunk_output(self.stem(x)))
        return self.fc(x.flatten(1))


# name -> (depth, w_0, w_a, w_m, group_width, se_ratio)
_REGNET = {
    "regnet_y_400mf": (16, 48, 27.89, 2.09, 8, 0.25), "regnet_y_800mf": (14, 56, 38.84, 2.4, 16, 0.25),
    "regnet_y_1_6gf": (27, 48, 20.71, 2.65, 24, 0.25), "regnet_y_3_2gf": (21, 80, 42.63, 2.66, 24, 0.25),
    "regnet_y_8gf": (17, 192, 76.82, 2.19, 56, 0.25), "regnet_y_16gf": (18, 200, 106.23, 2.48, 112, 0.25),
    "regnet_y_32gf": (20, 232, 115.89, 2.53, 232, 0.25), "regnet_y_128gf": (27, 456, 160.83, 2.52, 264, 0.25),
    "regnet_x_400mf": (22, 24, 24.48, 2.54, 16, None), "regnet_x_800mf": (16, 56, 35.73, 2.28, 16, None),
    "regnet_x_1_6gf": (18, 80, 34.01, 2.25, 24, None), "regnet_x_3_2gf": (25, 88, 26.31, 2.25, 48, None),
    "regnet_x_8gf": (23, 80, 49.56, 2.88, 120, None), "regnet_x_16gf": (22, 216, 55.59, 2.1, 128, None),
    "regnet_x_32gf": (23, 320, 69.86, 2.0, 168, None),
}


def _regnet_ctor(name: str):
    def ctor(**kwargs) -> RegNet:
        return RegNet(*_REGNET[name], **kwargs)
    ctor.__name__ = name
    return ctor


REGNETS = {name: _regnet_ctor(name) for name in _REGNET}


# ------------------------------------------------------------------------------------------ ConvNeXt
class LayerNorm2d(nn.LayerNorm):
    """LayerNorm over the channel dim of an NCHW tensor."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.permute(0, 2, 3, 1)
        x = nn.functional.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
        return x.permute(0, 3, 1, 2)


class _Permute(nn.Module):
    def __init__(self, dims: List[int]):
        super().__init__()
        self.dims = dims

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.permute(x, self.dims)


class CNBlock(nn.Module):
    """7x7 depthwise -> LN -> 4x MLP (GELU) -> layer scale -> stochastic depth, residual."""

    def __init__(self, dim: int, layer_scale: float, sd_prob: float):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(dim, dim, 7, padding=3, groups=dim, bias=True), _Permute([0, 2, 3, 1]),
            nn.LayerNorm(dim, eps=1e-6), nn.Linear(dim, 4 * dim), nn.GELU(), nn.Linear(4 * dim, dim),
            _Permute([0, 3, 1, 2]))
        self.layer_scale = nn.Parameter(torch.ones(dim, 1, 1) * layer_scale)
        self.stochastic_depth = StochasticDepth(sd_prob)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x + self.stochastic_depth(self.layer_scale * self.block(x))


class ConvNeXt(nn.Module):
    def __init__(self, dims: List[int], depths: List[int], sd_prob: float, num_classes: int = 1000,
                 layer_scale: float = 1e-6):
        super().__init__()
        ln = partial(LayerNorm2d, eps=1e-6)
        layers: List[nn.Module] = [nn.Sequential(nn.Conv2d(3, dims[0], 4, 4, bias=True), ln(dims[0]))]
        total, bid = sum(depths), 0
        for i, (dim, depth) in enumerate(zip(dims, depths)):
            stage = []
            for _ in range(depth):
                stage.append(CNBlock(dim, layer_scale, sd_prob * bid / (total - 1.0)))
                bid += 1
            layers.append(nn.Sequential(*stage))
            if i + 1 < len(dims):
                layers.append(nn.Sequential(ln(dim), nn.Conv2d(dim, dims[i + 1], 2, 2)))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(ln(dims[-1]), nn.Flatten(1), nn.Linear(dims[-1], num_classes))
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.classifier(self.avgpool(self.features(x)))


def convnext_tiny(**kwargs) -> ConvNeXt:
    return ConvNeXt([96, 192, 384, 768], [3, 3, 9, 3], kwargs.pop("stochastic_depth_prob", 0.1), **kwargs)


def convnext_small(**kwargs) -> ConvNeXt:
    return ConvNeXt([96, 192, 384, 768], [3, 3, 27, 3], kwargs.pop("stochastic_depth_prob", 0.4), **kwargs)


def convnext_base(**kwargs) -> ConvNeXt:
    return ConvNeXt([128, 256, 512, 1024], [3, 3, 27, 3], kwargs.pop("stochastic_depth_prob", 0.5), **kwargs)


def convnext_large(**kwargs) -> ConvNeXt:
    return ConvNeXt([192, 384, 768, 1536], [3, 3, 27, 3], kwargs.pop("stochastic_depth_prob", 0.5), **kwargs)


# ------------------------------------------------------------------------------------------ ViT
class _MLPBlock(nn.Sequential):
    def __init__(self, dim: int, mlp_dim: int, dropout: float):
        super().__init__(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Dropout(dropout), nn.Linear(mlp_dim, dim),
                         nn.Dropout(dropout))
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)


class EncoderBlock(nn.Module):
    """Pre-LN transformer block; attention is PyTorch's fused SDPA path inside ``nn.MultiheadAttention``."""

    def __init__(self, heads: int, dim: int, mlp_dim: int, dropout: float, attn_dropout: float):
        super().__init__()
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = nn.MultiheadAttention(dim, heads, dropout=attn_dropout, batch_first=True)
        self.dropout = nn.Dropout(dropout)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _MLPBlock(dim, mlp_dim, dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.ln_1(x)
        y, _ = self.self_attention(y, y, y, need_weights=False)
        x = x + self.dropout(y)
        return x + self.mlp(self.ln_2(x))


class Encoder(nn.Module):
    def __init__(self, seq_len: int, layers: int, heads: int, dim: int, mlp_dim: int, dropout: float,
                 attn_dropout: float):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_len, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(dropout)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim, dropout, attn_dropout)) for i in range(layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int, patch_size: int, layers: int, heads: int, dim: int, mlp_dim: int,
                 dropout: float = 0.0, attention_dropout: float = 0.0, num_classes: int = 1000):
        super().__init__()
        if image_size % patch_size:
            raise ValueError("image_size must be divisible by patch_size")
        self.image_size, self.patch_size, self.hidden_dim = image_size, patch_size, dim
        self.conv_proj = nn.Conv2d(3, dim, patch_size, patch_size)
        self.class_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.encoder = Encoder((image_size // patch_size) ** 2 + 1, layers, heads, dim, mlp_dim, dropout,
                               attention_dropout)
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(dim, num_classes)))
        fan_in = 3 * patch_size * patch_size
        nn.init.trunc_normal_(self.conv_proj.weight, std=math.sqrt(1 / fan_in))
        nn.init.zeros_(self.conv_proj.bias)
        nn.init.zeros_(self.heads.head.weight)
        nn.init.zeros_(self.heads.head.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n, _, h, w = x.shape
        if h != self.image_size or w != self.image_size:
            raise ValueError(f"expected {self.image_size}x{self.image_size} input, got {h}x{w}")
        x = self.conv_proj(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.class_token.expand(n, -1, -1), x], dim=1)
        return self.heads(self.encoder(x)[:, 0])


def _vit(patch: int, layers: int, heads: int, dim: int, mlp_dim: int, **kwargs) -> VisionTransformer:
    return VisionTransformer(kwargs.pop("image_size", 224), patch, layers, heads, dim, mlp_dim, **kwargs)


def vit_b_16(**kwargs) -> VisionTransformer:
    return _vit(16, 12, 12, 768, 3072, **kwargs)


def vit_b_32(**kwargs) -> VisionTransformer:
    return _vit(32, 12, 12, 768, 3072, **kwargs)


def vit_l_16(**kwargs) -> VisionTransformer:
    return _vit(16, 24, 16, 1024, 4096, **kwargs)


def vit_l_32(**kwargs) -> VisionTransformer:
    return _vit(32, 24, 16, 1024, 4096, **kwargs)


def vit_h_14(**kwargs) -> VisionTransformer:
    return _vit(14, 32, 16, 1280, 5120, **kwargs)


MODERN = {
    **REGNETS,
    "convnext_tiny": convnext_tiny, "convnext_small": convnext_small, "convnext_base": convnext_base,
    "convnext_large": convnext_large,
    "vit_b_16": vit_b_16, "vit_b_32": vit_b_32, "vit_l_16": vit_l_16, "vit_l_32": vit_l_32, "vit_h_14": vit_h_14,
}
