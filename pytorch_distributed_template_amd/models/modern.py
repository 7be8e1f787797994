"""RegNet-X/Y, ConvNeXt, Vision Transformer, Swin Transformer (V1/V2) and MaxViT with torchvision-identical module names, shapes, parameter
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


# ------------------------------------------------------------------------------------------ Swin
class ShiftedWindowAttention(nn.Module):
    """Windowed MHSA with a learned relative-position bias and cyclic shift; the (bias + shift mask) is one
    additive mask so the attention itself runs as PyTorch's fused scaled-dot-product kernel."""

    def __init__(self, dim: int, window: int, shift: int, heads: int, attn_dropout: float, dropout: float,
                 v2: bool = False):
        super().__init__()
        self.window_size, self.shift_size, self.num_heads = [window, window], [shift, shift], heads
        self.attention_dropout, self.dropout, self.v2 = attn_dropout, dropout, v2
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)
        if v2:  # Swin V2: cosine attention with a learned per-head temperature, log-spaced continuous bias MLP
            self.logit_scale = nn.Parameter(torch.log(10 * torch.ones((heads, 1, 1))))
            self.cpb_mlp = nn.Sequential(nn.Linear(2, 512), nn.ReLU(inplace=True), nn.Linear(512, heads, bias=False))
            r = torch.arange(-(window - 1), window, dtype=torch.float32) / (window - 1) * 8
            t = torch.stack(torch.meshgrid(r, r, indexing="ij")).permute(1, 2, 0).unsqueeze(0)
            self.register_buffer("relative_coords_table", torch.sign(t) * torch.log2(t.abs() + 1.0) / 3.0)
        else:
            self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * window - 1) ** 2, heads))
            nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        c = torch.stack(torch.meshgrid(torch.arange(window), torch.arange(window), indexing="ij")).flatten(1)
        rel = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0) + (window - 1)
        self.register_buffer("relative_position_index", (rel[..., 0] * (2 * window - 1) + rel[..., 1]).flatten())

    def _bias(self) -> torch.Tensor:
        n = self.window_size[0] * self.window_size[1]
        # buffers are cloned: the trainer's buffer sync may rewrite them in place before backward
        table = (self.cpb_mlp(self.relative_coords_table.clone()).view(-1, self.num_heads) if self.v2
                 else self.relative_position_bias_table)
        b = table[self.relative_position_index.clone()].view(n, n, -1).permute(2, 0, 1).unsqueeze(0)
        return 16 * torch.sigmoid(b) if self.v2 else b

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, H, W, C = x.shape
        ws = self.window_size[0]
        pad_r, pad_b = (ws - W % ws) % ws, (ws - H % ws) % ws
        x = nn.functional.pad(x, (0, 0, 0, pad_r, 0, pad_b))
        pH, pW = x.shape[1], x.shape[2]
        sh = self.shift_size[0] if ws < pH else 0
        sw = self.shift_size[1] if ws < pW else 0
        if sh or sw:
            x = torch.roll(x, shifts=(-sh, -sw), dims=(1, 2))
        nwin = (pH // ws) * (pW // ws)
        x = x.view(B, pH // ws, ws, pW // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B * nwin, ws * ws, C)
        hd = C // self.num_heads
        qkv_bias = self.qkv.bias
        if self.v2:  # the key bias is held at zero
            qkv_bias = torch.cat([qkv_bias[:C], torch.zeros_like(qkv_bias[C:2 * C]), qkv_bias[2 * C:]])
        qkv = nn.functional.linear(x, self.qkv.weight, qkv_bias)
        q, k, v = qkv.reshape(x.size(0), x.size(1), 3, self.num_heads, hd).permute(2, 0, 3, 1, 4)
        scale = None
        if self.v2:
            q = nn.functional.normalize(q, dim=-1) * torch.clamp(self.logit_scale, max=math.log(100.0)).exp()
            k = nn.functional.normalize(k, dim=-1)
            scale = 1.0
        mask = self._bias().to(q.dtype)                                     # [1, heads, N, N]
        if sh or sw:
            region = x.new_zeros((pH, pW))
            cnt = 0
            for hs in ((0, -ws), (-ws, -sh), (-sh, None)):
                for wsl in ((0, -ws), (-ws, -sw), (-sw, None)):
                    region[hs[0]:hs[1], wsl[0]:wsl[1]] = cnt
                    cnt += 1
            region = region.view(pH // ws, ws, pW // ws, ws).permute(0, 2, 1, 3).reshape(nwin, ws * ws)
            shift = (region.unsqueeze(1) - region.unsqueeze(2)).ne(0).to(q.dtype) * -100.0
            mask = (mask + shift.unsqueeze(1)).repeat(B, 1, 1, 1)           # [B*nwin, heads, N, N]
        y = nn.functional.scaled_dot_product_attention(
            q, k, v, attn_mask=mask, dropout_p=self.attention_dropout if self.training else 0.0, scale=scale)
        y = self.proj(y.transpose(1, 2).reshape(x.size(0), x.size(1), C))
        y = nn.functional.dropout(y, self.dropout, self.training)
        y = y.view(B, pH // ws, pW // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, pH, pW, C)
        if sh or sw:
            y = torch.roll(y, shifts=(sh, sw), dims=(1, 2))
        return y[:, :H, :W, :].contiguous()


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim: int, heads: int, window: int, shift: int, sd_prob: float, dropout: float = 0.0,
                 attn_dropout: float = 0.0, v2: bool = False):
        super().__init__()
        self.v2 = v2
        self.norm1 = nn.LayerNorm(dim, eps=1e-5)
        self.attn = ShiftedWindowAttention(dim, window, shift, heads, attn_dropout, dropout, v2)
        self.stochastic_depth = StochasticDepth(sd_prob)
        self.norm2 = nn.LayerNorm(dim, eps=1e-5)
        self.mlp = _MLPBlock(dim, 4 * dim, dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.v2:  # residual post-norm
            x = x + self.stochastic_depth(self.norm1(self.attn(x)))
            return x + self.stochastic_depth(self.norm2(self.mlp(x)))
        x = x + self.stochastic_depth(self.attn(self.norm1(x)))
        return x + self.stochastic_depth(self.mlp(self.norm2(x)))


class PatchMerging(nn.Module):
    """2x2 space-to-depth (channels-last), LayerNorm, linear 4C -> 2C."""

    def __init__(self, dim: int, v2: bool = False):
        super().__init__()
        self.v2 = v2
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(2 * dim if v2 else 4 * dim, eps=1e-5)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        H, W = x.shape[-3], x.shape[-2]
        x = nn.functional.pad(x, (0, 0, 0, W % 2, 0, H % 2))
        x = torch.cat([x[..., 0::2, 0::2, :], x[..., 1::2, 0::2, :], x[..., 0::2, 1::2, :],
                       x[..., 1::2, 1::2, :]], -1)
        return self.norm(self.reduction(x)) if self.v2 else self.reduction(self.norm(x))


class SwinTransformer(nn.Module):
    def __init__(self, embed_dim: int, depths: List[int], heads: List[int], sd_prob: float, window: int = 7,
                 patch: int = 4, num_classes: int = 1000, v2: bool = False):
        super().__init__()
        layers: List[nn.Module] = [nn.Sequential(nn.Conv2d(3, embed_dim, patch, patch), _Permute([0, 2, 3, 1]),
                                                 nn.LayerNorm(embed_dim, eps=1e-5))]
        total, bid = sum(depths), 0
        for i, (depth, h) in enumerate(zip(depths, heads)):
            dim = embed_dim * 2 ** i
            stage = []
            for j in range(depth):
                stage.append(SwinTransformerBlock(dim, h, window, 0 if j % 2 == 0 else window // 2,
                                                  sd_prob * bid / (total - 1.0), v2=v2))
                bid += 1
            layers.append(nn.Sequential(*stage))
            if i + 1 < len(depths):
                layers.append(PatchMerging(dim, v2))
        self.features = nn.Sequential(*layers)
        nf = embed_dim * 2 ** (len(depths) - 1)
        self.norm = nn.LayerNorm(nf, eps=1e-5)
        self.permute = _Permute([0, 3, 1, 2])
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.flatten = nn.Flatten(1)
        self.head = nn.Linear(nf, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.permute(self.norm(self.features(x)))
        return self.head(self.flatten(self.avgpool(x)))


def swin_t(**kwargs) -> SwinTransformer:
    return SwinTransformer(96, [2, 2, 6, 2], [3, 6, 12, 24], kwargs.pop("stochastic_depth_prob", 0.2), **kwargs)


def swin_s(**kwargs) -> SwinTransformer:
    return SwinTransformer(96, [2, 2, 18, 2], [3, 6, 12, 24], kwargs.pop("stochastic_depth_prob", 0.3), **kwargs)


def swin_b(**kwargs) -> SwinTransformer:
    return SwinTransformer(128, [2, 2, 18, 2], [4, 8, 16, 32], kwargs.pop("stochastic_depth_prob", 0.5), **kwargs)


def swin_v2_t(**kwargs) -> SwinTransformer:
    return SwinTransformer(96, [2, 2, 6, 2], [3, 6, 12, 24], kwargs.pop("stochastic_depth_prob", 0.2), window=8,
                           v2=True, **kwargs)


def swin_v2_s(**kwargs) -> SwinTransformer:
    return SwinTransformer(96, [2, 2, 18, 2], [3, 6, 12, 24], kwargs.pop("stochastic_depth_prob", 0.3), window=8,
                           v2=True, **kwargs)


def swin_v2_b(**kwargs) -> SwinTransformer:
    return SwinTransformer(128, [2, 2, 18, 2], [4, 8, 16, 32], kwargs.pop("stochastic_depth_prob", 0.5), window=8,
                           v2=True, **kwargs)


# ------------------------------------------------------------------------------------------ MaxViT
class _MaxVitMBConv(nn.Module):
    """Pre-norm inverted bottleneck (1x1 -> 3x3 depthwise -> SE -> 1x1) with an avg-pool + 1x1 projection."""

    def __init__(self, cin: int, cout: int, expansion: float, squeeze: float, stride: int,
                 norm: Callable[..., nn.Module], sd_prob: float):
        super().__init__()
        mid, sqz = int(cout * expansion), int(cout * squeeze)
        self.stochastic_depth = StochasticDepth(sd_prob) if sd_prob else nn.Identity()
        if stride != 1 or cin != cout:
            proj: List[nn.Module] = [nn.AvgPool2d(3, stride, 1)] if stride == 2 else []
            self.proj = nn.Sequential(*proj, nn.Conv2d(cin, cout, 1, bias=True))
        else:
            self.proj = nn.Identity()
        f = OrderedDict()
        f["pre_norm"] = norm(cin)
        f["conv_a"] = nn.Sequential(nn.Conv2d(cin, mid, 1, bias=False), norm(mid), nn.GELU())
        f["conv_b"] = nn.Sequential(nn.Conv2d(mid, mid, 3, stride, 1, groups=mid, bias=False), norm(mid), nn.GELU())
        f["squeeze_excitation"] = _SE(mid, sqz)
        f["conv_c"] = nn.Conv2d(mid, cout, 1, bias=True)
        self.layers = nn.Sequential(f)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.proj(x) + self.stochastic_depth(self.layers(x))


class _SE(_RegNetSE):
    """Squeeze-excitation with a SiLU squeeze."""

    def __init__(self, channels: int, squeeze: int):
        super().__init__(channels, squeeze)
        self.activation = nn.SiLU()


class RelativePositionalMultiHeadAttention(nn.Module):
    """MHSA over a P-token partition with a learned 2-D relative-position bias (fused SDPA; the query scale is
    feat_dim^-0.5, as in torchvision's MaxViT)."""

    def __init__(self, feat_dim: int, head_dim: int, max_seq_len: int):
        super().__init__()
        self.n_heads, self.head_dim = feat_dim // head_dim, head_dim
        self.size, self.max_seq_len = int(math.sqrt(max_seq_len)), max_seq_len
        self.to_qkv = nn.Linear(feat_dim, self.n_heads * head_dim * 3)
        self.scale_factor = feat_dim ** -0.5
        self.merge = nn.Linear(self.n_heads * head_dim, feat_dim)
        n = self.size
        self.relative_position_bias_table = nn.Parameter(torch.empty((2 * n - 1) ** 2, self.n_heads))
        c = torch.stack(torch.meshgrid(torch.arange(n), torch.arange(n), indexing="ij")).flatten(1)
        rel = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0) + (n - 1)
        self.register_buffer("relative_position_index", rel[..., 0] * (2 * n - 1) + rel[..., 1])
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)

    def get_relative_positional_bias(self) -> torch.Tensor:
        b = self.relative_position_bias_table[self.relative_position_index.view(-1).clone()]  # see _bias above
        return b.view(self.max_seq_len, self.max_seq_len, -1).permute(2, 0, 1).unsqueeze(0)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, G, P, D = x.shape
        q, k, v = (t.reshape(B, G, P, self.n_heads, self.head_dim).permute(0, 1, 3, 2, 4)
                   for t in self.to_qkv(x).chunk(3, dim=-1))
        bias = self.get_relative_positional_bias().to(q.dtype)
        out = nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=self.scale_factor)
        return self.merge(out.permute(0, 1, 3, 2, 4).reshape(B, G, P, D))


class PartitionAttentionLayer(nn.Module):
    """Block (window) or grid (dilated) partition -> attention + MLP (pre-LN, stochastic depth) -> departition."""

    def __init__(self, channels: int, head_dim: int, partition: int, kind: str, grid: int, mlp_ratio: int,
                 attn_dropout: float, mlp_dropout: float, sd_prob: float):
        super().__init__()
        self.n_partitions = grid // partition
        self.p = partition if kind == "window" else self.n_partitions
        self.grid = kind == "grid"
        self.attn_layer = nn.Sequential(nn.LayerNorm(channels),
                                        RelativePositionalMultiHeadAttention(channels, head_dim, partition ** 2),
                                        nn.Dropout(attn_dropout))
        self.mlp_layer = nn.Sequential(nn.LayerNorm(channels), nn.Linear(channels, channels * mlp_ratio), nn.GELU(),
                                       nn.Linear(channels * mlp_ratio, channels), nn.Dropout(mlp_dropout))
        self.stochastic_dropout = StochasticDepth(sd_prob)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x.shape
        p, gh, gw = self.p, H // self.p, W // self.p
        x = x.reshape(B, C, gh, p, gw, p).permute(0, 2, 4, 3, 5, 1).reshape(B, gh * gw, p * p, C)
        if self.grid:
            x = x.transpose(-2, -3)
        x = x + self.stochastic_dropout(self.attn_layer(x))
        x = x + self.stochastic_dropout(self.mlp_layer(x))
        if self.grid:
            x = x.transpose(-2, -3)
        return x.reshape(B, gh, gw, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(B, C, gh * p, gw * p)


class MaxVit(nn.Module):
    def __init__(self, input_size=(224, 224), stem_channels: int = 64, partition_size: int = 7,
                 block_channels=(64, 128, 256, 512), block_layers=(2, 2, 5, 2), head_dim: int = 32,
                 stochastic_depth_prob: float = 0.2, squeeze_ratio: float = 0.25, expansion_ratio: float = 4,
                 mlp_ratio: int = 4, mlp_dropout: float = 0.0, attention_dropout: float = 0.0,
                 num_classes: int = 1000):
        super().__init__()
        norm = partial(nn.BatchNorm2d, eps=1e-3, momentum=0.01)
        self.stem = nn.Sequential(
            nn.Sequential(nn.Conv2d(3, stem_channels, 3, 2, 1, bias=False), norm(stem_channels), nn.GELU()),
            nn.Sequential(nn.Conv2d(stem_channels, stem_channels, 3, 1, 1, bias=True)))
        grid = (input_size[0] - 1) // 2 + 1
        sd = torch.linspace(0, stochastic_depth_prob, sum(block_layers)).tolist()
        self.partition_size = partition_size
        self.blocks = nn.ModuleList()
        cin, li = stem_channels, 0
        for cout, n in zip(block_channels, block_layers):
            grid = (grid - 1) // 2 + 1
            if grid % partition_size:
                raise ValueError(f"feature grid {grid} not divisible by partition size {partition_size}")
            blk = nn.Module()
            blk.layers = nn.ModuleList()
            for j in range(n):
                f = OrderedDict()
                f["MBconv"] = _MaxVitMBConv(cin if j == 0 else cout, cout, expansion_ratio, squeeze_ratio,
                                            2 if j == 0 else 1, norm, sd[li])
                for kind in ("window", "grid"):
                    f[f"{kind}_attention"] = PartitionAttentionLayer(cout, head_dim, partition_size, kind, grid,
                                                                     mlp_ratio, attention_dropout, mlp_dropout, sd[li])
                layer = nn.Module()
                layer.layers = nn.Sequential(f)
                blk.layers.append(layer)
                li += 1
            self.blocks.append(blk)
            cin = cout
        c = block_channels[-1]
        self.classifier = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.LayerNorm(c), nn.Linear(c, c),
                                        nn.Tanh(), nn.Linear(c, num_classes, bias=False))
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.stem(x)
        for blk in self.blocks:
            for layer in blk.layers:
                x = layer.layers(x)
        return self.classifier(x)


def maxvit_t(**kwargs) -> MaxVit:
    return MaxVit(**kwargs)


MODERN = {
    **REGNETS,
    "convnext_tiny": convnext_tiny, "convnext_small": convnext_small, "convnext_base": convnext_base,
    "convnext_large": convnext_large,
    "vit_b_16": vit_b_16, "vit_b_32": vit_b_32, "vit_l_16": vit_l_16, "vit_l_32": vit_l_32, "vit_h_14": vit_h_14,
    "swin_t": swin_t, "swin_s": swin_s, "swin_b": swin_b,
    "swin_v2_t": swin_v2_t, "swin_v2_s": swin_v2_s, "swin_v2_b": swin_v2_b,
    "maxvit_t": maxvit_t,
}
