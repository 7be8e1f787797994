"""DenseNet, MobileNetV2 and ShuffleNetV2 with torchvision-identical module names, shapes and init.

Registry members (reference C05); executed by the stock-PyTorch engine.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------- DenseNet
class _DenseLayer(nn.Module):
    def __init__(self, num_input_features: int, growth_rate: int, bn_size: int, drop_rate: float):
        super().__init__()
        self.norm1 = nn.BatchNorm2d(num_input_features)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(num_input_features, bn_size * growth_rate, kernel_size=1, stride=1, bias=False)
        self.norm2 = nn.BatchNorm2d(bn_size * growth_rate)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(bn_size * growth_rate, growth_rate, kernel_size=3, stride=1, padding=1, bias=False)
        self.drop_rate = float(drop_rate)

    def forward(self, inputs: List[torch.Tensor]) -> torch.Tensor:
        x = torch.cat(inputs, 1)
        out = self.conv2(self.relu2(self.norm2(self.conv1(self.relu1(self.norm1(x))))))
        if self.drop_rate > 0:
            out = F.dropout(out, p=self.drop_rate, training=self.training)
        return out


class _DenseBlock(nn.ModuleDict):
    def __init__(self, num_layers: int, num_input_features: int, bn_size: int, growth_rate: int, drop_rate: float):
        super().__init__()
        for i in range(num_layers):
            self.add_module("denselayer%d" % (i + 1),
                            _DenseLayer(num_input_features + i * growth_rate, growth_rate, bn_size, drop_rate))

    def forward(self, init_features: torch.Tensor) -> torch.Tensor:
        features = [init_features]
        for _, layer in self.items():
            features.append(layer(features))
        return torch.cat(features, 1)


class _Transition(nn.Sequential):
    def __init__(self, num_input_features: int, num_output_features: int):
        super().__init__()
        self.norm = nn.BatchNorm2d(num_input_features)
        self.relu = nn.ReLU(inplace=True)
        self.conv = nn.Conv2d(num_input_features, num_output_features, kernel_size=1, stride=1, bias=False)
        self.pool = nn.AvgPool2d(kernel_size=2, stride=2)


class DenseNet(nn.Module):
    def __init__(self, growth_rate: int = 32, block_config: Tuple[int, ...] = (6, 12, 24, 16),
                 num_init_features: int = 64, bn_size: int = 4, drop_rate: float = 0, num_classes: int = 1000):
        super().__init__()
        self.features = nn.Sequential(OrderedDict([
            ("conv0", nn.Conv2d(3, num_init_features, kernel_size=7, stride=2, padding=3, bias=False)),
            ("norm0", nn.BatchNorm2d(num_init_features)),
            ("relu0", nn.ReLU(inplace=True)),
            ("pool0", nn.MaxPool2d(kernel_size=3, stride=2, padding=1)),
        ]))
        num_features = num_init_features
        for i, num_layers in enumerate(block_config):
            self.features.add_module("denseblock%d" % (i + 1),
                                     _DenseBlock(num_layers, num_features, bn_size, growth_rate, drop_rate))
            num_features = num_features + num_layers * growth_rate
            if i != len(block_config) - 1:
                self.features.add_module("transition%d" % (i + 1), _Transition(num_features, num_features // 2))
                num_features = num_features // 2
        self.features.add_module("norm5", nn.BatchNorm2d(num_features))
        self.classifier = nn.Linear(num_features, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        out = F.relu(self.features(x), inplace=True)
        out = torch.flatten(F.adaptive_avg_pool2d(out, (1, 1)), 1)
        return self.classifier(out)


def densenet121(pretrained=False, **kw): return DenseNet(32, (6, 12, 24, 16), 64, **kw)
def densenet161(pretrained=False, **kw): return DenseNet(48, (6, 12, 36, 24), 96, **kw)
def densenet169(pretrained=False, **kw): return DenseNet(32, (6, 12, 32, 32), 64, **kw)
def densenet201(pretrained=False, **kw): return DenseNet(32, (6, 12, 48, 32), 64, **kw)


# ------------------------------------------------------------------------------------- MobileNetV2
def _make_divisible(v: float, divisor: int = 8, min_value: Optional[int] = None) -> int:
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNAct(nn.Sequential):
    """Conv2d -> BatchNorm2d -> activation (torchvision ``Conv2dNormActivation`` layout: '0','1','2')."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1, act=nn.ReLU6):
        pad = (kernel_size - 1) // 2
        layers = [nn.Conv2d(cin, cout, kernel_size, stride, pad, groups=groups, bias=False), nn.BatchNorm2d(cout)]
        if act is not None:
            layers.append(act(inplace=True))
        super().__init__(*layers)


class InvertedResidualV2(nn.Module):
    def __init__(self, inp: int, oup: int, stride: int, expand_ratio: int):
        super().__init__()
        hidden_dim = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers: List[nn.Module] = []
        if expand_ratio != 1:
            layers.append(ConvBNAct(inp, hidden_dim, kernel_size=1))
        layers += [ConvBNAct(hidden_dim, hidden_dim, stride=stride, groups=hidden_dim),
                   nn.Conv2d(hidden_dim, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)
        self.out_channels = oup

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2(nn.Module):
    def __init__(self, num_classes: int = 1000, width_mult: float = 1.0, round_nearest: int = 8, dropout: float = 0.2):
        super().__init__()
        input_channel, last_channel = 32, 1280
        setting = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
                   [6, 320, 1, 1]]
        input_channel = _make_divisible(input_channel * width_mult, round_nearest)
        self.last_channel = _make_divisible(last_channel * max(1.0, width_mult), round_nearest)
        features: List[nn.Module] = [ConvBNAct(3, input_channel, stride=2)]
        for t, c, n, s in setting:
            output_channel = _make_divisible(c * width_mult, round_nearest)
            for i in range(n):
                features.append(InvertedResidualV2(input_channel, output_channel, s if i == 0 else 1, t))
                input_channel = output_channel
        features.append(ConvBNAct(input_channel, self.last_channel, kernel_size=1))
        self.features = nn.Sequential(*features)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout), nn.Linear(self.last_channel, num_classes))
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

    def forward(self, x):
        x = F.adaptive_avg_pool2d(self.features(x), (1, 1))
        return self.classifier(torch.flatten(x, 1))


def mobilenet_v2(pretrained=False, **kw): return MobileNetV2(**kw)


# ------------------------------------------------------------------------------------ ShuffleNetV2
def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    b, c, h, w = x.size()
    x = x.view(b, groups, c // groups, h, w).transpose(1, 2).contiguous()
    return x.view(b, c, h, w)


class ShuffleUnit(nn.Module):
    def __init__(self, inp: int, oup: int, stride: int):
        super().__init__()
        self.stride = stride
        bf = oup // 2
        if stride > 1:
            self.branch1 = nn.Sequential(
                nn.Conv2d(inp, inp, 3, stride, 1, bias=False, groups=inp), nn.BatchNorm2d(inp),
                nn.Conv2d(inp, bf, 1, 1, 0, bias=False), nn.BatchNorm2d(bf), nn.ReLU(inplace=True))
        else:
            self.branch1 = nn.Sequential()
        self.branch2 = nn.Sequential(
            nn.Conv2d(inp if stride > 1 else bf, bf, 1, 1, 0, bias=False), nn.BatchNorm2d(bf), nn.ReLU(inplace=True),
            nn.Conv2d(bf, bf, 3, stride, 1, bias=False, groups=bf), nn.BatchNorm2d(bf),
            nn.Conv2d(bf, bf, 1, 1, 0, bias=False), nn.BatchNorm2d(bf), nn.ReLU(inplace=True))

    def forward(self, x):
        if self.stride == 1:
            x1, x2 = x.chunk(2, dim=1)
            out = torch.cat((x1, self.branch2(x2)), dim=1)
        else:
            out = torch.cat((self.branch1(x), self.branch2(x)), dim=1)
        return channel_shuffle(out, 2)


class ShuffleNetV2(nn.Module):
    def __init__(self, stages_repeats: List[int], stages_out_channels: List[int], num_classes: int = 1000):
        super().__init__()
        input_channels = 3
        output_channels = stages_out_channels[0]
        self.conv1 = nn.Sequential(nn.Conv2d(input_channels, output_channels, 3, 2, 1, bias=False),
                                   nn.BatchNorm2d(output_channels), nn.ReLU(inplace=True))
        input_channels = output_channels
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        for name, repeats, output_channels in zip(["stage2", "stage3", "stage4"], stages_repeats,
                                                  stages_out_channels[1:]):
            seq = [ShuffleUnit(input_channels, output_channels, 2)]
            seq += [ShuffleUnit(output_channels, output_channels, 1) for _ in range(repeats - 1)]
            setattr(self, name, nn.Sequential(*seq))
            input_channels = output_channels
        output_channels = stages_out_channels[-1]
        self.conv5 = nn.Sequential(nn.Conv2d(input_channels, output_channels, 1, 1, 0, bias=False),
                                   nn.BatchNorm2d(output_channels), nn.ReLU(inplace=True))
        self.fc = nn.Linear(output_channels, num_classes)

    def forward(self, x):
        x = self.maxpool(self.conv1(x))
        x = self.conv5(self.stage4(self.stage3(self.stage2(x))))
        return self.fc(x.mean([2, 3]))


def shufflenet_v2_x0_5(pretrained=False, **kw): return ShuffleNetV2([4, 8, 4], [24, 48, 96, 192, 1024], **kw)
def shufflenet_v2_x1_0(pretrained=False, **kw): return ShuffleNetV2([4, 8, 4], [24, 116, 232, 464, 1024], **kw)
def shufflenet_v2_x1_5(pretrained=False, **kw): return ShuffleNetV2([4, 8, 4], [24, 176, 352, 704, 1024], **kw)
def shufflenet_v2_x2_0(pretrained=False, **kw): return ShuffleNetV2([4, 8, 4], [24, 244, 488, 976, 2048], **kw)
