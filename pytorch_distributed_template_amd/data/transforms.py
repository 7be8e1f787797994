"""Image transforms with torchvision semantics (torchvision is not installed here).

Reference pipelines (`dataparallel.py:133-151`):
  train: RandomResizedCrop(224) -> RandomHorizontalFlip() -> ToTensor() -> Normalize(mean, std)
  val:   Resize(256) -> CenterCrop(224) -> ToTensor() -> Normalize(mean, std)

Implemented on PIL images + numpy; random draws use ``torch``'s global RNG exactly like
torchvision (``torch.empty(1).uniform_``, ``torch.randint``, ``torch.rand``), so a seeded run draws
the same crop boxes.

``draft=True`` (``--jpeg-draft``, off by default): JPEG decode at reduced size.  The crop box / resize target
is known from the file header before any pixel is decoded, so libjpeg is asked (``Image.draft``) for the
largest DCT-domain downscale (1/2, 1/4, 1/8) that still leaves at least the output resolution inside the
crop; decode cost falls roughly with the pixel count.  Pixels differ slightly from a full decode
(DCT-domain vs bilinear downscale), so it is an opt-in throughput option (tools/data_bench.py).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch
from PIL import Image

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class Compose:
    def __init__(self, transforms: Sequence):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


def _size(img: Image.Image) -> Tuple[int, int]:
    return img.size  # (w, h)


def _draft(img: Image.Image, factor: float) -> Tuple[float, float]:
    """Ask a not-yet-decoded JPEG for a DCT-domain downscale of up to ``factor`` (>= 2 to matter); returns
    the (x, y) scale actually applied (1.0 when not a JPEG / already decoded / factor < 2)."""
    if factor < 2 or getattr(img, "format", None) != "JPEG" or not getattr(img, "tile", None):  # tile: undecoded
        return 1.0, 1.0
    W, H = img.size
    img.draft("RGB", (max(1, math.ceil(W / factor)), max(1, math.ceil(H / factor))))
    return img.size[0] / W, img.size[1] / H


class Resize:
    """Resize the shorter side to ``size`` (int) keeping the aspect ratio, bilinear."""

    def __init__(self, size, interpolation=Image.BILINEAR, draft: bool = False):
        self.size = size
        self.interpolation = interpolation
        self.draft = draft

    def __call__(self, img: Image.Image) -> Image.Image:
        if self.draft and not isinstance(self.size, (tuple, list)):
            _draft(img, min(_size(img)) / self.size)
        if isinstance(self.size, (tuple, list)):
            h, w = self.size
            return img.resize((w, h), self.interpolation)
        w, h = _size(img)
        short, long_ = (w, h) if w <= h else (h, w)
        if short == self.size:
            return img
        new_short, new_long = self.size, int(self.size * long_ / short)
        nw, nh = (new_short, new_long) if w <= h else (new_long, new_short)
        return img.resize((nw, nh), self.interpolation)


class CenterCrop:
    def __init__(self, size):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def __call__(self, img: Image.Image) -> Image.Image:
        w, h = _size(img)
        th, tw = self.size
        if tw > w or th > h:  # pad like torchvision, then crop
            pad_img = Image.new(img.mode, (max(w, tw), max(h, th)))
            pad_img.paste(img, ((max(w, tw) - w) // 2, (max(h, th) - h) // 2))
            img = pad_img
            w, h = _size(img)
        top = int(round((h - th) / 2.0))
        left = int(round((w - tw) / 2.0))
        return img.crop((left, top, left + tw, top + th))


class RandomResizedCrop:
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), interpolation=Image.BILINEAR,
                 draft: bool = False):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.scale = scale
        self.ratio = ratio
        self.interpolation = interpolation
        self.draft = draft

    @staticmethod
    def get_params(img: Image.Image, scale, ratio):
        width, height = _size(img)
        area = height * width
        log_ratio = torch.log(torch.tensor(ratio))
        for _ in range(10):
            target_area = area * torch.empty(1).uniform_(scale[0], scale[1]).item()
            aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1])).item()
            w = int(round(math.sqrt(target_area * aspect_ratio)))
            h = int(round(math.sqrt(target_area / aspect_ratio)))
            if 0 < w <= width and 0 < h <= height:
                i = torch.randint(0, height - h + 1, size=(1,)).item()
                j = torch.randint(0, width - w + 1, size=(1,)).item()
                return i, j, h, w
        in_ratio = float(width) / float(height)
        if in_ratio < min(ratio):
            w = width
            h = int(round(w / min(ratio)))
        elif in_ratio > max(ratio):
            h = height
            w = int(round(h * max(ratio)))
        else:
            w, h = width, height
        return (height - h) // 2, (width - w) // 2, h, w

    def __call__(self, img: Image.Image) -> Image.Image:
        i, j, h, w = self.get_params(img, self.scale, self.ratio)  # on the header size: no decode yet
        th, tw = self.size
        if self.draft:
            fx, fy = _draft(img, min(w / tw, h / th))
            if (fx, fy) != (1.0, 1.0):  # crop box in the reduced image (float box: no re-rounding)
                return img.resize((tw, th), self.interpolation, box=(j * fx, i * fy, (j + w) * fx, (i + h) * fy))
        return img.crop((j, i, j + w, i + h)).resize((tw, th), self.interpolation)


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img: Image.Image) -> Image.Image:
        if torch.rand(1).item() < self.p:
            return img.transpose(Image.FLIP_LEFT_RIGHT)
        return img


class ToTensor:
    """HWC uint8 PIL image -> CHW float32 tensor in [0, 1]."""

    def __call__(self, img: Image.Image) -> torch.Tensor:
        arr = np.asarray(img.convert("RGB"), dtype=np.uint8)
        return torch.from_numpy(arr.copy()).permute(2, 0, 1).float().div_(255.0)


class ToUint8Tensor:
    """HWC uint8 PIL image -> CHW uint8 tensor (normalisation then happens on the GPU)."""

    def __call__(self, img: Image.Image) -> torch.Tensor:
        arr = np.asarray(img.convert("RGB"), dtype=np.uint8)
        return torch.from_numpy(arr.copy()).permute(2, 0, 1).contiguous()


class Normalize:
    def __init__(self, mean: List[float], std: List[float]):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return (t - self.mean) / self.std


def train_transform(image_size: int = 224, gpu_normalize: bool = False, draft: bool = False) -> Compose:
    """Reference train transform (`dataparallel.py:133-141`); with ``gpu_normalize`` the samples stay
    uint8 (4x less host->device traffic) and ToTensor + Normalize happen on the GPU."""
    tail = [ToUint8Tensor()] if gpu_normalize else [ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)]
    return Compose([RandomResizedCrop(image_size, draft=draft), RandomHorizontalFlip()] + tail)


def val_transform(image_size: int = 224, resize: int = 256, gpu_normalize: bool = False,
                  draft: bool = False) -> Compose:
    tail = [ToUint8Tensor()] if gpu_normalize else [ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)]
    return Compose([Resize(resize, draft=draft), CenterCrop(image_size)] + tail)


def normalize_on_device(x: torch.Tensor) -> torch.Tensor:
    """uint8 NCHW batch -> normalised float32 (the GPU half of ``gpu_normalize`` for the torch engine)."""
    mean = torch.tensor(IMAGENET_MEAN, device=x.device).view(1, -1, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=x.device).view(1, -1, 1, 1)
    return (x.float().div_(255.0) - mean) / std
