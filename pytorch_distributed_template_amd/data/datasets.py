"""Datasets: ImageFolder (reference C16) and synthetic ImageNet-shaped data.

``ImageFolder(root)`` follows torchvision: classes are the sorted sub-directory names, samples are
all files with an image extension under them (sorted walk), target = class index.
``SyntheticImageNet`` yields deterministic ``(3 x S x S float32, label)`` pairs derived from the
sample index, so every rank/worker sees the same data for the same index without any files.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Tuple

import torch
from PIL import Image
from torch.utils.data import Dataset

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def pil_loader(path: str) -> Image.Image:
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


def lazy_pil_loader(path: str) -> Image.Image:
    """Header-only open: pixels are decoded by the first transform that needs them, so a JPEG can still be
    asked for a reduced-size decode (``Image.draft``, transforms ``draft=True``).  Non-RGB modes are
    converted by ToTensor / ToUint8Tensor at the end of the pipeline."""
    return Image.open(path)


def find_classes(directory: str) -> Tuple[List[str], dict]:
    classes = sorted(e.name for e in os.scandir(directory) if e.is_dir())
    if not classes:
        raise FileNotFoundError(f"Couldn't find any class folder in {directory}.")
    return classes, {c: i for i, c in enumerate(classes)}


class ImageFolder(Dataset):
    def __init__(self, root: str, transform: Optional[Callable] = None, target_transform: Optional[Callable] = None,
                 loader: Callable = pil_loader):
        self.root = root
        self.transform = transform
        self.target_transform = target_transform
        self.loader = loader
        self.classes, self.class_to_idx = find_classes(root)
        samples = []
        for cls in self.classes:
            d = os.path.join(root, cls)
            for dirpath, _, fnames in sorted(os.walk(d, followlinks=True)):
                for fn in sorted(fnames):
                    if fn.lower().endswith(IMG_EXTENSIONS):
                        samples.append((os.path.join(dirpath, fn), self.class_to_idx[cls]))
        if not samples:
            raise FileNotFoundError(f"Found no valid image file in {root}")
        self.samples = samples
        self.targets = [s[1] for s in samples]

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, index: int):
        path, target = self.samples[index]
        img = self.loader(path)
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target


class SyntheticImageNet(Dataset):
    """Deterministic random images (standard-normal, i.e. already "normalised") and labels."""

    def __init__(self, size: int = 1281167, image_size: int = 224, num_classes: int = 1000, seed: int = 0,
                 uint8: bool = False):
        self.size = size
        self.image_size = image_size
        self.num_classes = num_classes
        self.seed = seed
        self.uint8 = uint8  # raw-pixel samples (the gpu_normalize pipeline)

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, index: int):
        g = torch.Generator()
        g.manual_seed(self.seed * 1000003 + index)
        if self.uint8:
            img = torch.randint(0, 256, (3, self.image_size, self.image_size), generator=g, dtype=torch.uint8)
        else:
            img = torch.randn(3, self.image_size, self.image_size, generator=g)
        target = int(torch.randint(0, self.num_classes, (1,), generator=g).item())
        return img, target
