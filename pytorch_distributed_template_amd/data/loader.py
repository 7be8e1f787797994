"""Data pipeline assembly (reference C16-C18: ImageFolder + transforms, DistributedSampler,
``DataLoader(batch, num_workers=-j, pin_memory=True)``; `distributed.py:157-179`).

GPU-side additions:
* :class:`DevicePrefetcher` copies the next batch host->device on a side HIP stream while the current
  step runs (the reference's ``.cuda(non_blocking=True)`` happens on the compute stream);
* :class:`DeviceSyntheticLoader` produces synthetic ImageNet-shaped batches directly in HBM (no PCIe
  traffic, no CPU decode), with the same per-rank sample counts as the distributed sampler;
* native single-process DataParallel on several GPUs gets :class:`ShardedBatch` objects instead: the node batch
  is split the way ``nn.DataParallel`` scatters it (``torch.tensor_split`` along dim 0) and shard i goes
  host -> GPU i directly (:class:`ScatterPrefetcher`), or is generated on GPU i (synthetic data), so no batch
  crosses GPU 0 on its way to the other replicas.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
from torch.utils.data import DataLoader

from .datasets import ImageFolder, SyntheticImageNet, lazy_pil_loader, pil_loader
from .sampler import DistributedSampler
from .transforms import normalize_on_device, train_transform, val_transform


class ShardedBatch:
    """A node batch already split over devices: ``parts[i]`` lives on device i.  ``size(0)`` is the node batch."""

    def __init__(self, parts):
        self.parts = list(parts)

    def size(self, dim: int = 0) -> int:
        if dim != 0:
            return self.parts[0].size(dim)
        return sum(p.size(0) for p in self.parts)

    @property
    def shape(self):
        return (self.size(0),) + tuple(self.parts[0].shape[1:])


def shard_bounds(n: int, parts: int):
    """Row ranges of ``torch.tensor_split(range(n), parts)`` (nn.DataParallel's scatter)."""
    q, r = divmod(n, parts)
    out, lo = [], 0
    for i in range(parts):
        hi = lo + q + (1 if i < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


class DeviceSyntheticLoader:
    """Synthetic batches generated on the device.

    ``len()`` and the last-batch size follow ``DistributedSampler(n) + DataLoader(batch)``; the
    contents come from a small pool of distinct device-resident batches (deterministic in the seed).
    """

    def __init__(self, n_samples: int, batch_size: int, world: int, rank: int, device, image_size: int = 224,
                 num_classes: int = 1000, seed: int = 0, pool: int = 4):
        self.num_samples = math.ceil(n_samples / world)
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.image_size = image_size
        self.num_classes = num_classes
        self.seed = seed + 7919 * rank
        self.pool_n = pool
        self.epoch = 0
        self._pool = None

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __len__(self) -> int:
        return math.ceil(self.num_samples / self.batch_size)

    def _make_pool(self):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed)
        bs = min(self.batch_size, self.num_samples)
        self._pool = [(torch.randn(bs, 3, self.image_size, self.image_size, device=self.device, generator=g),
                       torch.randint(0, self.num_classes, (bs,), device=self.device, generator=g))
                      for _ in range(self.pool_n)]

    def __iter__(self):
        if self._pool is None:
            self._make_pool()
        n = len(self)
        for i in range(n):
            x, t = self._pool[(i + self.epoch) % self.pool_n]
            bs = min(self.batch_size, self.num_samples - i * self.batch_size)
            yield (x[:bs], t[:bs]) if bs < x.shape[0] else (x, t)


class ShardedDeviceSyntheticLoader:
    """Synthetic node batches for native DataParallel: shard i of every batch is generated on device i."""

    def __init__(self, n_samples: int, batch_size: int, devices, image_size: int = 224, num_classes: int = 1000,
                 seed: int = 0, pool: int = 4):
        self.inner = [DeviceSyntheticLoader(n_samples, batch_size, 1, 0, d, image_size, num_classes, seed + 104729 * i,
                                            pool) for i, d in enumerate(devices)]
        self.devices = [torch.device(d) for d in devices]
        self.num_samples = n_samples
        self.batch_size = batch_size

    def set_epoch(self, epoch: int) -> None:
        for it in self.inner:
            it.set_epoch(epoch)

    def __len__(self) -> int:
        return math.ceil(self.num_samples / self.batch_size)

    def __iter__(self):
        for it in self.inner:
            if it._pool is None:
                it._make_pool()
        n = len(self)
        for i in range(n):
            bs = min(self.batch_size, self.num_samples - i * self.batch_size)
            xs, ts = [], []
            for k, ((lo, hi), it) in enumerate(zip(shard_bounds(bs, len(self.devices)), self.inner)):
                x, t = it._pool[(i + it.epoch) % it.pool_n]
                xs.append(x[:hi - lo])
                ts.append(t[:hi - lo])
            yield ShardedBatch(xs), ShardedBatch(ts)


class ScatterPrefetcher:
    """Host loader -> per-device shards: batch i+1's shard k is copied host -> GPU k on GPU k's side stream while
    step i runs (the DataParallel counterpart of :class:`DevicePrefetcher`)."""

    def __init__(self, loader, devices, normalize_uint8: bool = False):
        self.loader = loader
        self.devices = [torch.device(d) for d in devices]
        self.streams = [torch.cuda.Stream(device=d) for d in self.devices]
        self.normalize_uint8 = normalize_uint8

    def __len__(self) -> int:
        return len(self.loader)

    @property
    def sampler(self):
        return getattr(self.loader, "sampler", None)

    def _copy(self, batch):
        x, t = batch
        xs, ts = [], []
        for (lo, hi), d, s in zip(shard_bounds(x.shape[0], len(self.devices)), self.devices, self.streams):
            with torch.cuda.device(d), torch.cuda.stream(s):
                xi = x[lo:hi].to(d, non_blocking=True)
                if self.normalize_uint8 and xi.dtype == torch.uint8:
                    xi = normalize_on_device(xi)
                xs.append(xi)
                ts.append(t[lo:hi].to(d, non_blocking=True))
        return xs, ts

    def __iter__(self):
        it = iter(self.loader)
        try:
            nxt = self._copy(next(it))
        except StopIteration:
            return
        while nxt is not None:
            xs, ts = nxt
            for d, s, xi, ti in zip(self.devices, self.streams, xs, ts):
                cur = torch.cuda.current_stream(d)
                cur.wait_stream(s)
                xi.record_stream(cur)
                ti.record_stream(cur)
            try:
                nxt = self._copy(next(it))
            except StopIteration:
                nxt = None
            yield ShardedBatch(xs), ShardedBatch(ts)


class DevicePrefetcher:
    """Wrap a host DataLoader: batch i+1 is copied to the device on a side stream during step i."""

    def __init__(self, loader, device, normalize_uint8: bool = False):
        self.loader = loader
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        # uint8 batches: keep them uint8 (the native engine normalises inside its stem kernel) or
        # normalise on the side stream (torch engine)
        self.normalize_uint8 = normalize_uint8

    def __len__(self) -> int:
        return len(self.loader)

    @property
    def sampler(self):
        return getattr(self.loader, "sampler", None)

    def _copy(self, batch):
        x, t = batch
        with torch.cuda.stream(self.stream):
            x = x.to(self.device, non_blocking=True)
            if self.normalize_uint8 and x.dtype == torch.uint8:
                x = normalize_on_device(x)
            return x, t.to(self.device, non_blocking=True)

    def __iter__(self):
        it = iter(self.loader)
        try:
            nxt = self._copy(next(it))
        except StopIteration:
            return
        cur_stream = torch.cuda.current_stream(self.device)
        while nxt is not None:
            cur_stream.wait_stream(self.stream)
            x, t = nxt
            x.record_stream(cur_stream)
            t.record_stream(cur_stream)
            try:
                nxt = self._copy(next(it))
            except StopIteration:
                nxt = None
            yield x, t


def build_loaders(args, world: int, rank: int, device, distributed: bool, batch_size: int, shard_devices=None):
    """Returns ``(train_loader, val_loader, train_sampler, val_sampler)``.

    ``batch_size`` is the per-process batch (the reference divides the node-total ``-b`` by the
    process count for DDP, `distributed.py:143`; DataParallel uses the node-total batch).
    ``shard_devices`` (native DataParallel on > 1 GPU): yield :class:`ShardedBatch` pairs, shard i on device i."""
    device = torch.device(device)
    on_gpu = device.type == "cuda"
    # gpu_normalize: samples stay uint8 on the host and cross PCIe as uint8 (K28); "native" keeps them
    # uint8 on the device too (fused into the stem kernel), "torch" normalises after the copy
    gpu_norm = getattr(args, "gpu_normalize_mode", "off") if on_gpu else "off"
    u8 = gpu_norm in ("native", "torch")
    if args.synthetic and on_gpu and shard_devices:
        tr = ShardedDeviceSyntheticLoader(args.synthetic_train_size, batch_size, shard_devices, args.image_size,
                                          args.num_classes, seed=args.seed or 0)
        va = ShardedDeviceSyntheticLoader(args.synthetic_val_size, batch_size, shard_devices, args.image_size,
                                          args.num_classes, seed=(args.seed or 0) + 1, pool=2)
        return tr, va, tr, va
    if args.synthetic and on_gpu:
        tr = DeviceSyntheticLoader(args.synthetic_train_size, batch_size, world, rank, device, args.image_size,
                                   args.num_classes, seed=args.seed or 0)
        va = DeviceSyntheticLoader(args.synthetic_val_size, batch_size, world, rank, device, args.image_size,
                                   args.num_classes, seed=(args.seed or 0) + 1, pool=2)
        return tr, va, tr, va
    if args.synthetic:
        train_ds = SyntheticImageNet(args.synthetic_train_size, args.image_size, args.num_classes, seed=0, uint8=u8)
        val_ds = SyntheticImageNet(args.synthetic_val_size, args.image_size, args.num_classes, seed=1, uint8=u8)
    else:
        draft = bool(getattr(args, "jpeg_draft", False))
        ld = lazy_pil_loader if draft else pil_loader
        train_ds = ImageFolder(os.path.join(args.data, "train"),
                               train_transform(args.image_size, gpu_normalize=u8, draft=draft), loader=ld)
        resize = round(args.image_size * 256 / 224)  # 256 for the 224 crop, 342 for Inception-v3's 299
        val_ds = ImageFolder(os.path.join(args.data, "val"),
                             val_transform(args.image_size, resize, gpu_normalize=u8, draft=draft), loader=ld)
    if distributed:
        train_sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank)
        val_sampler = DistributedSampler(val_ds, num_replicas=world, rank=rank)
        train_loader = DataLoader(train_ds, batch_size=batch_size, num_workers=args.workers, pin_memory=on_gpu,
                                  sampler=train_sampler, persistent_workers=args.workers > 0)
        val_loader = DataLoader(val_ds, batch_size=batch_size, num_workers=args.workers, pin_memory=on_gpu,
                                sampler=val_sampler, persistent_workers=args.workers > 0)
    else:
        train_sampler = val_sampler = None
        train_loader = DataLoader(train_ds, batch_size=batch_size, shuffle=True, num_workers=args.workers,
                                  pin_memory=on_gpu, persistent_workers=args.workers > 0)
        val_loader = DataLoader(val_ds, batch_size=batch_size, shuffle=False, num_workers=args.workers,
                                pin_memory=on_gpu, persistent_workers=args.workers > 0)
    if on_gpu and shard_devices:
        nz = gpu_norm == "torch"
        train_loader = ScatterPrefetcher(train_loader, shard_devices, normalize_uint8=nz)
        val_loader = ScatterPrefetcher(val_loader, shard_devices, normalize_uint8=nz)
    elif on_gpu:
        nz = gpu_norm == "torch"
        train_loader = DevicePrefetcher(train_loader, device, normalize_uint8=nz)
        val_loader = DevicePrefetcher(val_loader, device, normalize_uint8=nz)
    return train_loader, val_loader, train_sampler, val_sampler
