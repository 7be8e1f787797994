"""Distributed sampler with the exact partition of ``torch.utils.data.DistributedSampler``.

Reference usage: ``DistributedSampler(train_dataset)`` / ``DistributedSampler(val_dataset)`` with
defaults (shuffle, seed 0, no drop_last) and ``set_epoch(epoch)`` every epoch
(`distributed.py:167,177,188-189`).  Partition: a permutation drawn from a CPU
generator seeded with ``seed + epoch``, padded by wrapping to a multiple of the world size, then
strided ``indices[rank::world]`` -- so every rank gets the same number of samples (and the
validation set is padded with duplicates, like the reference).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
import torch.distributed as dist
from torch.utils.data import Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        n = len(dataset)
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def _global_order(self):
        n = len(self.dataset)
        if self.shuffle:
            gen = torch.Generator()
            gen.manual_seed(self.seed + self.epoch)
            order = torch.randperm(n, generator=gen).tolist()
        else:
            order = list(range(n))
        if self.drop_last:
            return order[:self.total_size]
        short = self.total_size - len(order)
        while short > 0:  # wrap around (repeatedly if the dataset is tiny)
            take = order[:short]
            order += take
            short -= len(take)
        return order

    def __iter__(self) -> Iterator[int]:
        order = self._global_order()
        assert len(order) == self.total_size
        mine = order[self.rank:self.total_size:self.num_replicas]
        assert len(mine) == self.num_samples
        return iter(mine)

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
