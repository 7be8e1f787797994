"""Metric helpers: learning-rate getter, running-average meter and top-k accuracy.

Behavioural contract: ``get_learning_rate`` returns the first param group's lr
(`utils.py:65-69`); the meter exposes ``val/avg/sum/count`` with an ``n``-weighted ``update`` and a
``"<name> <val> (<avg>)"`` string form (`utils.py:78-102`); accuracy is a 0-d tensor FRACTION of the
batch (`utils.py:105-111`; the README's Top-1 column is in percent -- SURVEY Q10).
"""
from __future__ import annotations

import torch


def get_learning_rate(optimizer) -> float:
    groups = optimizer.param_groups
    return groups[0]["lr"]


class AverageMeter:
    """Weighted running average of a scalar (python number or 0-d tensor)."""

    def __init__(self, name: str, fmt: str = ":f"):
        self.name, self.fmt = name, fmt
        self.val = self.avg = self.sum = 0
        self.count = 0

    def reset(self) -> None:
        self.__init__(self.name, self.fmt)

    def update(self, val, n: int = 1) -> None:
        self.val = val
        self.count += n
        self.sum = self.sum + val * n
        self.avg = self.sum / self.count

    def __str__(self) -> str:
        spec = self.fmt.lstrip(":")
        return f"{self.name} {format(self.val, spec)} ({format(self.avg, spec)})"


def accuracy(scores: torch.Tensor, targets: torch.Tensor, k: int = 1) -> torch.Tensor:
    """Fraction of rows whose top-``k`` predictions contain the target (0-d tensor)."""
    topk = torch.topk(scores, k, dim=1, largest=True, sorted=True).indices
    hits = (topk == targets.long().unsqueeze(1)).any(dim=1)
    return hits.float().sum() / targets.size(0)
