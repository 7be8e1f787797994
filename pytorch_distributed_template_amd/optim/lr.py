"""Learning-rate schedule (reference C15: only ``--lr-scheduler steplr`` is accepted; it builds
``MultiStepLR(optimizer, milestones=args.step, gamma)`` and calls ``lr_scheduler.step(epoch)`` at the
start of every epoch, `distributed.py:150-154,192`).

The deprecated ``step(epoch)`` form evaluates the closed form
``lr = base_lr * gamma ** bisect_right(milestones, epoch)`` (`T/optim/lr_scheduler.py:770`), which is
what :class:`MultiStepLR` implements directly: with the defaults the epochs 0..4 run at
0.1, 0.1, 0.1, 0.01, 0.001.
"""
from __future__ import annotations

from bisect import bisect_right
from typing import List, Optional


class MultiStepLR:
    def __init__(self, optimizer, milestones: List[int], gamma: float = 0.1):
        self.optimizer = optimizer
        self.milestones = sorted(int(m) for m in milestones)
        self.gamma = gamma
        for g in optimizer.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self.base_lrs = [g["initial_lr"] for g in optimizer.param_groups]
        self.last_epoch = -1

    def lr_at(self, epoch: int) -> List[float]:
        k = bisect_right(self.milestones, epoch)
        return [b * self.gamma ** k for b in self.base_lrs]

    def step(self, epoch: Optional[int] = None) -> None:
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        for g, lr in zip(self.optimizer.param_groups, self.lr_at(self.last_epoch)):
            g["lr"] = lr

    def get_last_lr(self) -> List[float]:
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self) -> dict:
        return {"milestones": self.milestones, "gamma": self.gamma, "base_lrs": self.base_lrs,
                "last_epoch": self.last_epoch}

    def load_state_dict(self, sd: dict) -> None:
        self.milestones = list(sd["milestones"])
        self.gamma = sd["gamma"]
        self.base_lrs = list(sd["base_lrs"])
        self.last_epoch = sd["last_epoch"]


def build_scheduler(name: str, optimizer, milestones, gamma):
    if name != "steplr":
        raise ValueError("invalid lr_scheduler={}".format(name))
    return MultiStepLR(optimizer, milestones, gamma)
