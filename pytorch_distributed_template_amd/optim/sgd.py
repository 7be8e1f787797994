"""Fused SGD (momentum, weight decay) over :class:`~.flat.FlatParams`.

Semantics are ``torch.optim.SGD(params, lr, momentum, weight_decay)`` with dampening 0 and no
nesterov (the reference's optimizer, `distributed.py:148`, `T/optim/sgd.py:346-378`):

    d_p = grad + weight_decay * p;  buf = d_p (first step) | momentum * buf + d_p;  p -= lr * buf

The momentum buffer starts at zero, so ``momentum*0 + d_p`` reproduces the first-step rule even
when an AMP-skipped step leaves it untouched.  On a GPU one kernel launch updates every parameter,
folding in the gradient pre-scale (1/world for the DDP mean, 1/loss_scale for AMP) and the
device-side skip-on-overflow, and writes the 16-bit compute copy of each parameter.
"""
from __future__ import annotations

from typing import Optional

import torch

from .flat import FlatParams


class FusedSGD:
    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9, weight_decay: float = 1e-4):
        self.flat = flat
        # ``param_groups`` mirrors torch.optim for get_learning_rate() / LR schedulers
        self.param_groups = [{"params": flat.params, "lr": lr, "initial_lr": lr, "momentum": momentum,
                              "weight_decay": weight_decay, "dampening": 0, "nesterov": False}]
        self.defaults = dict(self.param_groups[0])
        self.step_count = 0
        self.post_step_hooks = []

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def zero_grad(self, set_to_none: bool = False) -> None:
        """Zero the flat gradient buffer (the gradient views stay attached)."""
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, loss_scale: Optional[torch.Tensor] = None,
             found_inf: Optional[torch.Tensor] = None) -> None:
        g = self.param_groups[0]
        f = self.flat
        if f.data.is_cuda:
            from ..ops import native
            native.C.sgd(f.data, f.grad, f.momentum, f.shadow, None, g["lr"], g["momentum"], g["weight_decay"],
                         grad_scale, loss_scale, found_inf, self.step_count == 0)
        else:
            skip = found_inf is not None and bool(found_inf.item() != 0)
            if not skip:
                scale = grad_scale / (float(loss_scale.item()) if loss_scale is not None else 1.0)
                d = f.grad * scale + g["weight_decay"] * f.data
                if g["momentum"] != 0:
                    f.momentum.mul_(g["momentum"]).add_(d)
                    d = f.momentum
                f.data.add_(d, alpha=-g["lr"])
                if f.shadow is not None:
                    f.shadow.copy_(f.data)
        self.step_count += 1
        for h in self.post_step_hooks:
            h()

    def state_dict(self) -> dict:
        """torch.optim.SGD-compatible layout (per-parameter momentum_buffer)."""
        state = {}
        for s, p in zip(self.flat.slots, self.flat.params):
            buf = self.flat.momentum[s.offset:s.offset + s.numel]
            if s.channels_last:
                co, ci, kh, kw = s.shape
                buf = buf.view(co, kh, kw, ci).permute(0, 3, 1, 2)
            else:
                buf = buf.view(s.shape)
            state[s.index] = {"momentum_buffer": buf.detach().cpu().contiguous()}
        groups = [{k: v for k, v in self.param_groups[0].items() if k != "params"}]
        groups[0]["params"] = list(range(len(self.flat.slots)))
        return {"state": state, "param_groups": groups, "step_count": self.step_count}

    def load_state_dict(self, sd: dict) -> None:
        for s in self.flat.slots:
            st = sd["state"].get(s.index) or sd["state"].get(str(s.index))
            if st is None or st.get("momentum_buffer") is None:
                continue
            buf = self.flat.momentum[s.offset:s.offset + s.numel]
            src = st["momentum_buffer"].to(buf.device, torch.float32)
            if s.channels_last:
                co, ci, kh, kw = s.shape
                buf.view(co, kh, kw, ci).permute(0, 3, 1, 2).copy_(src)
            else:
                buf.view(s.shape).copy_(src)
        pg = sd["param_groups"][0]
        for k in ("lr", "momentum", "weight_decay", "initial_lr"):
            if k in pg:
                self.param_groups[0][k] = pg[k]
        self.step_count = int(sd.get("step_count", 1))
