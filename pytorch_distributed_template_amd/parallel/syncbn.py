"""Cross-replica BatchNorm (reference C11: ``nn.SyncBatchNorm.convert_sync_batchnorm(model)`` behind
``--sync_batchnorm``, `distributed_syncBN_amp.py:142-147`; upstream mechanics SURVEY §3.5).

Two implementations, one semantics:

* native path (GPU): :class:`~..models.executor.ResNetExecutor` takes ``syncbn_group``; each BN
  layer all-reduces its fp64 (sum, sum of squares) batch statistics -- one RCCL all-reduce of 2C values
  per layer in forward, one of the 2C backward sums in backward, no host synchronisation (counts are
  equal on every rank because the distributed sampler pads every rank to the same length);
* torch path (any device, incl. ``gloo`` on CPU): :class:`SyncBatchNorm` below, an autograd function
  with the same two collectives.

Semantics match upstream SyncBN: training-mode statistics are over the union of all ranks' batches,
running statistics use the unbiased global variance, ``weight``/``bias`` gradients are the LOCAL sums
(DDP then averages them like any parameter), the input gradient uses the GLOBAL means.
Eval mode is plain BatchNorm with running statistics.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, group):
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xf = x.float()
        local_n = x.numel() // C
        stats = torch.cat([xf.sum(dims).double(), (xf * xf).sum(dims).double(),
                           torch.tensor([float(local_n)], dtype=torch.float64, device=x.device)])
        dist.all_reduce(stats, group=group)
        n = stats[2 * C]
        mean = stats[:C] / n
        var = (stats[C:2 * C] / n - mean * mean).clamp_min(0)
        invstd = torch.rsqrt(var + eps)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(momentum * mean.float())
                running_var.mul_(1 - momentum).add_(momentum * (var * n / (n - 1).clamp_min(1)).float())
        shape = [1, C] + [1] * (x.dim() - 2)
        meanf, invf = mean.float().view(shape), invstd.float().view(shape)
        xhat = (xf - meanf) * invf
        y = xhat * weight.float().view(shape) + bias.float().view(shape)
        ctx.save_for_backward(xhat, weight, invf)
        ctx.group, ctx.n = group, float(n.item()) if n.device.type == "cpu" else n
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        xhat, weight, invf = ctx.saved_tensors
        C = xhat.shape[1]
        dims = [0] + list(range(2, xhat.dim()))
        dyf = dy.float()
        sum_dy = dyf.sum(dims)
        sum_dy_xhat = (dyf * xhat).sum(dims)
        both = torch.cat([sum_dy, sum_dy_xhat]).double()
        dist.all_reduce(both, group=ctx.group)
        n = ctx.n
        shape = [1, C] + [1] * (xhat.dim() - 2)
        mean_dy = (both[:C] / n).float().view(shape)
        mean_dy_xhat = (both[C:] / n).float().view(shape)
        dx = weight.float().view(shape) * invf * (dyf - mean_dy - xhat * mean_dy_xhat)
        return dx.to(dy.dtype), sum_dy_xhat.to(weight.dtype), sum_dy.to(weight.dtype), None, None, None, None, None


class SyncBatchNorm(nn.BatchNorm2d):
    """Drop-in for ``nn.BatchNorm2d`` (same parameters/buffers/state-dict keys)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, process_group=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        self.process_group = process_group

    def forward(self, x):
        world = dist.get_world_size(self.process_group) if dist.is_available() and dist.is_initialized() else 1
        if not self.training or world == 1:
            return super().forward(x)
        if self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
        mom = self.momentum if self.momentum is not None else 0.1
        return _SyncBNFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps, mom,
                               self.process_group)

    @classmethod
    def convert_sync_batchnorm(cls, module: nn.Module, process_group=None) -> nn.Module:
        out = module
        if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, SyncBatchNorm):
            out = cls(module.num_features, module.eps, module.momentum, module.affine, module.track_running_stats,
                      process_group)
            if module.affine:
                with torch.no_grad():
                    out.weight = module.weight
                    out.bias = module.bias
            out.running_mean = module.running_mean
            out.running_var = module.running_var
            out.num_batches_tracked = module.num_batches_tracked
            out.training = module.training
        for name, child in module.named_children():
            out.add_module(name, cls.convert_sync_batchnorm(child, process_group))
        return out
