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

import os

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


def native_syncbn_wiring(sync_bn: bool, ncomm, process_group, distributed: bool, dtype: torch.dtype,
                         comm_timeout_s: float = 0.0, comm_transport: str = "auto"):
    """Which communicator and stream every SyncBN statistic all-reduce of the native executor uses.

    Returns ``(ncomm_bn, kwargs)``: ``kwargs`` go to the executor (``syncbn_group`` for c10d, or
    ``syncbn_allreduce`` / ``syncbn_allreduce_fwd`` / ``syncbn_world`` for the native communicator), ``ncomm_bn`` is
    the statistics' own communicator (or None).

    With the native communicator (``--comm native``) the default, ``PDT_SYNCBN_COMM=own``, gives the statistics a
    communicator of their OWN, all-reduced inline on the compute stream, forward and backward.  They are tiny,
    latency-bound and on the critical path (dgrad -> BN sums -> all-reduce -> finalize -> apply -> next dgrad), so
    they must never queue behind a 25 MiB gradient bucket on the bucket communicator's stream.  RCCL orders
    collectives per communicator, and both sequences are issued in the same host order on every rank (the executor's
    schedule is fixed), so the two communicators stay consistent; tests/test_distributed_cpu.py records both
    sequences per rank at world 2 / 4 over the host transport.  ``PDT_SYNCBN_COMM=shared`` keeps ONE communicator
    (forward statistics inline, backward on the comm stream behind any bucket in flight) -- the round-5 default."""
    kw = dict(syncbn_group=(process_group or dist.group.WORLD) if (sync_bn and distributed and ncomm is None)
              else None)
    if not sync_bn or ncomm is None:
        return None, kw
    mode = os.environ.get("PDT_SYNCBN_COMM", "own")
    if mode not in ("own", "shared"):
        raise ValueError(f"PDT_SYNCBN_COMM must be 'own' or 'shared', got {mode!r}")
    if mode == "own":
        from .comm import NativeComm
        bn = NativeComm(ncomm.device, process_group, timeout_s=comm_timeout_s, transport=comm_transport)
        kw.update(syncbn_allreduce=bn.all_reduce_inline, syncbn_world=bn.world)
        return bn, kw
    kw.update(syncbn_allreduce=ncomm.all_reduce, syncbn_world=ncomm.world)
    if dtype != torch.float32:
        # forward statistics straight onto the compute stream (no bucket is in flight during the forward)
        kw["syncbn_allreduce_fwd"] = ncomm.all_reduce_inline
    return None, kw
