"""Training step on stock PyTorch ops ("torch engine").

This is the CPU reference execution path (BASELINE config 1, the numerics oracle of
the tests) and the explicit ``--engine torch`` choice for architectures the native executor does not
cover.  It shares everything else with the native path: the flat parameter/gradient storage, the
gradient bucketer (here driven by autograd post-accumulate hooks), the fused-SGD semantics, the
device-side loss scaler and the cross-rank metric reduction -- so DDP/SyncBN/AMP logic is exercised
on CPU with the ``gloo`` backend exactly as on GPU with RCCL.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..amp.scaler import DeviceGradScaler
from ..models.inception import split_outputs
from ..optim.flat import FlatBuffers, FlatParams
from ..optim.sgd import FusedSGD
from ..parallel.ddp import GradBucketer, broadcast_parameters, sync_buffers
from ..parallel.syncbn import SyncBatchNorm
from ..utils.meters import accuracy


class TorchTrainer:
    def __init__(self, model: nn.Module, device, dtype: torch.dtype = torch.float32, lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 1e-4, use_amp: bool = False, sync_bn: bool = False,
                 bucket_cap_mb: float = 25.0, first_bucket_mb: float = 1.0, broadcast_buffers: bool = True,
                 process_group=None, reduce_metrics: bool = True, channels_last: bool = True,
                 aux_loss_weight: float = 0.3, dp_device_ids=None, comm: str = "torch",
                 comm_timeout_s: float = 0.0, rebuild_buckets: bool = True):
        self.device = torch.device(device)
        self.pg = process_group
        self.distributed = dist.is_initialized() and dist.get_world_size(process_group) > 1
        self.world = dist.get_world_size(process_group) if self.distributed else 1
        if sync_bn and self.distributed:
            model = SyncBatchNorm.convert_sync_batchnorm(model, process_group)
        model = model.to(self.device)
        if channels_last and self.device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        self.dtype = dtype
        self.flat = FlatParams(model, self.device, None)
        # single-process multi-GPU (dataparallel.py on the torch engine): nn.DataParallel scatters the batch,
        # replicates the module per forward and reduce-adds the gradients into the flat views on device 0
        self.net = nn.DataParallel(model, device_ids=list(dp_device_ids)) if dp_device_ids else model
        self.buffers = FlatBuffers(model, self.device)
        broadcast_parameters(self.flat, self.buffers, process_group)
        # autograd decides the gradient order: rebuild the buckets from step 1's observed order, like DDP
        layout = GradBucketer(self.flat, process_group, bucket_cap_mb, first_bucket_mb, enabled=self.distributed,
                              rebuild=rebuild_buckets and dp_device_ids is None)
        # --comm native: gradient buckets, buffer broadcasts and metric all-reduces through this framework's C++
        # communicator + bucketer (host shared-memory transport on the CPU, csrc/comm.cpp) instead of c10d
        self.ncomm = None
        if comm == "native" and self.distributed:
            from ..parallel.comm import NativeBucketer, NativeComm
            self.ncomm = NativeComm(self.device, process_group, timeout_s=comm_timeout_s)
            self.bucketer = NativeBucketer(layout, self.ncomm)
        else:
            self.bucketer = layout
        for s_, p_ in zip(self.flat.slots, self.flat.params):
            p_.register_post_accumulate_grad_hook(lambda _p, i=s_.index: self.bucketer.grad_ready(i))
        self.optimizer = FusedSGD(self.flat, lr, momentum, weight_decay)
        self.scaler = DeviceGradScaler(self.device, enabled=use_amp and dtype == torch.float16)
        self.broadcast_buffers = broadcast_buffers and self.distributed
        self.reduce_metrics = reduce_metrics and self.distributed
        # GoogLeNet / Inception-v3 return auxiliary logits in training; their CE losses are added with this weight
        self.aux_loss_weight = aux_loss_weight
        self._steps = 0
        self._eval_sync_pending = False  # a train step ran since the last eval-forward buffer broadcast
        self.buffer_syncs = 0  # buffer broadcasts issued (tests: one per train step after the first + one per eval epoch)

    def on_state_loaded(self) -> None:
        """Parameters are views of the flat buffer, so ``load_state_dict`` already updated them."""

    def close(self) -> None:
        """Collective teardown of the native communicator (--comm native on CPU ranks); idempotent."""
        if self.ncomm is not None:
            self.ncomm.destroy()
            self.ncomm = None

    def abort(self) -> None:
        """Failure path: abort the native communicator (not collective)."""
        if self.ncomm is not None:
            self.ncomm.abort()
            self.ncomm = None

    def _autocast(self):
        if self.dtype == torch.float32:
            return contextlib.nullcontext()
        return torch.autocast(self.device.type, dtype=self.dtype)

    def _sync_buffers(self) -> None:
        self.buffer_syncs += 1
        if self.ncomm is None:
            sync_buffers(self.buffers, self.pg)
            return
        if self.buffers.n_float:
            self.ncomm.broadcast(self.buffers.fdata, 0)
        if self.buffers.n_int:
            self.ncomm.broadcast(self.buffers.idata, 0)

    def _reduce(self, met):
        if self.reduce_metrics:
            if self.ncomm is not None:
                self.ncomm.all_reduce(met)
            else:
                dist.all_reduce(met, group=self.pg)
            met.div_(self.world)
        return met

    def _inputs(self, images):
        if self.device.type == "cuda":
            images = images.contiguous(memory_format=torch.channels_last)
        return images

    def train_step(self, images, target):
        self.model.train()
        if self.broadcast_buffers and self._steps > 0:
            self._sync_buffers()
        self.optimizer.zero_grad()
        with self._autocast():
            out, aux = split_outputs(self.net(self._inputs(images)))
            loss = F.cross_entropy(out.float(), target)
            for a in aux:
                loss = loss + self.aux_loss_weight * F.cross_entropy(a.float(), target)
        acc = accuracy(out.detach().float(), target, 1)
        met = self._reduce(torch.stack([loss.detach().float(), acc.float()]))
        scale = self.scaler.scale_tensor
        (loss * scale if scale is not None else loss).backward()
        self.bucketer.finish()
        self.scaler.unscale_check(self.flat.grad)
        self.optimizer.step(grad_scale=self.bucketer.grad_scale(), loss_scale=scale, found_inf=self.scaler.found_inf)
        self.scaler.update()
        self._steps += 1
        self._eval_sync_pending = True
        return out.detach().float(), met

    @torch.no_grad()
    def eval_step(self, images, target):
        self.model.eval()
        if self.broadcast_buffers and self._eval_sync_pending:
            # DDP: only the FIRST eval forward after training re-broadcasts the buffers
            self._sync_buffers()
            self._eval_sync_pending = False
        out = self.net(self._inputs(images)).float()  # validation runs without autocast (`:316-317`)
        loss = F.cross_entropy(out, target)
        acc = accuracy(out, target, 1)
        return out, self._reduce(torch.stack([loss.float(), acc.float()]))
