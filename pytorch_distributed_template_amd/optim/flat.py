"""Flat parameter / gradient / optimizer-state storage.

All trainable parameters of a model live in ONE contiguous fp32 buffer, their gradients in a second
buffer of the same layout (so every ``param.grad`` is a view: the DDP gradient buckets are plain
slices of it and need no copy-in/copy-out), the SGD momentum in a third, and the 16-bit
compute copy (bf16/fp16 "shadow", written by the fused SGD kernel) in a fourth.

Conv weights are stored physically as [Cout][kh][kw][Cin] (PyTorch ``channels_last`` strides on the
logical [Cout, Cin, kh, kw] parameter), which is exactly the layout the NHWC implicit-GEMM kernels
consume, so forward weights need no per-step re-layout.  Parameter names, shapes and state-dict keys
are untouched.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn


@dataclass
class ParamSlot:
    index: int
    name: str
    offset: int
    numel: int
    shape: tuple
    channels_last: bool


def _phys_view(flat: torch.Tensor, offset: int, shape: tuple, channels_last: bool) -> torch.Tensor:
    n = 1
    for s in shape:
        n *= s
    v = flat[offset:offset + n]
    if channels_last:
        co, ci, kh, kw = shape
        return v.view(co, kh, kw, ci).permute(0, 3, 1, 2)
    return v.view(shape)


class FlatParams:
    """Flattened trainable parameters of ``model`` (in ``model.named_parameters()`` order)."""

    def __init__(self, model: nn.Module, device: torch.device, shadow_dtype: Optional[torch.dtype] = None,
                 align: int = 64, guards: bool = True):
        """``guards=False``: no validation canaries in the gradient gaps (DataParallel replicas, whose whole gradient
        buffers are reduce-added into GPU 0's: the canaries would be summed into its guard bands)."""
        self.device = torch.device(device)
        self.slots: List[ParamSlot] = []
        self.params: List[nn.Parameter] = []
        self.by_param: Dict[int, ParamSlot] = {}
        # PDT_VALIDATE guard bands (ops/validate.py): extra canary elements after every slot of the gradient buffer
        from ..ops import validate
        # (single process only: a multi-rank run all-reduces whole bucket ranges, canaries included -- so the slot
        # padding is only reserved when the canaries will be installed, and a multi-rank buffer can be re-laid)
        guarded = guards and int(os.environ.get("WORLD_SIZE", "1")) == 1
        guard = (int(os.environ.get("PDT_VALIDATE_GUARD", "0") or 0)
                 if guarded and validate.level_from_env() > 0 else 0)
        self.guard = guard
        self.align = align
        off = 0
        for name, p in model.named_parameters():
            if not p.requires_grad:
                continue
            cl = p.dim() == 4
            s = ParamSlot(len(self.slots), name, off, p.numel(), tuple(p.shape), cl)
            self.slots.append(s)
            self.params.append(p)
            self.by_param[id(p)] = s
            off += (p.numel() + guard + align - 1) // align * align
        self.total = off
        self.data = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.momentum = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.shadow = (torch.zeros(self.total, dtype=shadow_dtype, device=self.device)
                       if shadow_dtype is not None else None)
        with torch.no_grad():
            for s, p in zip(self.slots, self.params):
                _phys_view(self.data, s.offset, s.shape, s.channels_last).copy_(p.data)
                p.data = _phys_view(self.data, s.offset, s.shape, s.channels_last)
                p.grad = _phys_view(self.grad, s.offset, s.shape, s.channels_last)
        # parameters that receive weight decay: all of them, like the reference (SURVEY §2.2 --wd)
        self.refresh_shadow()
        if guard and self.device.type == "cuda":
            self._install_guards(validate)

    def _install_guards(self, validate) -> None:
        """Canary-fill every gap between slots in ``grad`` and register it with the validator."""
        idx, owners = [], []
        n = 0
        for i, s in enumerate(self.slots):
            end = self.slots[i + 1].offset if i + 1 < len(self.slots) else self.total
            if end > s.offset + s.numel:
                owners.append((n, s.name))
                idx.append(torch.arange(s.offset + s.numel, end, dtype=torch.int64))
                n += end - s.offset - s.numel
        if not idx:
            return
        gi = torch.cat(idx).to(self.device)
        self.grad.view(torch.int32)[gi] = validate.CANARY_BITS
        v = validate.validator()
        if v is not None:
            v.register_guard(self.grad, gi, owners)

    # -- views -----------------------------------------------------------------------------------
    def slot(self, p: torch.Tensor) -> ParamSlot:
        return self.by_param[id(p)]

    def data_flat(self, p: torch.Tensor) -> torch.Tensor:
        s = self.slot(p)
        return self.data[s.offset:s.offset + s.numel]

    def grad_flat(self, p: torch.Tensor) -> torch.Tensor:
        s = self.slot(p)
        return self.grad[s.offset:s.offset + s.numel]

    def shadow_flat(self, p: torch.Tensor) -> torch.Tensor:
        s = self.slot(p)
        return self.shadow[s.offset:s.offset + s.numel]

    def refresh_shadow(self) -> None:
        """Re-derive the 16-bit shadow from the fp32 master (after load_state_dict / broadcast)."""
        if self.shadow is None:
            return
        if self.shadow.is_cuda:
            from ..ops import native
            native.C.cast16(self.data, self.shadow)
        else:
            self.shadow.copy_(self.data)

    def master_read_index(self) -> torch.Tensor:
        """int32 flat offsets of every element of the 1-D parameters (BatchNorm gamma/beta, biases): the values the
        16-bit executor reads from the fp32 MASTER rather than from the shadow.  A DataParallel replica needs the
        shadow plus exactly these (``parallel/dp.py``)."""
        idx = [torch.arange(s.offset, s.offset + s.numel, dtype=torch.int64) for s in self.slots if len(s.shape) < 2]
        out = torch.cat(idx) if idx else torch.zeros(0, dtype=torch.int64)
        assert out.numel() == 0 or int(out.max()) < self.total
        return out.to(torch.int32)

    def zero_grad(self) -> None:
        self.grad.zero_()

    def reorder(self, mem_order: List[int]) -> None:
        """Re-lay the flat buffers so slot ``mem_order[0]`` comes first, ``mem_order[1]`` next, ... (the DDP bucket
        rebuild, parallel/ddp.py: a bucket must be a contiguous slice).  Contents of data / grad / momentum /
        shadow move with their slots IN PLACE -- the buffer tensors stay the same objects, so everything holding
        them (optimizer, C++ bucketer, scaler) stays valid; parameter and gradient views are re-pointed.  Slot
        indices (the bucketer's parameter ids) do not change."""
        assert sorted(mem_order) == list(range(len(self.slots))), "reorder needs a permutation of the slots"
        assert self.guard == 0, "flat reorder with PDT_VALIDATE guard bands"
        new_off, off = {}, 0
        for i in mem_order:
            new_off[i] = off
            off += (self.slots[i].numel + self.align - 1) // self.align * self.align
        assert off == self.total
        with torch.no_grad():
            for buf in (self.data, self.grad, self.momentum, self.shadow):
                if buf is None:
                    continue
                src = buf.clone()
                buf.zero_()
                for s in self.slots:
                    buf[new_off[s.index]:new_off[s.index] + s.numel].copy_(src[s.offset:s.offset + s.numel])
            for s, p in zip(self.slots, self.params):
                s.offset = new_off[s.index]
                p.data = _phys_view(self.data, s.offset, s.shape, s.channels_last)
                p.grad = _phys_view(self.grad, s.offset, s.shape, s.channels_last)

    def canonical(self, buf: torch.Tensor) -> torch.Tensor:
        """``buf`` (data / grad / momentum layout) with the slots concatenated in parameter-registration order and
        without alignment gaps: comparable across processes whatever their flat layout (bucket rebuild)."""
        return torch.cat([buf[s.offset:s.offset + s.numel] for s in self.slots])

    def reattach_grads(self) -> None:
        """Point every ``param.grad`` back at its flat view (after code that set grads to None)."""
        for s, p in zip(self.slots, self.params):
            p.grad = _phys_view(self.grad, s.offset, s.shape, s.channels_last)


class FlatBuffers:
    """BatchNorm running statistics in one fp32 buffer + one int64 buffer (one coalesced broadcast
    per dtype for DDP's per-forward buffer sync)."""

    def __init__(self, model: nn.Module, device: torch.device):
        self.device = torch.device(device)
        f_entries, i_entries = [], []
        for mname, m in model.named_modules():
            for bname, b in list(m._buffers.items()):
                if b is None:
                    continue
                (f_entries if b.is_floating_point() else i_entries).append((m, bname, b))
        nf = sum(b.numel() for _, _, b in f_entries)
        ni = sum(b.numel() for _, _, b in i_entries)
        self.fdata = torch.zeros(max(nf, 1), dtype=torch.float32, device=self.device)
        self.idata = torch.zeros(max(ni, 1), dtype=torch.int64, device=self.device)
        off = 0
        for m, bname, b in f_entries:
            v = self.fdata[off:off + b.numel()].view(b.shape)
            v.copy_(b.detach())
            m._buffers[bname] = v
            off += b.numel()
        off = 0
        for m, bname, b in i_entries:
            v = self.idata[off:off + b.numel()].view(b.shape)
            v.copy_(b.detach())
            m._buffers[bname] = v
            off += b.numel()
        self.n_float, self.n_int = nf, ni
