"""Native VGG / AlexNet executor (vgg11/13/16/19, their ``_bn`` forms, alexnet) over the gfx950 kernels.

The reference trains any torchvision constructor by name (`distributed.py:39-40,132-137`); this is the native engine's
second model family after the ResNets.  It reuses the ResNet executor's machinery -- the implicit-GEMM conv kernels
(forward with the BatchNorm-statistics epilogue, backward-data with the producer's fused ReLU-mask / BN-backward
reduce, split-K weight gradients on the side stream), the BN finalize / apply kernels, the fused loss, the flat fp32
master + 16-bit shadow, per-parameter ``grad_ready`` for the DDP bucketer and SyncBN -- and adds VGG's own pieces
(``csrc/kernels/vgg.hip``):

* conv bias + ReLU runs as a BatchNorm with coefficients ``[1 | bias | 0 | 1]`` (``bias_coef``), so bias layers use
  the same fused kernels as ``_bn`` layers: bn_apply + ReLU forward, the ReLU mask recomputed inside the consumer's
  backward-data epilogue, whose fused reduce then yields ``sum dz`` = the bias gradient;
* BN / bias + ReLU + MaxPool(2, 2) is ONE pass (``bn_relu_maxpool2``): the full-resolution post-ReLU tensor of the
  last conv of every stage is never written; its backward (``maxpool2_bwd``) writes the conv-output gradient
  (``A*dz + B*y + C`` for a BatchNorm, ``dz`` for a bias) with the ReLU mask taken from the pooled output, and the
  BN-backward sums come from the pooled tensors alone (``pooled_bwd_reduce``);
* the first conv (3 -> 64) runs in the stem's window mode over the zero-padded NHWC4 image: one 32-wide K-step per
  kernel row (8 pixels x 4 channels), no im2col buffer; its weight gradient uses kernel-row pairs (``dil`` 2);
* the classifier's GEMMs (25088 -> 4096 -> 4096 -> classes) are plain library GEMMs on hipBLASLt (``torch.mm`` in
  16-bit, fp32 accumulation); their weight gradients are the native split-K weight-gradient kernel (fp32 straight
  into the flat gradient buffer), bias + ReLU + Dropout is one pass (``fc_act_fwd``: counter-hash dropout), and its
  backward recovers the keep mask from the stored output (``fc_act_bwd``), so no mask tensor exists.

AlexNet (the reference's ``--arch alexnet``) runs on the same executor: its 11x11/4 first conv in the same window mode
(two 8-pixel windows per kernel row, ``tstep_w`` = 8; weight gradient on 6 kernel-row pairs), the 5x5 and 3x3 convs
on the generic implicit-GEMM kernels, bias + ReLU + MaxPool(3, 2) as one pass (``bn_relu_maxpool`` with pad 0, the
ResNet stem's kernel) with the gather-form backward (``maxpool_bwd_relu``), and its classifier order (Dropout before
each of the first two Linears: the feature dropout is ``fc_act_fwd`` with a zero bias -- the features are post-ReLU,
so its ReLU is the identity).

Every launch whose operands would pass the kernels' 32-bit offsets (``_MAX_ELEMS``: VGG's 224 x 224 x 64 activations
at a few hundred images per GPU) runs over image chunks: weight gradients accumulate across chunks, BN statistics are
summed from per-chunk slot buffers.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..ops import native
from .classic import VGG, AlexNet
from .executor import ResNetExecutor, _BN, _Conv

# largest element count of any operand of one conv / weight-gradient launch (the LDS-DMA buffer resources and the
# weight-gradient checks index with 32-bit offsets)
_MAX_ELEMS = (1 << 30) - 1


class _Layer:
    """One conv of ``features`` with its BatchNorm (``bn``) or bias (``bias_slot``), its ReLU and the max-pool that
    may follow it (``pool``: 0 none, 2 = MaxPool(2, 2), 3 = MaxPool(3, 2))."""

    def __init__(self, conv: nn.Conv2d, bn: Optional[nn.BatchNorm2d], pool: int, flat, derived_maps, off, device):
        if not _conv_ok(conv):
            raise NotImplementedError(f"native VGG/AlexNet executor: unsupported conv {conv}")
        self.first = conv.in_channels == 3
        self.conv = _Conv(conv, flat, [] if self.first else derived_maps, off if not self.first else [0])
        self.bn = _BN(bn, flat, device) if bn is not None else None
        self.bias_slot = flat.slot(conv.bias) if conv.bias is not None else None
        if self.bn is None and self.bias_slot is None:
            raise NotImplementedError("native VGG executor: conv without BatchNorm needs a bias")
        self.pool = pool
        C = conv.out_channels
        self.coef = self.bn.coef if self.bn is not None else torch.zeros(4 * C, dtype=torch.float32, device=device)
        self.bcoef = self.bn.bcoef if self.bn is not None else torch.zeros(3 * C, dtype=torch.float32, device=device)


def _conv_ok(conv: nn.Conv2d) -> bool:
    """The first (3-channel) conv: any square kernel up to 11 x 11 at stride <= 4 (window mode); the others: square
    stride-1 'same' convs (VGG's 3x3, AlexNet's 5x5 and 3x3) over channel counts the implicit-GEMM kernels tile."""
    k, st, pad = conv.kernel_size, conv.stride, conv.padding
    if k[0] != k[1] or st[0] != st[1] or pad[0] != pad[1] or conv.dilation != (1, 1) or conv.groups != 1:
        return False
    if conv.in_channels == 3:
        return k[0] <= 11 and st[0] <= 4
    return st[0] == 1 and 2 * pad[0] == k[0] - 1 and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0


def _pool_kind(m: nn.MaxPool2d) -> int:
    ks = m.kernel_size if isinstance(m.kernel_size, int) else m.kernel_size[0]
    st = m.stride if isinstance(m.stride, int) else m.stride[0]
    pad = m.padding if isinstance(m.padding, int) else m.padding[0]
    if ks == 2 and st == 2 and pad == 0 and not m.ceil_mode:
        return 2
    if ks == 3 and st == 2 and pad == 0 and not m.ceil_mode:
        return 3
    return 0


def vgg_supported(model) -> bool:
    """torchvision-layout VGG (3x3 convs (+ BN) + ReLU, 2x2 max-pools) or AlexNet (11x11/4, 5x5 and 3x3 convs + ReLU,
    3x3/2 max-pools), at 224-style inputs."""
    if not isinstance(model, (VGG, AlexNet)):
        return False
    for m in model.features:
        if isinstance(m, nn.Conv2d) and not _conv_ok(m):
            return False
        if isinstance(m, nn.MaxPool2d) and _pool_kind(m) != (3 if isinstance(model, AlexNet) else 2):
            return False
    return True


class VGGExecutor(ResNetExecutor):
    """Runs a torchvision-layout :class:`VGG` or :class:`AlexNet` on one GPU (same public interface as
    :class:`ResNetExecutor`)."""

    def __init__(self, model: nn.Module, flat, device: torch.device, dtype: torch.dtype,
                 grad_ready: Optional[Callable[[int], None]] = None, syncbn_group=None, wgrad_blocks: int = 2048,
                 wgrad_blocks_1x1: int = 512, autotune: bool = False,
                 syncbn_allreduce: Optional[Callable[[torch.Tensor], None]] = None, syncbn_world: int = 0,
                 syncbn_allreduce_fwd: Optional[Callable[[torch.Tensor], None]] = None):
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("native executor computes in bf16 or fp16")
        if not vgg_supported(model):
            raise NotImplementedError("native VGG executor: torchvision-layout VGG (3x3 convs, 2x2 max-pools) or "
                                      "AlexNet only")
        self.C = native.C
        self.n_slots = self.C.stat_slots()
        self.model = model
        self.flat = flat
        self.device = torch.device(device)
        self.dtype = dtype
        self._user_grad_ready = grad_ready or (lambda pid: None)
        self.side = None
        if self.device.type == "cuda" and os.environ.get("PDT_WGRAD_STREAM", "1") != "0":
            self.side = torch.cuda.Stream(device=self.device)
        self._on_side = False
        self._pending_reads: Dict[int, "torch.cuda.Event"] = {}
        self.syncbn_group = syncbn_group
        self.syncbn = syncbn_allreduce is not None or syncbn_group is not None
        if syncbn_allreduce is not None:
            self.syncbn_world = int(syncbn_world) if syncbn_world else 1
            self._sync_sum = syncbn_allreduce
        self._sync_sum_fwd = syncbn_allreduce_fwd
        if syncbn_group is not None and syncbn_allreduce is None:
            import torch.distributed as dist
            self.syncbn_world = dist.get_world_size(syncbn_group)
            self._sync_sum = lambda t: dist.all_reduce(t, group=syncbn_group)
        self.wgrad_blocks, self.wgrad_blocks_1x1 = wgrad_blocks, wgrad_blocks_1x1
        # the ResNet-specific paths of the inherited conv helpers stay off (layer1 halo kernels need W = 56 and the
        # persistent 1x1 kernels 1x1 convs; the inherited predicates decline them by shape, these by construction)
        self.wgrad_l1 = True
        self.bk32_short = True
        self._c1x1 = False
        self._c1x1x = False
        self.fuse_pre = False
        self.split_derived = False
        self.autotune = autotune or os.environ.get("PDT_AUTOTUNE", "0") == "1"
        self._tiles: Dict[tuple, Tuple[int, int]] = {}
        self.max_elems = _MAX_ELEMS
        from ..data.transforms import IMAGENET_MEAN, IMAGENET_STD
        std = torch.tensor(IMAGENET_STD)
        self.norm_scale = (1.0 / (255.0 * std)).to(self.device)
        self.norm_shift = (-torch.tensor(IMAGENET_MEAN) / std).to(self.device)
        # --- features: [conv, (bn), relu, (maxpool)] groups
        derived_maps: List[torch.Tensor] = []
        off = [0]
        # derived layouts: every conv's backward-data phase weights, then the first conv's window weights and the
        # padded last Linear
        mods = list(model.features)
        self.layers: List[_Layer] = []
        i = 0
        while i < len(mods):
            conv = mods[i]
            assert isinstance(conv, nn.Conv2d), f"unexpected feature module {conv}"
            i += 1
            bn = None
            if i < len(mods) and isinstance(mods[i], nn.BatchNorm2d):
                bn = mods[i]
                i += 1
            assert i < len(mods) and isinstance(mods[i], nn.ReLU), "conv (+ BN) must be followed by ReLU"
            i += 1
            pool = 0
            if i < len(mods) and isinstance(mods[i], nn.MaxPool2d):
                pool = _pool_kind(mods[i])
                i += 1
            self.layers.append(_Layer(conv, bn, pool, flat, derived_maps, off, self.device))
        # the first conv's window weights [cout][R][U][32]: window u of kernel row r holds columns u*8 .. u*8+7,
        # element j = column (j // 4) * 4 + channel (j % 4) of the NHWC4 image (U = 1 for VGG's 3x3, 2 for the 11x11)
        first = self.layers[0]
        assert first.first and all(not l.first for l in self.layers[1:]), "3-channel input conv first"
        fc = first.conv
        R0 = fc.R
        self.w0_U = U0 = (R0 + 7) // 8
        self.w0_T = T0 = (R0 + 1) // 2  # weight-gradient kernel-row pairs
        k = torch.arange(fc.cout).view(-1, 1, 1, 1)
        r = torch.arange(R0).view(1, -1, 1, 1)
        u = torch.arange(U0).view(1, 1, -1, 1)
        j = torch.arange(32).view(1, 1, 1, -1)
        s_, c_ = u * 8 + j // 4, j % 4
        src = fc.slot.offset + ((k * R0 + r) * R0 + s_.clamp(max=R0 - 1)) * 3 + c_.clamp(max=2)
        win = torch.where((s_ < R0) & (c_ < 3), src, torch.full_like(src, -1))
        self.w0_off = off[0]
        derived_maps.append(win.reshape(-1).to(torch.int32))
        off[0] += win.numel()
        # its weight gradient: [cout][T pairs][U windows][2 rows][32] window tile -> KRSC [cout][R][R][3]
        self.w0_ldw = T0 * U0 * 64
        kk = torch.arange(fc.cout).view(-1, 1, 1, 1)
        rr = torch.arange(R0).view(1, -1, 1, 1)
        ss = torch.arange(R0).view(1, 1, -1, 1)
        cc = torch.arange(3).view(1, 1, 1, -1)
        self.w0_gidx = (kk * self.w0_ldw + ((rr // 2) * U0 + ss // 8) * 64 + (rr % 2) * 32 + (ss % 8) * 4 +
                        cc).reshape(-1).to(torch.int32).to(self.device)
        # --- classifier: VGG [Linear, ReLU, Dropout] x 2 + Linear; AlexNet [Dropout, Linear, ReLU] x 2 + Linear
        lin = [m for m in model.classifier if isinstance(m, nn.Linear)]
        drops = [m for m in model.classifier if isinstance(m, nn.Dropout)]
        if len(lin) != 3 or len(drops) != 2:
            raise NotImplementedError("native VGG executor: torchvision's 3-Linear classifier")
        self.p_drop = float(drops[0].p)
        # dropout in front of the first two Linears (AlexNet) instead of behind their ReLUs (VGG)
        self.drop_first = isinstance(model.classifier[0], nn.Dropout)
        self.pool_hw = model.avgpool.output_size if isinstance(model.avgpool.output_size, tuple) else (
            model.avgpool.output_size, model.avgpool.output_size)
        self.lin = lin
        self.lin_slots = [(flat.slot(m.weight), flat.slot(m.bias)) for m in lin]
        self.feat = lin[0].in_features
        self.hidden = lin[0].out_features
        self.ncls = lin[2].out_features
        self.ncls_pad = (self.ncls + 127) // 128 * 128
        last_c = self.layers[-1].conv.cout
        if self.feat % last_c or self.hidden % 64:
            raise NotImplementedError("native VGG executor: classifier widths")
        self.fc_slot, self.fcb_slot = self.lin_slots[2]
        o = torch.arange(self.ncls_pad).view(-1, 1)
        f = torch.arange(self.hidden).view(1, -1)
        m = torch.where(o < self.ncls, self.fc_slot.offset + o * self.hidden + f, torch.full_like(o * f, -1))
        self.fc_w_off = off[0]
        derived_maps.append(m.reshape(-1).to(torch.int32))
        off[0] += m.numel()
        self.derived_idx = torch.cat([mm.to(torch.int32) for mm in derived_maps]).to(self.device)
        self.derived = torch.zeros(off[0], dtype=dtype, device=self.device)
        self._ones = {}
        self._bufs: Dict[Tuple, torch.Tensor] = {}
        self._plans: Dict[Tuple, Tuple[int, int]] = {}
        from ..ops import validate
        self._buf_guard = (int(os.environ.get("PDT_VALIDATE_GUARD", "0") or 0)
                           if validate.level_from_env() > 0 and self.device.type == "cuda" else 0)
        self._drop_seed = int(torch.initial_seed()) & 0xFFFFFFFF
        self._drop_step = 0
        self.update_derived()

    # ---------------------------------------------------------------------------------- helpers
    def update_derived(self) -> None:
        """Every derived 16-bit layout (first-conv window weights, the padded last Linear, each conv's backward-data
        phase weights) from the shadow, in one gather on the compute stream."""
        self.C.gather16(self.flat.shadow, self.derived_idx, self.derived)

    def _ones_like(self, C: int) -> torch.Tensor:
        t = self._ones.get(C)
        if t is None:
            t = self._ones[C] = torch.ones(C, dtype=torch.float32, device=self.device)
        return t

    def _zeros(self, C: int) -> torch.Tensor:
        t = self._ones.get(-C)
        if t is None:
            t = self._ones[-C] = torch.zeros(C, dtype=torch.float32, device=self.device)
        return t

    def _chunks(self, N: int, per_image: int) -> List[Tuple[int, int]]:
        nb = max(1, min(N, self.max_elems // max(1, per_image)))
        return [(i, min(N, i + nb)) for i in range(0, N, nb)]

    def _coef(self, L: _Layer, train: bool, sp, count: int) -> None:
        """The layer's (scale, shift, mean, invstd) coefficients: BatchNorm training finalize / eval, or the bias."""
        if L.bn is None:
            self.C.bias_coef(self._p(L.bias_slot), L.coef, L.conv.cout)
            return
        # torchvision's VGG-BN convs keep their bias: it only shifts the batch mean the BatchNorm removes, so the
        # kernels run without it and only the running mean (train) / the eval shift account for it
        if train:
            self.bn_train_finalize(L.bn, sp, 0, count)
            if L.bias_slot is not None:
                L.bn.mod.running_mean.add_(self._p(L.bias_slot), alpha=L.bn.momentum)
        else:
            self.bn_eval(L.bn)
            if L.bias_slot is not None:
                C = L.conv.cout
                L.coef[C:2 * C].addcmul_(self._p(L.bias_slot), L.coef[:C])

    def _finish(self, L: _Layer, slots, count: int) -> None:
        """Backward finalize from the layer's (sum dz, sum dz * xhat) slots: BatchNorm -> dgamma / dbeta / bcoef;
        bias -> dbias = sum dz (the BatchNorm finalize with gamma = 1: its dbeta)."""
        if L.bn is not None:
            self._bn_bwd_finish(slots, count, L.bn)
            if L.bias_slot is not None:  # a bias in front of a BatchNorm has an identically zero gradient
                self._g(L.bias_slot).zero_()
                self.grad_ready(L.bias_slot.index)
            return
        C = L.conv.cout
        self.C.bn_bwd_finalize_slots(slots, 2, float(count), L.coef, self._ones_like(C), None, self._g(L.bias_slot),
                                     L.bcoef, None, None, None, None, None, 1.0)
        self.grad_ready(L.bias_slot.index)

    # ---------------------------------------------------------------------------------- conv (chunked)
    def _conv_fwd(self, L: _Layer, x, N, H, W, y, stats: bool):
        c = L.conv
        per = H * W * max(c.cin, c.cout)
        chunks = self._chunks(N, per)
        if len(chunks) == 1:
            _, _, sp, _ = self.conv_fwd(c, x, N, H, W, y, stats)
            return sp
        sp_all = self._buf(("stats", c.cout), self.n_slots * c.cout * 2, torch.float64) if stats else None
        for k, (a, b) in enumerate(chunks):
            xs = x[a * H * W * c.cin:b * H * W * c.cin]
            ys = y[a * H * W * c.cout:b * H * W * c.cout]
            _, _, sp, _ = self.conv_fwd(c, xs, b - a, H, W, ys, stats, stats_tag="chunk")
            if stats:
                if k == 0:
                    sp_all.copy_(sp)
                else:
                    sp_all.add_(sp)
        return sp_all

    def _wgrad_chunked(self, c: _Conv, x, dy, N, H, W, gout):
        """Stride-1 'same' conv weight gradient over image chunks, accumulated into ``gout`` (fp32 KRSC)."""
        chunks = self._chunks(N, H * W * max(c.cin, c.cout))
        R, S, pad = c.R, c.S, c.pad
        ldw = R * S * c.cin
        for k, (a, b) in enumerate(chunks):
            xs = x[a * H * W * c.cin:b * H * W * c.cin]
            dys = dy[a * H * W * c.cout:b * H * W * c.cout]
            n = b - a
            if len(chunks) == 1:
                self._wgrad(c.cout, xs, dys, n, H, W, c.cin, R, S, H, W, 1, pad, gout, ldw)
                return
            key = (c.cout, R, S, c.cin, n * H * W, False)
            plan = self._plans.get(key)
            if plan is None:
                plan = tuple(self.C.conv_wgrad_plan(c.cout, R, S, c.cin, n * H * W, self.wgrad_blocks, False))[:2]
                self._plans[key] = plan
            splits, pps = plan
            ws = self._buf("ws", splits * c.cout * ldw, torch.float32)
            self.C.conv_wgrad(xs, dys, ws, n, H, W, c.cin, c.cout, R, S, H, W, 1, 1, pad, pad, 1, 1, ldw, splits, pps,
                              0, False)
            self.C.wgrad_reduce(ws, splits, c.cout, ldw, ldw, c.cout * ldw, gout, ldw, 1.0, k > 0)

    def _conv_bwd(self, L: _Layer, x, N, H, W, dy, dx, bnb_layer: Optional[_Layer], slots):
        """Weight gradient (side stream) + backward data into ``dx``; ``bnb_layer``: the producer layer whose ReLU mask
        (recomputed from its conv output and coefficients) and BN-backward sums are fused into the epilogue."""
        c = L.conv

        def wg():
            self._wgrad_chunked(c, x, dy, N, H, W, self._g(c.slot))
            self.grad_ready(c.pid)
        self._side_wgrad((dy, x), wg)
        chunks = self._chunks(N, H * W * max(c.cin, c.cout))
        if len(chunks) == 1:
            bnb = None if bnb_layer is None else (1, bnb_layer.y, bnb_layer.coef, None, None, None, slots)
            # (the inherited conv_bwd would also run the weight gradient: call its backward-data part only)
            self._dgrad(c, dy, N, H, W, dx, bnb)
            return
        for k, (a, b) in enumerate(chunks):
            dys = dy[a * H * W * c.cout:b * H * W * c.cout]
            dxs = dx[a * H * W * c.cin:b * H * W * c.cin]
            bnb = None
            if bnb_layer is not None:
                ys = bnb_layer.y[a * H * W * c.cin:b * H * W * c.cin]
                sk = slots if k == 0 else self._buf(("bnslots_chunk", c.cin), slots.numel(), torch.float64)
                bnb = (1, ys, bnb_layer.coef, None, None, None, sk)
            self._dgrad(c, dys, b - a, H, W, dxs, bnb)
            if bnb is not None and k > 0:
                slots.add_(bnb[6])

    def _dgrad(self, c: _Conv, dy, N, H, W, dx, bnb):
        phases = [[ph, pw, T, U, ioff_h, ioff_w, doff] for (ph, pw, T, U, ioff_h, ioff_w, doff, dn) in c.phases]
        bk = 64 if c.cout % 64 == 0 else 32

        def launch(bm, bn):
            if bnb is None:
                self.C.conv_dgrad(dy, self.derived, dx, None, N, H, W, c.cout, c.cin, H, W, 1, phases, bm, bn, bk)
            else:
                self.C.conv_dgrad_bn(dy, self.derived, dx, None, N, H, W, c.cout, c.cin, H, W, 1, phases, bm, bn, bk,
                                     *bnb, -1)
        key = ("dgrad", N, H, W, c.cin, c.cout, c.R, c.S, 1, False, bnb[0] if bnb else 0, -1)
        bm, bn = self._tile(key, c.cin, bk, launch, fused_epilogue=bnb is not None, kdim=c.cout * c.R * c.S,
                            m=N * H * W)
        launch(bm, bn)

    # ---------------------------------------------------------------------------------- forward
    def _forward(self, images: torch.Tensor, train: bool):
        Cn = self.C
        N = images.shape[0]
        assert images.dim() == 4 and images.shape[1] == 3, "expected NCHW images"
        H, W = images.shape[2], images.shape[3]
        if self.drop_first:
            if H < 63 or W < 63:
                raise NotImplementedError("native AlexNet executor: inputs of at least 63 x 63")
        elif H % 32 or W % 32:
            raise NotImplementedError("native VGG executor: input sides must be multiples of 32")
        u8 = images.dtype == torch.uint8
        x32 = images.contiguous() if u8 or images.dtype == torch.float32 else images.float().contiguous()
        # first conv: zero-padded NHWC4 image, window-mode implicit GEMM, U 32-wide K-steps (8 pixels x 4 channels) per
        # kernel row; spare rows / columns so every window and the weight gradient's row pairs stay inside the image
        c0 = self.layers[0].conv
        R0, st0, pad0 = c0.R, c0.st, c0.pad
        P0, Q0 = (H + 2 * pad0 - R0) // st0 + 1, (W + 2 * pad0 - R0) // st0 + 1
        Hp = max(H + 2 * pad0, (P0 - 1) * st0 + 2 * self.w0_T)
        Wp = max(W + 2 * pad0, (Q0 - 1) * st0 + 8 * self.w0_U)
        xp = self._buf("stem_in", N * Hp * Wp * 4)
        if u8:
            Cn.stem_pack_u8(x32, xp, N, 3, H, W, pad0, Hp, Wp, self.norm_scale, self.norm_shift)
        else:
            Cn.stem_pack(x32, xp, N, 3, H, W, pad0, Hp, Wp)
        saved = {"N": N, "H": H, "W": W, "xp": xp, "Hp": Hp, "Wp": Wp, "P0": P0, "Q0": Q0, "acts": []}
        x, h, w = None, H, W
        for li, L in enumerate(self.layers):
            c = L.conv
            ho_, wo_ = (P0, Q0) if L.first else (h, w)
            y = self._buf(("y", li), N * ho_ * wo_ * c.cout)
            stats = train and L.bn is not None
            if L.first:
                sp = self._buf(("stats", c.cout), self.n_slots * c.cout * 2, torch.float64) if stats else None
                w0 = self.derived[self.w0_off:self.w0_off + c.cout * R0 * self.w0_U * 32]
                for a, b in self._chunks(N, max(Hp * Wp * 4, P0 * Q0 * c.cout)):
                    sk = sp
                    if sp is not None and a > 0:
                        sk = self._buf(("stats_chunk", c.cout), sp.numel(), torch.float64)
                    Cn.conv_fwd(xp[a * Hp * Wp * 4:b * Hp * Wp * 4], w0, y[a * P0 * Q0 * c.cout:b * P0 * Q0 * c.cout],
                                None, sk, b - a, Hp, Wp, 32, c.cout, R0, self.w0_U, P0, Q0, st0, st0, 0, 0, 1, 8, P0,
                                Q0, 1, 1, 0, 0, 256, 64, 32, 4)
                    if sk is not sp:
                        sp.add_(sk)
                h, w = P0, Q0
            else:
                sp = self._conv_fwd(L, x, N, h, w, y, stats)
            self._coef(L, train, sp, N * h * w)
            L.y = y
            if L.pool == 2:
                ho, wo = h // 2, w // 2
                out = self._buf(("act", li), N * ho * wo * c.cout)
                idx = self._buf(("pidx", li), N * ho * wo * c.cout, torch.uint8) if train else None
                Cn.bn_relu_maxpool2(y, L.coef, out, idx, N, h, w, c.cout)
                saved["acts"].append((x, h, w, y, out, idx))
                x, h, w = out, ho, wo
            elif L.pool == 3:  # AlexNet: bias + ReLU + MaxPool(3, 2) (the argmax is kept for eval too: one path)
                ho, wo = (h - 3) // 2 + 1, (w - 3) // 2 + 1
                out = self._buf(("act", li), N * ho * wo * c.cout)
                idx = self._buf(("pidx", li), N * ho * wo * c.cout, torch.uint8)
                Cn.bn_relu_maxpool(y, L.coef, out, idx, N, h, w, c.cout, pad=0)
                saved["acts"].append((x, h, w, y, out, idx))
                x, h, w = out, ho, wo
            else:
                a_ = self._buf(("act", li), N * h * w * c.cout)
                Cn.bn_apply(y, L.coef, None, None, a_, c.cout, 0, True, None)
                saved["acts"].append((x, h, w, y, a_, None))
                x = a_
        # classifier input: torchvision flattens NCHW (the adaptive average pool is the identity at its own output size:
        # 7 x 7 for VGG, 6 x 6 for AlexNet at 224)
        C_last = self.layers[-1].conv.cout
        if (h, w) != tuple(self.pool_hw) or h * w * C_last != self.feat:
            raise NotImplementedError(f"native VGG executor: {h}x{w}x{C_last} features vs a {self.feat}-wide classifier "
                                      f"(adaptive pooling to {self.pool_hw} from other sizes is not native)")
        featc = self._buf("featc", N * self.feat)
        Cn.nhwc_nchw16(x, featc, N, h * w, C_last, True)
        p = self.p_drop if train else 0.0
        self._drop_step += 1
        seed = (self._drop_seed * 0x100000001B3 + self._drop_step) & 0x7FFFFFFFFFFFFFFF
        a_in = featc.view(N, self.feat)
        x0 = None
        if self.drop_first:  # AlexNet: Dropout on the (post-ReLU) features -> fc_act_fwd with a zero bias
            x0 = self._buf("fcx0", N * self.feat)
            Cn.fc_act_fwd(featc, self._zeros(self.feat), x0, N, self.feat, p, seed + 7)
            a_in = x0.view(N, self.feat)
        hs = []
        for i in range(2):
            wsl, bsl = self.lin_slots[i]
            out_f = self.lin[i].out_features
            z = self._buf(("fcz", i), N * out_f)
            torch.mm(a_in, self._w_slot(wsl).view(out_f, -1).t(), out=z.view(N, out_f))
            h_ = self._buf(("fch", i), N * out_f)
            # VGG: Dropout behind both hidden ReLUs; AlexNet: behind the first only (its second Dropout feeds Linear 2)
            pi = p if (not self.drop_first or i == 0) else 0.0
            Cn.fc_act_fwd(z, self._p(bsl), h_, N, out_f, pi, seed + i)
            hs.append(h_)
            a_in = h_.view(N, out_f)
        logits = self._buf("logits16", N * self.ncls_pad)
        w3 = self.derived[self.fc_w_off:self.fc_w_off + self.ncls_pad * self.hidden].view(self.ncls_pad, self.hidden)
        torch.mm(a_in, w3.t(), out=logits.view(N, self.ncls_pad))
        saved.update(featc=featc, x0=x0, hs=hs, logits=logits, hw_last=(h, w), p=p)
        return saved

    def _w_slot(self, slot):
        return self.flat.shadow[slot.offset:slot.offset + slot.numel]

    # ---------------------------------------------------------------------------------- backward
    def _backward(self, saved, dlog):
        Cn = self.C
        N = saved["N"]
        p = saved["p"]
        hs = saved["hs"]
        # last Linear: bias (column sums), weight (split-K weight gradient over the batch), data (GEMM)
        Cn.colsum(dlog, N, self.ncls_pad, self.ncls, self._g(self.fcb_slot), 1.0)
        self.grad_ready(self.fcb_slot.index)

        def fc_wg(x_in, dz, wslot, cout, cin, rows):
            def fn():
                self._wgrad(cout, x_in, dz, N, 1, 1, cin, 1, 1, 1, 1, 1, 0, self._g(wslot), cin, rows=rows, cols=cin)
                self.grad_ready(wslot.index)
            self._side_wgrad((dz, x_in), fn)
        fc_wg(hs[1], dlog, self.fc_slot, self.ncls_pad, self.hidden, self.ncls)
        w3 = self.derived[self.fc_w_off:self.fc_w_off + self.ncls_pad * self.hidden].view(self.ncls_pad, self.hidden)
        dh = self._buf(("fcdh", 1), N * self.hidden)
        torch.mm(dlog.view(N, self.ncls_pad), w3, out=dh.view(N, self.hidden))
        x_ins = [saved["featc"] if saved["x0"] is None else saved["x0"], hs[0]]
        for i in (1, 0):
            wsl, bsl = self.lin_slots[i]
            out_f, in_f = self.lin[i].out_features, self.lin[i].in_features
            dz = self._buf(("fcdz", i), N * out_f)
            Cn.fc_act_bwd(dh, hs[i], dz, p if (not self.drop_first or i == 0) else 0.0)
            Cn.colsum(dz, N, out_f, out_f, self._g(bsl), 1.0)
            self.grad_ready(bsl.index)
            fc_wg(x_ins[i], dz, wsl, out_f, in_f, out_f)
            dprev = self._buf(("fcdh", i - 1) if i > 0 else "dfeatc", N * in_f)
            torch.mm(dz.view(N, out_f), self._w_slot(wsl).view(out_f, in_f), out=dprev.view(N, in_f))
            dh = dprev
        if saved["x0"] is not None:  # the feature Dropout's backward (keep mask recovered from x0)
            dfeat = self._buf("dfeat0", N * self.feat)
            Cn.fc_act_bwd(dh, saved["x0"], dfeat, p)
            dh = dfeat
        # back to NHWC: the gradient of the last pooled activation
        h, w = saved["hw_last"]
        C_last = self.layers[-1].conv.cout
        g = self._buf("g_pool", N * h * w * C_last)
        Cn.nhwc_nchw16(dh, g, N, h * w, C_last, False)
        # features in reverse: g is the gradient of layer li's output activation (pooled or not); for an unpooled
        # output, the next conv's backward data already applied the ReLU mask and reduced the BN sums (``fused``)
        fused = None
        for li in range(len(self.layers) - 1, -1, -1):
            L = self.layers[li]
            x_in, hin, win_, y, out, idx = saved["acts"][li]
            c = L.conv
            C = c.cout
            cnt = N * hin * win_
            if L.pool:
                slots = self._buf(("bnslots", C, 2), self.n_slots * C * 2, torch.float64)
                Cn.pooled_bwd_reduce(g, out, L.coef, slots, out.numel() // C, C)
                self._finish(L, slots, cnt)
                dy = self._buf(("dy", li), N * hin * win_ * C)
                if L.pool == 3:  # bias layer (AlexNet): dy = dz, gathered from the <= 4 windows that chose each pixel
                    assert L.bn is None, "MaxPool(3, 2) after a BatchNorm is not native"
                    Cn.maxpool_bwd_relu(g, idx, y, L.coef, dy, N, hin, win_, C, pad=0)
                elif L.bn is not None:
                    Cn.maxpool2_bwd(g, idx, out, y, L.bcoef, dy, N, hin, win_, C)
                else:
                    Cn.maxpool2_bwd(g, idx, out, None, None, dy, N, hin, win_, C)
            else:
                self._finish(L, fused, cnt)
                if L.bn is not None:
                    dy = self._buf(("dy", li), N * hin * win_ * C)
                    Cn.bn_bwd_apply(g, None, y, L.bcoef, dy, None, None, None, None, C)
                else:
                    dy = g  # dz is the conv-output gradient of a bias layer
            if L.first:
                self._first_wgrad(saved, dy)
                break
            prev = self.layers[li - 1]
            gp = self._buf(("g", li - 1), N * hin * win_ * c.cin)
            if prev.pool:
                self._conv_bwd(L, x_in, N, hin, win_, dy, gp, None, None)
                fused = None
            else:
                slots = self._buf(("bnslots", c.cin, 2), self.n_slots * c.cin * 2, torch.float64)
                prev.y = saved["acts"][li - 1][3]
                self._conv_bwd(L, x_in, N, hin, win_, dy, gp, prev, slots)
                fused = slots
            g = gp
        self._join_side()

    def _first_wgrad(self, saved, dy0):
        """First conv's weight gradient in window mode: kernel-row pairs (rows 0-1 | 2-3 | ..., the weights of a
        padding row are zero) x 8-pixel windows over the padded NHWC4 image, gathered into the KRSC gradient."""
        N, xp, Hp, Wp = saved["N"], saved["xp"], saved["Hp"], saved["Wp"]
        P, Q = saved["P0"], saved["Q0"]
        c = self.layers[0].conv
        T, U, ldw = self.w0_T, self.w0_U, self.w0_ldw

        def wg():
            tmp = self._buf("w0_dw", c.cout * ldw, torch.float32)
            chunks = self._chunks(N, max(Hp * Wp * 4, P * Q * c.cout))
            for k, (a, b) in enumerate(chunks):
                n = b - a
                key = (c.cout, T, U, 64, n * P * Q, True)
                plan = self._plans.get(key)
                if plan is None:
                    plan = tuple(self.C.conv_wgrad_plan(c.cout, T, U, 64, n * P * Q, self.wgrad_blocks, True))[:2]
                    self._plans[key] = plan
                splits, pps = plan
                ws = self._buf("ws", splits * c.cout * ldw, torch.float32)
                self.C.conv_wgrad(xp[a * Hp * Wp * 4:b * Hp * Wp * 4], dy0[a * P * Q * c.cout:b * P * Q * c.cout], ws, n,
                                  Hp, Wp, 64, c.cout, T, U, P, Q, c.st, c.st, 0, 0, 2, 8, ldw, splits, pps, 4, True)
                self.C.wgrad_reduce(ws, splits, c.cout, ldw, ldw, c.cout * ldw, tmp, ldw, 1.0, k > 0)
            self.C.gather32(tmp, self.w0_gidx, self._g(c.slot))
            self.grad_ready(c.pid)
        self._side_wgrad((dy0, xp), wg)


def make_executor(model, flat, device, dtype, **kw):
    """The native 16-bit executor for ``model``: :class:`ResNetExecutor` (ResNet / Wide-ResNet / ResNeXt) or
    :class:`VGGExecutor` (VGG / VGG-BN / AlexNet)."""
    if isinstance(model, (VGG, AlexNet)):
        return VGGExecutor(model, flat, device, dtype, **kw)
    return ResNetExecutor(model, flat, device, dtype, **kw)
