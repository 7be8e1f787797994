"""Native ResNet executor: explicit NHWC forward/backward over the gfx950 kernels.

Instead of tracing a graph or dispatching op-by-op through autograd, the executor walks the ResNet
topology (torchvision-compatible :class:`~.resnet.ResNet`, Basic and Bottleneck blocks) and launches
our HIP kernels directly, with the cross-op fusions a CNN training step needs on MI355X:

* conv forward = implicit-GEMM MFMA kernel whose epilogue emits the BatchNorm batch statistics
  (no extra pass over the conv output to compute mean/var);
* BN-apply + residual (+ BN of the downsample branch) + ReLU = one elementwise pass;
* stem BN + ReLU + 3x3/2 max-pool = one pass (the 112x112 post-ReLU tensor never exists);
* backward: one reduction pass per block output computes the BN-backward sums of BOTH residual
  branches; the identity-gradient add of a residual block happens in the dgrad epilogue;
* weight gradients are written straight into the flat fp32 gradient buffer (DDP bucket views) and
  the bucketer is notified per parameter so RCCL all-reduces overlap the rest of backward;
* cross-entropy forward+backward+accuracy is one kernel with the AMP loss scale folded in.

Numerics: 16-bit (bf16 or fp16) activations and weights, fp32 accumulation/statistics, fp32 master
weights and gradients.  Reference call sites mirrored here:
`distributed.py:246-263` (forward, loss, backward, step) and `distributed_syncBN_amp.py:259-278`.
"""
from __future__ import annotations

import json
import os

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..ops import native
from ..ops.conv import conv_tile as _conv_tile, dgrad_phases, dgrad_weight_index
from .resnet import BasicBlock, Bottleneck, ResNet

_BUF_POISON = os.environ.get("PDT_BUF_POISON", "0") == "1"


def _load_tuned():
    """Shipped autotune results (the analogue of a cudnn.benchmark cache, `distributed.py:104`): per-shape conv tiles
    that PDT_AUTOTUNE=1 measured faster than ops.conv.conv_tile on MI355X (models/tuned_tiles_mi355x.json: ResNet-50
    at B = 1200).  PDT_TUNED_TILES=0 ignores them."""
    if os.environ.get("PDT_TUNED_TILES", "1") != "1":
        return {}
    from .tuned import ARITY16, TABLE16, load_table
    out = load_table(TABLE16, ARITY16)
    if os.environ.get("PDT_TUNED_EXTRA"):  # more tables (A/B of candidate entries); later files win
        for path in os.environ["PDT_TUNED_EXTRA"].split(os.pathsep):
            out.update(load_table(path, ARITY16, shipped=False))
    return out


_TUNED = _load_tuned()

class _Conv:
    """Static description of one convolution and its derived (dgrad) weight layouts."""

    def __init__(self, conv: nn.Conv2d, flat, derived_maps: List[torch.Tensor], derived_off: List[int],
                 fwd_maps: Optional[list] = None):
        """``fwd_maps``: grouped convs append (conv, map) pairs of their FORWARD weight layouts here; the executor
        places those where the forward-read layouts are gathered (update_derived)."""
        assert conv.dilation == (1, 1), "native executor: dilation unsupported"
        self.mod = conv
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.groups = conv.groups
        self.R, self.S = conv.kernel_size
        self.st = conv.stride[0]
        self.pad = conv.padding[0]
        assert conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
        self.slot = flat.slot(conv.weight)
        self.pid = self.slot.index
        self.phases = []  # (ph, pw, T, U, ioff_h, ioff_w, derived offset, derived numel)
        base = self.slot.offset
        if self.groups > 1:
            self._init_grouped(base, derived_maps, derived_off, fwd_maps)
            return
        for ph, pw, rs, ss, ioff_h, ioff_w in dgrad_phases(self.R, self.S, self.st, self.pad):
            m = (base + dgrad_weight_index(self.cout, self.cin, self.R, self.S, rs, ss)).to(torch.int32)
            self.phases.append((ph, pw, len(rs), len(ss), ioff_h, ioff_w, derived_off[0], m.numel()))
            derived_maps.append(m)
            derived_off[0] += m.numel()

    GSLICE = 64  # channel slice of the grouped convolutions (csrc/bindings.cpp gconv_*)

    def _init_grouped(self, base: int, derived_maps, derived_off, fwd_maps) -> None:
        """Grouped conv (ResNeXt) as width / 64 dense channel slices with block-diagonal weights: per slice j the
        forward layout [64][R][S][64] and the backward-data phase layouts, gathered from the grouped parameter
        [cout][R][S][cg] (zeros off the diagonal blocks); the weight gradient keeps the diagonal blocks of the dense
        slice gradients (``gidx``)."""
        G, cg, S_, R, S = self.groups, self.cin // self.groups, self.GSLICE, self.R, self.S
        if not (self.cin == self.cout and self.cin % S_ == 0 and S_ % cg == 0):
            raise NotImplementedError(f"native executor: grouped conv {self.cin}->{self.cout} / {G} groups needs "
                                      "equal widths, width % 64 == 0 and 64 % (channels per group) == 0")
        self.cg, self.nslice = cg, self.cin // S_
        k = torch.arange(S_).view(-1, 1, 1, 1)
        t = torch.arange(R).view(1, -1, 1, 1)
        u = torch.arange(S).view(1, 1, -1, 1)
        c = torch.arange(S_).view(1, 1, 1, -1)
        self.gfwd = []     # per slice: (derived offset) of its forward layout, filled by the executor
        self.gphases = []  # per slice: list of phases (ph, pw, T, U, ioff_h, ioff_w, derived offset)
        for j in range(self.nslice):
            src = base + (((j * S_ + k) * R + t) * S + u) * cg + c % cg
            dense = torch.where(k // cg == c // cg, src, torch.full_like(src, -1)).reshape(-1)
            fwd_maps.append((self, j, dense.to(torch.int32)))
            ph_list = []
            for ph, pw, rs, ss, ioff_h, ioff_w in dgrad_phases(R, S, self.st, self.pad):
                m = dense[dgrad_weight_index(S_, S_, R, S, rs, ss)].to(torch.int32)
                ph_list.append([ph, pw, len(rs), len(ss), ioff_h, ioff_w, derived_off[0]])
                derived_maps.append(m)
                derived_off[0] += m.numel()
            self.gphases.append(ph_list)
        # weight gradient: grouped [cout][R][S][cg] <- dense slice partials [nslice][64][R*S*64]
        kk = torch.arange(self.cout).view(-1, 1, 1, 1)
        cl = torch.arange(cg).view(1, 1, 1, -1)
        jj, kl = kk // S_, kk % S_
        self.gidx = ((jj * S_ + kl) * (R * S * S_) + (t * S + u) * S_ + (kl // cg) * cg + cl).reshape(-1).to(torch.int32)

    def out_hw(self, H: int, W: int) -> Tuple[int, int]:
        return (H + 2 * self.pad - self.R) // self.st + 1, (W + 2 * self.pad - self.S) // self.st + 1


class _BN:
    def __init__(self, bn: nn.BatchNorm2d, flat, device):
        self.mod = bn
        self.C = bn.num_features
        self.eps = bn.eps
        self.momentum = bn.momentum if bn.momentum is not None else 0.1
        self.gslot = flat.slot(bn.weight)
        self.bslot = flat.slot(bn.bias)
        self.coef = torch.zeros(4 * self.C, dtype=torch.float32, device=device)
        self.bcoef = torch.zeros(3 * self.C, dtype=torch.float32, device=device)
        self.sums = torch.zeros(2 * self.C, dtype=torch.float64, device=device)
        self.bsums = torch.zeros(4 * self.C, dtype=torch.float64, device=device)


class ResNetExecutor:
    """Runs a :class:`ResNet` on one GPU with the native kernels.

    ``train_step`` = forward + loss/accuracy + backward (gradients into ``flat.grad``);
    ``eval_step`` = forward with running statistics.  The optimizer step is separate
    (:class:`~pytorch_distributed_template_amd.optim.sgd.FusedSGD`).
    """

    def __init__(self, model: ResNet, flat, device: torch.device, dtype: torch.dtype,
                 grad_ready: Optional[Callable[[int], None]] = None,
                 syncbn_group=None, wgrad_blocks: int = 2048, wgrad_blocks_1x1: int = 512, autotune: bool = False,
                 syncbn_allreduce: Optional[Callable[[torch.Tensor], None]] = None, syncbn_world: int = 0,
                 syncbn_allreduce_fwd: Optional[Callable[[torch.Tensor], None]] = None):
        if dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("native executor computes in bf16 or fp16")
        if not isinstance(model, ResNet):
            raise NotImplementedError("native executor supports torchvision-style ResNets / ResNeXts")
        self.C = native.C
        self.n_slots = self.C.stat_slots()
        self.model = model
        self.flat = flat
        self.device = torch.device(device)
        self.dtype = dtype
        self._user_grad_ready = grad_ready or (lambda pid: None)
        # Weight gradients run on a side HIP stream, concurrently with the rest of the backward chain
        # (dgrad -> BN-backward passes of the earlier layers): the compute-bound wgrad kernels overlap the
        # memory-bound elementwise passes.  Ordering: the side stream waits for the main stream before
        # each wgrad (its dY is ready); a main-stream write to a buffer a pending wgrad still reads waits
        # for that wgrad (_buf); gradient-bucket all-reduces are launched from the side stream after it
        # caught up with the main stream (so they see both streams' gradient writes); the main stream joins
        # the side stream at the end of backward.  PDT_WGRAD_STREAM=0 runs everything on one stream.
        self.side = None
        if self.device.type == "cuda" and os.environ.get("PDT_WGRAD_STREAM", "1") != "0":
            self.side = torch.cuda.Stream(device=self.device)
        self._on_side = False
        self._pending_reads: Dict[int, "torch.cuda.Event"] = {}
        self.syncbn_group = syncbn_group
        # SyncBN statistic all-reduce (fp64 sums): a native RCCL communicator's all_reduce when one is given
        # (``syncbn_world`` = its size; a world of 1 runs the whole SyncBN path with identity all-reduces, which
        # measures its overhead on one GPU), else torch.distributed on syncbn_group
        self.syncbn = syncbn_allreduce is not None or syncbn_group is not None
        if syncbn_allreduce is not None:
            self.syncbn_world = int(syncbn_world) if syncbn_world else 1
            self._sync_sum = syncbn_allreduce
        self._sync_sum_fwd = syncbn_allreduce_fwd  # forward statistics (None: same as _sync_sum)
        if syncbn_group is not None and syncbn_allreduce is None:
            import torch.distributed as dist
            self.syncbn_world = dist.get_world_size(syncbn_group)
            self._sync_sum = lambda t: dist.all_reduce(t, group=syncbn_group)
        self.wgrad_blocks = wgrad_blocks  # split-K targets (tools/conv_bench.py sweep: 3x3 best ~2048, 1x1 ~512)
        self.wgrad_blocks_1x1 = wgrad_blocks_1x1
        # generic-path stem tile (window mode, BK=32) and the dedicated stem kernel's workgroups per CU (round-3/4
        # sweeps; their tuning knobs were removed in round 6)
        self.stem_tile = (256, 64)
        self.stem_blocks_per_cu = 2
        self.wgrad_l1 = os.environ.get("PDT_WGRAD_L1", "1") == "1"
        self.bk32_short = True
        self._c1x1 = hasattr(self.C, "conv1x1_c64")
        self._c1x1x = hasattr(self.C, "conv1x1x")
        # a layer1 block's inner BN + ReLU applied by its consumers (conv2 forward and conv2 weight
        # gradient) to their staged input tiles in LDS; the activation relu(bn(z1)) is never written or re-read
        self.fuse_pre = os.environ.get("PDT_FUSE_PRE", "1") == "1"
        # ... and ResNet-50 layer1's bn2 + ReLU applied by conv3 (the persistent 1x1 64 -> 256 kernel) and conv3's
        # weight gradient (the 128-pair tile): a2 = relu(bn2(z2)) is never written or re-read
        self.fuse_pre_1x1 = os.environ.get("PDT_FUSE_PRE1X1", "1") == "1"
        # stem backward: weight gradient with in-kernel dY (PDT_STEM_FUSED=0: separate apply pass + wgrad)
        self.stem_fused = os.environ.get("PDT_STEM_FUSED", "1") == "1"
        # 1x1/2 downsample data gradient written compact and added by phase 0 of the 3x3/2 dgrad
        self.compact_ds = True
        self.bwd_buf_per_block = True
        # backward-only derived weight layouts gathered on the side stream under the forward
        self.split_derived = True
        # block-output BN-backward reduce fused into the next block's first dgrad epilogue where dX has at most
        # this many pixels per image (larger: plain dgrad + a separate reduce pass).  Round 2 made the fused masked
        # epilogues straight-line (tools/epi_bench.py: layer1 803 -> 598 us, layer2 2-branch 766 -> 508 us), after
        # which fusing at every resolution measured equal or faster than the separate reduce (A/B 21.76 -> 21.71
        # ms/step), so it is on everywhere.
        self.fuse_block_bn_maxhw = 1000000
        # uint8 input batches are normalised inside stem_pack: x/255 -> (x - mean) / std
        from ..data.transforms import IMAGENET_MEAN, IMAGENET_STD
        std = torch.tensor(IMAGENET_STD)
        self.norm_scale = (1.0 / (255.0 * std)).to(self.device)
        self.norm_shift = (-torch.tensor(IMAGENET_MEAN) / std).to(self.device)
        self.autotune = autotune or os.environ.get("PDT_AUTOTUNE", "0") == "1"
        self._tiles: Dict[tuple, Tuple[int, int]] = {}
        derived_maps: List[torch.Tensor] = []
        off = [0]
        gfwd_maps: list = []  # forward layouts of the grouped convs (gathered with the stem / fc ones, see below)

        def conv(c):
            return _Conv(c, flat, derived_maps, off, gfwd_maps)

        self.stem = conv(model.conv1)
        self.stem_bn = _BN(model.bn1, flat, self.device)
        self.blocks: List[dict] = []
        for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
            for blk in layer:
                d = {"kind": "basic" if isinstance(blk, BasicBlock) else "bottleneck"}
                convs = [blk.conv1, blk.conv2] + ([blk.conv3] if d["kind"] == "bottleneck" else [])
                bns = [blk.bn1, blk.bn2] + ([blk.bn3] if d["kind"] == "bottleneck" else [])
                d["convs"] = [conv(c) for c in convs]
                d["bns"] = [_BN(b, flat, self.device) for b in bns]
                if blk.downsample is not None:
                    d["ds_conv"] = conv(blk.downsample[0])
                    d["ds_bn"] = _BN(blk.downsample[1], flat, self.device)
                else:
                    d["ds_conv"] = None
                    d["ds_bn"] = None
                self.blocks.append(d)
        # stem weight in "window" layout [Cout][R][32]: column j = s*4 + c of kernel row r (s < 7, c < 3),
        # matching 8-pixel x 4-channel windows of the zero-padded NHWC4 image (no im2col)
        st = self.stem
        assert st.cin <= 4 and st.S <= 8, "window-mode stem needs Cin <= 4 and kernel width <= 8"
        self.stem_pairs = (st.R + 1) // 2  # the stem weight gradient works on kernel-row pairs
        k = torch.arange(st.cout).view(-1, 1, 1)
        r = torch.arange(st.R).view(1, -1, 1)
        j = torch.arange(32).view(1, 1, -1)
        s_, c_ = j // 4, j % 4
        src = st.slot.offset + ((k * st.R + r) * st.S + s_) * st.cin + c_
        m = torch.where((s_ < st.S) & (c_ < st.cin), src, torch.full_like(src, -1))
        # dedicated persistent stem kernel (csrc/kernels/stem.hip) for the torchvision stem geometry
        self.stem_kernel = st.cout == 64 and st.R == 7 and st.S == 7 and st.st == 2 and st.pad == 3
        self.stem_w_off = off[0]
        derived_maps.append(m.reshape(-1).to(torch.int32))
        off[0] += m.numel()
        # grouped convs' forward layouts right behind the stem's: inside the range update_derived gathers on the
        # compute stream ahead of the forward
        for gc, j, gm in gfwd_maps:
            gc.gfwd.append(off[0])
            derived_maps.append(gm)
            off[0] += gm.numel()
        # stem weight-gradient scatter: [Cout][R/2 pairs][2][32] (wgrad window tile) -> KRSC [Cout][R][S][Cin]
        kk = torch.arange(st.cout).view(-1, 1, 1, 1)
        rr = torch.arange(st.R).view(1, -1, 1, 1)
        ss = torch.arange(st.S).view(1, 1, -1, 1)
        cc = torch.arange(st.cin).view(1, 1, 1, -1)
        self.stem_gidx = (kk * (self.stem_pairs * 64) + (rr // 2) * 64 + (rr % 2) * 32 + ss * 4 + cc).reshape(-1).to(
            torch.int32).to(self.device)
        # fc: padded [NP][F] (forward) and its transpose [F][NP] (backward-data)
        fc = model.fc
        self.ncls, self.feat = fc.out_features, fc.in_features
        self.ncls_pad = (self.ncls + 127) // 128 * 128
        self.fc_slot = flat.slot(fc.weight)
        self.fcb_slot = flat.slot(fc.bias)
        o = torch.arange(self.ncls_pad).view(-1, 1)
        f = torch.arange(self.feat).view(1, -1)
        m = torch.where(o < self.ncls, self.fc_slot.offset + o * self.feat + f, torch.full_like(o * f, -1))
        self.fc_w_off = off[0]
        derived_maps.append(m.reshape(-1).to(torch.int32))
        off[0] += m.numel()
        self.fc_wt_off = off[0]
        mt = m.t().contiguous()
        derived_maps.append(mt.reshape(-1))
        off[0] += mt.numel()
        self.derived_idx = torch.cat([m.to(torch.int32) for m in derived_maps]).to(self.device)
        self.derived = torch.zeros(off[0], dtype=dtype, device=self.device)
        for b in self.blocks:
            for c in b["convs"]:
                if c.groups > 1:
                    c.gidx = c.gidx.to(self.device)
        self._bufs: Dict[Tuple, torch.Tensor] = {}
        self._plans: Dict[Tuple, Tuple[int, int]] = {}
        from ..ops import validate
        self._buf_guard = (int(os.environ.get("PDT_VALIDATE_GUARD", "0") or 0)
                           if validate.level_from_env() > 0 and self.device.type == "cuda" else 0)
        self.update_derived()

    # ---------------------------------------------------------------------------------- helpers
    def update_derived(self) -> None:
        """Rebuild every derived 16-bit weight layout from the shadow (after each optimizer step).

        With the side stream, only the layouts the forward pass reads (stem, fc) are gathered on the compute
        stream; the backward-data layouts (every conv's phase weights, the transposed fc) are gathered on the
        side stream, overlapped with the forward pass, and backward waits for them (``_derived_ev``)."""
        if self.side is None or not self.split_derived or torch.cuda.is_current_stream_capturing():
            # (a captured step must end joined: no side-stream work may trail the graph)
            self.C.gather16(self.flat.shadow, self.derived_idx, self.derived)
            return
        lo, hi = self.stem_w_off, self.fc_wt_off
        with torch.cuda.device(self.device):
            self.C.gather16(self.flat.shadow, self.derived_idx[lo:hi], self.derived[lo:hi])
            self.side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side):
                if lo > 0:
                    self.C.gather16(self.flat.shadow, self.derived_idx[:lo], self.derived[:lo])
                if hi < self.derived.numel():
                    self.C.gather16(self.flat.shadow, self.derived_idx[hi:], self.derived[hi:])
                ev = torch.cuda.Event()
                ev.record(self.side)
        self._derived_ev = ev

    def _wait_derived(self) -> None:
        ev = getattr(self, "_derived_ev", None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._derived_ev = None

    def _buf(self, key, numel: int, dtype=None) -> torch.Tensor:
        dtype = dtype or self.dtype
        k = (key, dtype)
        t = self._bufs.get(k)
        if t is None or t.numel() < numel:
            if getattr(self, "_buf_guard", 0):  # PDT_VALIDATE_GUARD: a canary tail behind every work buffer (ops/validate.py)
                from ..ops import validate
                full = torch.empty(numel + self._buf_guard, dtype=dtype, device=self.device)
                validate.fill_canary(full[numel:])
                validate.validator().register_tail_guard(f"{key}/{str(dtype).replace('torch.', '')}", full[numel:])
                t = full[:numel]
            else:
                t = torch.empty(numel, dtype=dtype, device=self.device)
                if _BUF_POISON:  # PDT_BUF_POISON=1: NaN / 0xFF so a buffer read before any kernel wrote it shows
                    t.fill_(float("nan") if t.is_floating_point() else -1)
            self._bufs[k] = t
        if self._pending_reads:  # the caller is about to overwrite it: wait for side-stream readers
            ev = self._pending_reads.pop(t.data_ptr(), None)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
        return t[:numel]

    def grad_ready(self, pid: int) -> None:
        """Forward a parameter's gradient readiness to the bucketer; with the side stream, from the side
        stream after it caught up with the main stream (see __init__)."""
        if self.side is None or self._on_side:
            self._user_grad_ready(pid)
            return
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self._user_grad_ready(pid)

    def _stem_fused_ok(self, Q0: int) -> bool:
        return self.stem_fused and self.stem_pairs == 4 and Q0 % 2 == 0

    def _side_wgrad(self, reads, fn) -> None:
        """Run ``fn`` (a weight gradient + its grad_ready) on the side stream behind the main stream's work
        so far; later main-stream writes to ``reads`` (a tensor or a tuple of them) wait for it.  ``reads`` must
        list EVERY tensor ``fn`` reads that the main stream could rewrite before the end of backward: its dY, its
        input activation, the producer-BN coefficients it applies (layer1), the stem's packed image / argmax /
        pre-BN output; a buffer taken from ``_buf`` for writing then waits for the pending read."""
        if self.side is None:
            fn()
            return
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self._on_side = True
            try:
                fn()
            finally:
                self._on_side = False
            ev = torch.cuda.Event()
            ev.record(self.side)
        for r in reads if isinstance(reads, tuple) else (reads,):
            r.record_stream(self.side)  # the allocator must not recycle it before the side stream read it
            self._pending_reads[r.data_ptr()] = ev

    def _join_side(self) -> None:
        if self.side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self._pending_reads.clear()

    def _w(self, c: _Conv) -> torch.Tensor:
        s = c.slot
        return self.flat.shadow[s.offset:s.offset + s.numel]

    def _p(self, slot):
        return self.flat.data[slot.offset:slot.offset + slot.numel]

    def _g(self, slot):
        return self.flat.grad[slot.offset:slot.offset + slot.numel]

    # ---------------------------------------------------------------------------------- conv ops
    def _pre_ok(self, nxt: _Conv, N: int, H: int, W: int, train: bool) -> bool:
        """Can ``nxt`` (the conv consuming a block-internal BN + ReLU) apply that BN itself (conv_fwd_pre +
        the fused layer1 weight gradient)?"""
        if not (self.fuse_pre and train and nxt.groups == 1):
            return False
        if nxt.R == 1:
            return (self.fuse_pre_1x1 and nxt.S == 1 and nxt.st == 1 and nxt.pad == 0 and nxt.cin == 64 and
                    nxt.cout == 256 and self._c1x1 and self.C.conv1x1_c64_supported(64, 256) and
                    os.environ.get("PDT_WGRAD_PAIR", "1") != "0")
        return (self.wgrad_l1 and hasattr(self.C, "conv_fwd_pre") and
                nxt.R == 3 and nxt.S == 3 and nxt.st == 1 and
                nxt.pad == 1 and nxt.cin == 64 and nxt.cout == 64 and self.C.conv_fwd_pre_supported(N, H, W) and
                self.C.wgrad_3x3c64_supported(64, 64, 3, 3, W, 1, 1))

    def conv_fwd(self, c: _Conv, x, N, H, W, y, stats: bool, w=None, cin=None, R=None, S=None, st=None, pad=None,
                 pre=None, stats_tag=None, fin: Optional[_BN] = None):
        """``fin``: the BatchNorm consuming y -- its training finalize is launched right behind the conv."""
        if c.groups > 1:
            return self._gconv_fwd(c, x, N, H, W, y, stats, stats_tag, fin)
        if pre is not None:  # x is the producer conv's raw output; pre = its BN coefficients (layer1 only)
            key = ("stats", c.cout) if stats_tag is None else ("stats", c.cout, stats_tag)
            sp = self._buf(key, self.n_slots * c.cout * 2, torch.float64)
            if c.R == 1:  # ResNet-50 layer1 conv3 (see _pre_ok)
                self.C.conv1x1_c64(x, self._w(c), y, sp, N * H * W, pre=pre)
            else:
                self.C.conv_fwd_pre(x, self._w(c), y, sp, pre, N, H, W)
            if fin is not None:
                self.bn_train_finalize(fin, sp, 0, N * H * W)
            return H, W, sp, N * H * W
        cin = cin or c.cin
        R = R or c.R
        S = S or c.S
        st = st or c.st
        pad = c.pad if pad is None else pad
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1
        bk = 64 if cin % 64 == 0 else 32
        tkey = ("fwd", N, H, W, cin, c.cout, R, S, st, stats)
        if cin * R * S == 64 and c.cout >= 256 and self.bk32_short and tkey not in _TUNED:
            # a single 64-wide K-step: two 32-wide steps on the 3-stage ring overlap load and MFMA
            # (tools/conv_bench.py --r50: ResNet-50 1x1 64->256 with statistics 162 vs 142 TF/s)
            bk = 32
        M = N * P * Q
        sp = None
        if stats:
            key = ("stats", c.cout) if stats_tag is None else ("stats", c.cout, stats_tag)
            sp = self._buf(key, self.n_slots * c.cout * 2, torch.float64)
        wt = self._w(c) if w is None else w
        if (R == 1 and S == 1 and st == 1 and pad == 0 and cin == 64 and c.cout == 256 and
                self._c1x1 and self.C.conv1x1_c64_supported(cin, c.cout)):
            # ResNet-50 layer1's expanding 1x1 convs: the persistent store-overlapped kernel (conv1x1.hip)
            self.C.conv1x1_c64(x, wt, y, sp, M)
            if stats and fin is not None:
                self.bn_train_finalize(fin, sp, 0, M)
            return P, Q, sp, M
        if (R == 1 and S == 1 and pad == 0 and self._c1x1x and (
                (st == 1 and c.cout == 4 * cin) or (st == 2 and c.cout == 2 * cin)) and
                self.C.conv1x1x_supported(cin, c.cout)):
            # layers 2-4's expanding 1x1 convs (bottleneck conv3 and the stride-2 downsample convs of layers 2-3):
            # the persistent sliced kernel (conv1x1x.hip).  (The reducing 512 -> 128 conv1 of layer2 on the same
            # kernel measured 72.32/72.35 -> 72.32/72.25 ms/step: not taken.)
            self.C.conv1x1x(x, wt, y, sp, M, cin, c.cout, st, N, H, W)
            if stats and fin is not None:
                self.bn_train_finalize(fin, sp, 0, M)
            return P, Q, sp, M

        def launch(bm, bn):
            self.C.conv_fwd(x, wt, y, None, sp, N, H, W, cin, c.cout, R, S, P, Q, st, st,
                            -pad, -pad, 1, 1, P, Q, 1, 1, 0, 0, bm, bn, bk, 0)
        bm, bn = self._tile(tkey, c.cout, bk, launch, kdim=cin * R * S, m=M)
        launch(bm, bn)
        if stats and fin is not None:
            self.bn_train_finalize(fin, sp, 0, M)
        return P, Q, sp, M

    def _gconv_fwd(self, c: _Conv, x, N, H, W, y, stats: bool, stats_tag, fin):
        """Grouped conv forward: one launch per 64-channel slice (block-diagonal dense weights, strided operands);
        the slices' BN statistics land in their channel ranges of ONE statistics buffer."""
        P, Q = c.out_hw(H, W)
        sp = None
        if stats:
            key = ("stats", c.cout) if stats_tag is None else ("stats", c.cout, stats_tag)
            sp = self._buf(key, self.n_slots * c.cout * 2, torch.float64)
        bm, bn = _conv_tile(c.GSLICE, c.GSLICE * c.R * c.S)
        n = c.GSLICE * c.R * c.S * c.GSLICE
        # every slice in ONE launch (blockIdx.z = slice; the slices' forward layouts are consecutive in derived)
        o = c.gfwd[0]
        self.C.gconv_fwd(x, self.derived[o:o + n * c.nslice], y, sp, N, H, W, c.cout, c.R, c.st, c.pad, P, Q, -1, bm, bn)
        if stats and fin is not None:
            self.bn_train_finalize(fin, sp, 0, N * P * Q)
        return P, Q, sp, N * P * Q

    def _gconv_bwd(self, c: _Conv, x, N, H, W, dy, P, Q, dx, bnb, fin):
        """Grouped conv backward: per 64-channel slice the dense weight-gradient partials (diagonal blocks gathered
        into the grouped gradient) and the backward data with the producer BN's fused reduce (bnb mode 1)."""
        def wg():
            R, S, S_ = c.R, c.S, c.GSLICE
            ldw = R * S * S_
            if self.wgrad_l1 and self.C.wgrad_3x3c64_supported(S_, S_, R, S, W, c.st, c.pad):
                # ResNeXt stage 1: every slice on the layer1 halo weight-gradient kernel (all 9 taps per staged tile)
                blocks = self.C.wgrad_blocks_3x3c64()
                ws = self._buf("ws", blocks * c.nslice * S_ * ldw, torch.float32)
                tmp = self._buf("gconv_dw", c.nslice * S_ * ldw, torch.float32)
                parts = self.C.gconv_wgrad_l1(x, dy, ws, N, H, W, c.cin)
                self.C.wgrad_reduce(ws, parts, c.nslice * S_, ldw, ldw, c.nslice * S_ * ldw, tmp, ldw, 1.0, False)
                self.C.gather32(tmp, c.gidx, self._g(c.slot))
                self.grad_ready(c.pid)
                return
            key = (S_, R, S, S_, N * P * Q, False)
            plan = self._plans.get(key)
            if plan is None:
                plan = tuple(self.C.conv_wgrad_plan(S_, R, S, S_, N * P * Q, self.wgrad_blocks, False))[:2]
                self._plans[key] = plan
            splits, pps = plan
            # every slice in ONE launch: partials [splits][nslice][64][ldw], one reduction over nslice * 64 rows
            ws = self._buf("ws", splits * c.nslice * S_ * ldw, torch.float32)
            tmp = self._buf("gconv_dw", c.nslice * S_ * ldw, torch.float32)
            self.C.gconv_wgrad(x, dy, ws, N, H, W, c.cin, R, P, Q, c.st, c.pad, -1, ldw, splits, pps)
            self.C.wgrad_reduce(ws, splits, c.nslice * S_, ldw, ldw, c.nslice * S_ * ldw, tmp, ldw, 1.0, False)
            self.C.gather32(tmp, c.gidx, self._g(c.slot))
            self.grad_ready(c.pid)
        self._side_wgrad((dy, x), wg)
        if dx is None:
            return
        assert bnb is None or bnb[0] == 1, "grouped conv backward-data: inner-BN epilogue only"
        bm, bn = _conv_tile(c.GSLICE, c.GSLICE * c.R * c.S)
        # every slice in ONE launch: slice 0's phases, the other slices' phase weights follow at the stride of one
        # slice's whole phase set (so every phase must be present; a degenerate tiny image runs slice by slice)
        phases = [p for p in c.gphases[0] if H - p[0] > 0 and W - p[1] > 0]
        kw = {} if bnb is None else dict(bn_y1=bnb[1], bn_coef1=bnb[2], bn_slots=bnb[6])
        if len(phases) == len(c.gphases[0]):
            self.C.gconv_dgrad(dy, self.derived, dx, N, P, Q, c.cin, H, W, c.st, phases, -1, bm, bn, **kw)
        else:
            for j in range(c.nslice):
                phases = [p for p in c.gphases[j] if H - p[0] > 0 and W - p[1] > 0]
                self.C.gconv_dgrad(dy, self.derived, dx, N, P, Q, c.cin, H, W, c.st, phases, j, bm, bn, **kw)
        if fin is not None and bnb is not None:
            self._bn_bwd_finish(bnb[6], fin[0], fin[1], fin[2])

    # per-shape tile choice: the static table (ops.conv.conv_tile), or -- with autotune on, the analogue of
    # the reference's cudnn.benchmark=True (`distributed.py:104`) -- the fastest candidate timed once per shape
    _CANDIDATES = ((128, 128), (256, 64), (128, 64), (64, 128), (256, 128), (256, 256), (512, 128))

    def _tile(self, key, n_dim, bk, launch, fused_epilogue: bool = False, kdim: int = 0, m: int = 0):
        hit = self._tiles.get(key)
        if hit is not None:
            return hit
        choice = _TUNED.get(key) or _conv_tile(n_dim, kdim if bk == 64 else 0, m)
        if self.autotune and bk == 64:
            cands = [(bm, bn) for bm, bn in self._CANDIDATES if n_dim % bn == 0 and
                     (not fused_epilogue or bm * bn in (16384, 32768, 65536))]
            best = None
            for bm, bn in cands:
                launch(bm, bn)  # warm
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                launch(bm, bn)
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1)
                if best is None or ms < best[0]:
                    best = (ms, (bm, bn))
            choice = best[1]
            dump = os.environ.get("PDT_AUTOTUNE_DUMP")  # tuned-table candidates: shapes where the static rule lost
            if dump and choice != _conv_tile(n_dim, kdim if bk == 64 else 0, m):
                with open(dump, "a") as f:
                    f.write(json.dumps([list(key), list(choice)]) + "\n")
        self._tiles[key] = choice
        return choice

    def bn_train_finalize(self, bn: _BN, sp, tiles: int, count: int):
        C = bn.C
        if not self.syncbn:  # slot sum + finalize in one launch
            self.C.bn_finalize_slots(sp, float(count), self._p(bn.gslot), self._p(bn.bslot), bn.eps, bn.momentum,
                                     bn.mod.running_mean, bn.mod.running_var, bn.coef, bn.sums, True)
            return
        self.C.bn_slot_sum(sp, C, 2, bn.sums)
        (self._sync_sum_fwd or self._sync_sum)(bn.sums)
        count = count * self.syncbn_world
        self.C.bn_finalize(bn.sums, float(count), self._p(bn.gslot), self._p(bn.bslot), bn.eps, bn.momentum,
                           bn.mod.running_mean, bn.mod.running_var, bn.coef, True)

    def bn_train_finalize_pair(self, bn_a: _BN, sp_a, count_a: int, bn_b: _BN, sp_b, count_b: int):
        """Two BatchNorms whose statistics are ready together (a downsample block's main-branch and downsample
        BN): with SyncBN, ONE all-reduce carries both layers' sums (one latency-bound collective fewer per
        downsample block); without it, the plain per-layer finalize."""
        if not self.syncbn:
            self.bn_train_finalize(bn_a, sp_a, 0, count_a)
            self.bn_train_finalize(bn_b, sp_b, 0, count_b)
            return
        ca, cb = bn_a.C, bn_b.C
        pair = self._buf(("syncbn_pair", ca, cb), 2 * (ca + cb), torch.float64)
        self.C.bn_slot_sum(sp_a, ca, 2, pair[:2 * ca])
        self.C.bn_slot_sum(sp_b, cb, 2, pair[2 * ca:])
        (self._sync_sum_fwd or self._sync_sum)(pair)
        for bn, sums, cnt in ((bn_a, pair[:2 * ca], count_a), (bn_b, pair[2 * ca:], count_b)):
            self.C.bn_finalize(sums, float(cnt * self.syncbn_world), self._p(bn.gslot), self._p(bn.bslot), bn.eps,
                               bn.momentum, bn.mod.running_mean, bn.mod.running_var, bn.coef, True)

    def bn_eval(self, bn: _BN):
        self.C.bn_eval_coef(self._p(bn.gslot), self._p(bn.bslot), bn.mod.running_mean, bn.mod.running_var,
                            bn.eps, bn.coef)

    def conv_bwd(self, c: _Conv, x, N, H, W, dy, P, Q, dx, res=None, wgrad_x=None, wgrad_geom=None, bnb=None,
                 res_phase: int = -1, compact: bool = False, pre=None, fin=None):
        """Weight gradient into the flat grad buffer (+ notify), then data gradient into ``dx``.

        ``bnb`` = (mode, y1, coef1, y2, coef2, out_mask, slots): fuse the consuming BatchNorm's backward
        reduce into the data-gradient epilogue (``dx`` then holds dz = dx * relu'; see conv_fwd.h).
        ``res_phase >= 0``: ``res`` is compact and belongs to that sub-pixel phase only (conv_fwd.h).
        ``compact``: a 1x1 strided conv's data gradient written only on its nonzero phase (0, 0), as a dense
        [N, P, Q, Cin] tensor -- a stride-1 GEMM over the P x Q pixels (the zeros of the other phases are
        neither written nor re-read by the consumer)."""
        if c.groups > 1:
            assert res is None and res_phase < 0 and not compact and pre is None and wgrad_geom is None
            return self._gconv_bwd(c, x, N, H, W, dy, P, Q, dx, bnb, fin)
        # --- wgrad
        if wgrad_geom is None:
            xg, Hx, Wx, Cx, R, S, st, pad = x, H, W, c.cin, c.R, c.S, c.st, c.pad
        else:
            xg, Hx, Wx, Cx, R, S, st, pad = wgrad_geom
        def wg():
            self._wgrad(c.cout, xg, dy, N, Hx, Wx, Cx, R, S, P, Q, st, pad, self._g(c.slot), R * S * Cx, pre=pre)
            self.grad_ready(c.pid)
        self._side_wgrad((dy, xg) + ((pre,) if pre is not None else ()), wg)
        # --- dgrad
        if dx is None:
            return
        bk = 64 if c.cout % 64 == 0 else 32
        dst = c.st
        if compact:
            ph0 = c.phases[0]
            assert c.R == 1 and c.S == 1 and c.pad == 0 and tuple(ph0[:6]) == (0, 0, 1, 1, 0, 0), "compact: 1x1 only"
            phases, H, W, dst = [[0, 0, 1, 1, 0, 0, ph0[6]]], P, Q, 1
        else:
            phases = [[ph, pw, T, U, ioff_h, ioff_w, doff] for (ph, pw, T, U, ioff_h, ioff_w, doff, dn) in c.phases
                      if H - ph > 0 and W - pw > 0]

        def launch(bm, bn):
            if bnb is None and res_phase < 0:
                self.C.conv_dgrad(dy, self.derived, dx, res, N, P, Q, c.cout, c.cin, H, W, dst, phases, bm, bn, bk)
            else:
                self.C.conv_dgrad_bn(dy, self.derived, dx, res, N, P, Q, c.cout, c.cin, H, W, dst, phases, bm, bn,
                                     bk, *(bnb or (0, None, None, None, None, None, None)), res_phase)
        # the binding's own dispatch predicate (csrc/bindings.cpp dgrad_persistent_kind): never re-derived here
        persistent = self.C.conv_dgrad_persistent(c.cout, c.cin, bnb[0] if bnb else 0, dst, phases, H, W, P, Q,
                                                  res_phase) != 0
        if persistent:
            # the binding runs a persistent 1x1 backward-data kernel (conv1x1.hip / conv1x1x.hip), which has no
            # tile: no tile choice (or autotune timing) for this shape (the static tile only satisfies the binding's
            # checks)
            launch(*_conv_tile(c.cin))
        else:
            key = ("dgrad", N, H, W, c.cin, c.cout, c.R, c.S, dst, res is not None, bnb[0] if bnb else 0, res_phase)
            bm, bn = self._tile(key, c.cin, bk, launch, fused_epilogue=bnb is not None, kdim=c.cout * c.R * c.S,
                                m=N * H * W)
            launch(bm, bn)
        if fin is not None and bnb is not None:  # fin = (count, bn1, bn2): the fused reduce's BN-backward finalize
            self._bn_bwd_finish(bnb[6], fin[0], fin[1], fin[2])

    def _wgrad(self, cout, x, dy, N, H, W, C, R, S, P, Q, st, pad, gout, ldo, rows=None, cols=None, cs=0,
               win=False, dil=1, pre=None):
        if not win and self.wgrad_l1 and self.C.wgrad_3x3c64_supported(C, cout, R, S, W, st, pad):
            # ResNet layer1 3x3 convs: all 9 taps per block over staged 4-row tiles (csrc conv_wgrad.hip); with
            # ``pre`` x is the producer's raw output and the kernel applies its BN + ReLU to each staged tile
            blocks = self.C.wgrad_blocks_3x3c64()
            ws = self._buf("ws", blocks * 64 * 576, torch.float32)
            if pre is None:
                parts = self.C.conv_wgrad_3x3c64(x, dy, ws, N, H, W)
            else:
                parts = self.C.conv_wgrad_3x3c64(x, dy, ws, N, H, W, pre)
            self.C.wgrad_reduce(ws, parts, 64, 576, 576, 64 * 576, gout, ldo, 1.0, False)
            return
        assert pre is None or (R == 1 and S == 1 and C == 64 and st == 1 and pad == 0 and not win), \
            "fused producer BN: the layer1 3x3 weight-gradient kernel or a 1x1 C = 64 conv (128-pair tile)"
        key = (cout, R, S, C, N * P * Q, win)
        plan = self._plans.get(key)
        if plan is None:
            target = self.wgrad_blocks if R * S > 1 else self.wgrad_blocks_1x1
            plan = tuple(self.C.conv_wgrad_plan(cout, R, S, C, N * P * Q, target, win))[:2]
            self._plans[key] = plan
        splits, pps = plan
        ldw = R * S * C
        ws = self._buf("ws", splits * cout * ldw, torch.float32)
        self.C.conv_wgrad(x, dy, ws, N, H, W, C, cout, R, S, P, Q, st, st, pad, pad, dil, dil, ldw, splits, pps, cs,
                          win, pre=pre)
        self.C.wgrad_reduce(ws, splits, rows or cout, cols or ldw, ldw, cout * ldw, gout, ldo, 1.0, False)

    def bn_bwd(self, bn1: _BN, y1, g, out_mask, count: int, bn2: Optional[_BN] = None, y2=None):
        """Reduce pass + finalize (dgamma/dbeta into grad buffer).  Returns nothing; coefficients in bcoef."""
        C = bn1.C
        rows = g.numel() // C
        blocks = self.C.bn_bwd_reduce_blocks(rows, C)
        K = 4 if bn2 is not None else 2
        slots = self._buf(("bnslots", C, K), self.n_slots * C * K, torch.float64)
        self.C.bn_bwd_reduce(g, out_mask, y1, bn1.coef, y2, bn2.coef if bn2 is not None else None, slots, blocks, rows, C)
        self._bn_bwd_finish(slots, count, bn1, bn2)

    def _bn_bwd_finish(self, slots, count: int, bn1: _BN, bn2: Optional[_BN] = None):
        """Slot sums (+ SyncBN all-reduce) -> dgamma/dbeta and the apply coefficients."""
        C = bn1.C
        K = 4 if bn2 is not None else 2
        if not self.syncbn:  # slot sum + finalize of both branches in one launch
            self.C.bn_bwd_finalize_slots(
                slots, K, float(count), bn1.coef, self._p(bn1.gslot), self._g(bn1.gslot), self._g(bn1.bslot),
                bn1.bcoef, bn2.coef if bn2 is not None else None, self._p(bn2.gslot) if bn2 is not None else None,
                self._g(bn2.gslot) if bn2 is not None else None, self._g(bn2.bslot) if bn2 is not None else None,
                bn2.bcoef if bn2 is not None else None, 1.0)
            for b in (bn1, bn2):
                if b is not None:
                    self.grad_ready(b.gslot.index)
                    self.grad_ready(b.bslot.index)
            return
        sums = bn1.bsums[:C * K]
        self.C.bn_slot_sum(slots, C, K, sums)
        self._sync_sum(sums)
        count = count * self.syncbn_world
        # sums layout: k*C + c for k in [sum dz1, sum dz1*x1, (sum dz2, sum dz2*x2)].  The data gradient needs
        # the GLOBAL sums, but dgamma/dbeta must be this rank's share: upstream SyncBN returns the local sums
        # and DDP then averages them, i.e. global / world after averaging.  Writing global / world here gives
        # exactly that after the bucket all-reduce + 1/world (global sums would make them world x too large).
        gs = 1.0 / self.syncbn_world
        self.C.bn_bwd_finalize(sums[:2 * C], float(count), bn1.coef, self._p(bn1.gslot), self._g(bn1.gslot),
                               self._g(bn1.bslot), gs, bn1.bcoef)
        self.grad_ready(bn1.gslot.index)
        self.grad_ready(bn1.bslot.index)
        if bn2 is not None:
            self.C.bn_bwd_finalize(sums[2 * C:4 * C], float(count), bn2.coef, self._p(bn2.gslot), self._g(bn2.gslot),
                                   self._g(bn2.bslot), gs, bn2.bcoef)
            self.grad_ready(bn2.gslot.index)
            self.grad_ready(bn2.bslot.index)

    # ---------------------------------------------------------------------------------- forward
    def _forward(self, images: torch.Tensor, train: bool):
        Cn = self.C
        N = images.shape[0]
        assert images.dim() == 4 and images.shape[1] == 3, "expected NCHW images"
        u8 = images.dtype == torch.uint8  # raw pixels: ImageNet Normalize fused into the stem packing
        x32 = images.contiguous() if u8 or images.dtype == torch.float32 else images.float().contiguous()
        H, W = images.shape[2], images.shape[3]
        st = self.stem
        P0, Q0 = st.out_hw(H, W)
        saved = {"N": N, "H": H, "W": W}
        # stem: zero-padded NHWC4 image + window-mode implicit GEMM with BN statistics (no im2col)
        Hp = max(H + 2 * st.pad, 2 * (P0 - 1) + 2 * self.stem_pairs)
        Wp = max(W + 2 * st.pad, (Q0 - 1) * st.st + 8)
        xp = self._buf("stem_in", N * Hp * Wp * 4)
        if u8:
            Cn.stem_pack_u8(x32, xp, N, 3, H, W, st.pad, Hp, Wp, self.norm_scale, self.norm_shift)
        else:
            Cn.stem_pack(x32, xp, N, 3, H, W, st.pad, Hp, Wp)
        y0 = self._buf("y0", N * P0 * Q0 * st.cout)
        wst = self.derived[self.stem_w_off:self.stem_w_off + st.cout * st.R * 32]
        sp = self._buf(("stats", st.cout), self.n_slots * st.cout * 2, torch.float64) if train else None
        if self.stem_kernel and Cn.stem_fwd_supported(Hp, Wp, P0, Q0):
            Cn.stem_fwd(xp, wst, y0, sp, N, Hp, Wp, P0, Q0, self.stem_blocks_per_cu)
        else:  # generic implicit GEMM in window mode (one 32-wide K step per kernel row)
            bm, bn = self.stem_tile
            Cn.conv_fwd(xp, wst, y0, None, sp, N, Hp, Wp, 32, st.cout, st.R, 1, P0, Q0, st.st, st.st, 0, 0, 1, 0,
                        P0, Q0, 1, 1, 0, 0, bm, bn, 32, 4)
        if train:
            self.bn_train_finalize(self.stem_bn, sp, 0, N * P0 * Q0)
        else:
            self.bn_eval(self.stem_bn)
        H1, W1 = (P0 - 1) // 2 + 1, (Q0 - 1) // 2 + 1
        x = self._buf("act_in", N * H1 * W1 * st.cout)
        idx = self._buf("mp_idx", N * H1 * W1 * st.cout, torch.uint8)
        Cn.bn_relu_maxpool(y0, self.stem_bn.coef, x, idx, N, P0, Q0, st.cout)
        saved.update(xp=xp, Hp=Hp, Wp=Wp, y0=y0, P0=P0, Q0=Q0, idx=idx, x0=x, H1=H1, W1=W1)
        Hc, Wc, Cc = H1, W1, st.cout
        blk_saved = []
        for bi, b in enumerate(self.blocks):
            rec = {"x": x, "H": Hc, "W": Wc, "C": Cc, "ys": [], "as": [], "pre": [], "hw": []}
            cur, h, w = x, Hc, Wc
            nconv = len(b["convs"])
            pre = None  # BN coefficients the current conv applies to its (raw) input itself
            for ci, (c, bn) in enumerate(zip(b["convs"], b["bns"])):
                P, Q = c.out_hw(h, w)
                y = self._buf(("y", bi, ci), N * P * Q * c.cout)
                # SyncBN + downsample block: the last BN's statistics wait for the downsample conv's and share
                # its all-reduce (bn_train_finalize_pair); its partial rows get their own buffer meanwhile
                defer = train and self.syncbn and ci == nconv - 1 and b["ds_conv"] is not None
                _, _, sp, tiles = self.conv_fwd(c, cur, N, h, w, y, train, pre=pre,
                                                stats_tag="deferred" if defer else None,
                                                fin=bn if train and not defer else None)
                if defer:
                    deferred = (bn, sp, N * P * Q)
                elif not train:
                    self.bn_eval(bn)
                rec["ys"].append(y)
                rec["hw"].append((h, w, P, Q))
                if ci < nconv - 1:
                    if self._pre_ok(b["convs"][ci + 1], N, P, Q, train):
                        pre = bn.coef  # consumers apply BN + ReLU to their staged tiles: no bn_apply pass
                        rec["as"].append(y)
                        rec["pre"].append(bn.coef)
                        cur, h, w = y, P, Q
                        continue
                    pre = None
                    a = self._buf(("a", bi, ci), N * P * Q * c.cout)
                    Cn.bn_apply(y, bn.coef, None, None, a, c.cout, 0, True, None)
                    rec["as"].append(a)
                    rec["pre"].append(None)
                    cur, h, w = a, P, Q
                else:
                    h, w = P, Q
            cl, bnl = b["convs"][-1], b["bns"][-1]
            out = self._buf(("out", bi), N * h * w * cl.cout)
            # backward reads the block output's ReLU as a bitmask (1 bit/element instead of 16)
            om = self._buf(("omask", bi), N * h * w * cl.cout // 8, torch.uint8) if train else None
            if b["ds_conv"] is not None:
                dc, dbn = b["ds_conv"], b["ds_bn"]
                yd = self._buf(("yd", bi), N * h * w * dc.cout)
                _, _, sp, tiles = self.conv_fwd(dc, x, N, Hc, Wc, yd, train,
                                                fin=dbn if train and not self.syncbn else None)
                if train and self.syncbn:
                    self.bn_train_finalize_pair(deferred[0], deferred[1], deferred[2], dbn, sp, N * h * w)
                elif not train:
                    self.bn_eval(dbn)
                Cn.bn_apply(rec["ys"][-1], bnl.coef, yd, dbn.coef, out, cl.cout, 2, True, om)
                rec["yd"] = yd
            else:
                Cn.bn_apply(rec["ys"][-1], bnl.coef, x, None, out, cl.cout, 1, True, om)
            rec["out"], rec["omask"] = out, om
            blk_saved.append(rec)
            x, Hc, Wc, Cc = out, h, w, cl.cout
        # head: global average pool -> fc (1x1 GEMM over the padded class dimension)
        HW = Hc * Wc
        feat = self._buf("feat", N * self.feat)
        Cn.avgpool_fwd(x, feat, N, HW, Cc, self.feat)
        logits = self._buf("logits16", N * self.ncls_pad)
        wfc = self.derived[self.fc_w_off:self.fc_w_off + self.ncls_pad * self.feat]
        bm, bn = _conv_tile(self.ncls_pad)
        Cn.conv_fwd(feat, wfc, logits, None, None, N, 1, 1, self.feat, self.ncls_pad, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1,
                    1, 1, 1, 1, 0, 0, bm, bn, 64, 0)
        saved.update(blocks=blk_saved, feat=feat, logits=logits, Hc=Hc, Wc=Wc, Cc=Cc)
        return saved

    def _loss(self, saved, target, dlogits, loss_scale, grad_div):
        N = saved["N"]
        out = torch.empty(N, self.ncls, dtype=torch.float32, device=self.device)
        rl = self._buf("row_loss", N, torch.float32)
        rc = self._buf("row_correct", N, torch.float32)
        self.C.xent(saved["logits"], self.ncls_pad, self._p(self.fcb_slot), target, N, self.ncls, out, dlogits,
                    loss_scale, float(grad_div), rl, rc)
        met = torch.empty(2, dtype=torch.float32, device=self.device)
        self.C.metrics(rl, rc, N, met)
        return out, met

    @torch.no_grad()
    def eval_step(self, images, target):
        saved = self._forward(images, train=False)
        return self._loss(saved, target, None, None, 1.0)

    @torch.no_grad()
    def train_step(self, images, target, loss_scale: Optional[torch.Tensor] = None, grad_div: Optional[float] = None):
        """Forward + loss + backward.  Gradients (scaled by loss_scale / grad_div) land in flat.grad."""
        saved = self._forward(images, train=True)
        N = saved["N"]
        dlog = self._buf("dlogits", N * self.ncls_pad)
        logits, met = self._loss(saved, target, dlog, loss_scale, grad_div or N)
        self._backward(saved, dlog)
        return logits, met

    # ---------------------------------------------------------------------------------- backward
    def _backward(self, saved, dlog):
        Cn = self.C
        N = saved["N"]
        self._wait_derived()  # backward-data weight layouts (gathered on the side stream after the last step)
        # fc: bias grad (column sums), weight grad (1x1 wgrad over the batch), data grad
        Cn.colsum(dlog, N, self.ncls_pad, self.ncls, self._g(self.fcb_slot), 1.0)
        self.grad_ready(self.fcb_slot.index)
        def fc_wg():
            self._wgrad(self.ncls_pad, saved["feat"], dlog, N, 1, 1, self.feat, 1, 1, 1, 1, 1, 0,
                        self._g(self.fc_slot), self.feat, rows=self.ncls, cols=self.feat)
            self.grad_ready(self.fc_slot.index)
        self._side_wgrad((dlog, saved["feat"]), fc_wg)
        dfeat = self._buf("dfeat", N * self.feat)
        wt = self.derived[self.fc_wt_off:self.fc_wt_off + self.ncls_pad * self.feat]
        bm, bn = _conv_tile(self.feat)
        Cn.conv_fwd(dlog, wt, dfeat, None, None, N, 1, 1, self.ncls_pad, self.feat, 1, 1, 1, 1, 1, 1, 0, 0, 1, 1,
                    1, 1, 1, 1, 0, 0, bm, bn, 64, 0)
        Hc, Wc, Cc = saved["Hc"], saved["Wc"], saved["Cc"]
        g = self._buf("g_a", N * Hc * Wc * Cc)
        Cn.avgpool_bwd(dfeat, g, N, Hc * Wc, Cc, self.feat)
        gsel = 0
        g_fused = None  # BN-backward sums of this block's output BN, produced by the previous dgrad epilogue
        for bi in range(len(self.blocks) - 1, -1, -1):
            b, rec = self.blocks[bi], saved["blocks"][bi]
            convs, bns = b["convs"], b["bns"]
            nconv = len(convs)
            h_last, w_last = rec["hw"][-1][2], rec["hw"][-1][3]
            cnt = N * h_last * w_last
            x, Hin, Win, Cin = rec["x"], rec["H"], rec["W"], rec["C"]
            # block-output reduction: BN of the last conv (+ downsample BN) share dz = g * relu'(out)
            ds = b["ds_conv"] is not None
            dsbn = b["ds_bn"] if ds else None
            if g_fused is not None:  # g already holds dz; its BN-backward sums were finalized with that dgrad
                mask_src = None
            else:
                self.bn_bwd(bns[-1], rec["ys"][-1], g, rec["omask"], cnt, dsbn, rec["yd"] if ds else None)
                mask_src = rec["omask"]
            # per-block dY buffers (instead of two shared ones): a shared buffer's next write has
            # to wait for the side-stream weight gradient still reading it, and each such cross-stream
            # wait left the GPU idle ~20-35 us (rocprof trace); per block costs a few GB of HBM, not time
            bk_ = (lambda nm: (nm, bi)) if self.bwd_buf_per_block else (lambda nm: nm)
            dy_last = self._buf(bk_("dy_a"), rec["ys"][-1].numel())
            if ds:
                dyd = self._buf(bk_("dy_b"), rec["yd"].numel())
                Cn.bn_bwd_apply(g, mask_src, rec["ys"][-1], bns[-1].bcoef, dy_last, rec["yd"], dsbn.bcoef,
                                dyd, None, convs[-1].cout)
            elif g_fused is not None:
                dz = g
                Cn.bn_bwd_apply(g, None, rec["ys"][-1], bns[-1].bcoef, dy_last, None, None, None, None,
                                convs[-1].cout)
            else:
                dz = self._buf("dz_id", g.numel())
                Cn.bn_bwd_apply(g, rec["omask"], rec["ys"][-1], bns[-1].bcoef, dy_last, None, None, None, dz,
                                convs[-1].cout)
            # gradient w.r.t. the block input accumulates in g_next
            gnext = self._buf("g_b" if gsel == 0 else "g_a", N * Hin * Win * Cin)
            res_phase = -1
            if ds:
                dc = b["ds_conv"]
                P, Q = dc.out_hw(Hin, Win)
                c0 = convs[0]
                if (self.compact_ds and dc.R == 1 and dc.st == 2 and dc.pad == 0 and c0.st == 2 and c0.R == 3
                        and c0.S == 3 and c0.pad == 1):
                    # the 1x1/2 downsample's data gradient is nonzero only on sub-pixel phase (0, 0), which is
                    # exactly phase 0 of the 3x3/2 conv's dgrad: write it compact and let that phase add it
                    res = self._buf("ds_compact", N * P * Q * Cin)
                    self.conv_bwd(dc, x, N, Hin, Win, dyd, P, Q, res, compact=True)
                    res_phase = 0
                else:
                    self.conv_bwd(dc, x, N, Hin, Win, dyd, P, Q, gnext)  # writes every element of gnext
                    res = gnext
            else:
                res = dz
            # chain through the block's convs in reverse
            dy, dname = dy_last, "dy_a"
            for ci in range(nconv - 1, -1, -1):
                c = convs[ci]
                h, w, P, Q = rec["hw"][ci]
                xin = rec["as"][ci - 1] if ci > 0 else x
                xpre = rec["pre"][ci - 1] if ci > 0 else None
                if ci > 0:
                    # dgrad epilogue applies the ReLU mask (recomputed from the BN input) and reduces the
                    # inner BN's backward sums: da holds dz, no separate reduce pass
                    da = self._buf("da", N * h * w * c.cin)
                    bnp = bns[ci - 1]
                    yp = rec["ys"][ci - 1]
                    slots = self._buf(("bnslots", c.cin, 2), self.n_slots * c.cin * 2, torch.float64)
                    self.conv_bwd(c, xin, N, h, w, dy, P, Q, da, bnb=(1, yp, bnp.coef, None, None, None, slots),
                                  pre=xpre, fin=(N * h * w, bnp, None))
                    dname = "dy_c" if dname == "dy_a" else "dy_a"
                    dyp = self._buf(bk_(dname), yp.numel())
                    Cn.bn_bwd_apply(da, None, yp, bnp.bcoef, dyp, None, None, None, None, c.cin)
                    dy = dyp
                elif bi > 0 and h * w <= self.fuse_block_bn_maxhw:
                    # gnext is the previous block's output gradient: fuse that block's output-BN reduce
                    # (ReLU mask from its output, one or two BN branches) into this dgrad's epilogue
                    pb, prec = self.blocks[bi - 1], saved["blocks"][bi - 1]
                    pds = pb["ds_conv"] is not None
                    K = 4 if pds else 2
                    slots = self._buf(("bnslots", c.cin, K), self.n_slots * c.cin * K, torch.float64)
                    bnb = (3 if pds else 2, prec["ys"][-1], pb["bns"][-1].coef, prec["yd"] if pds else None,
                           pb["ds_bn"].coef if pds else None, prec["omask"], slots)
                    # (that block's BN-backward finalize runs with this launch: conv_bwd fin)
                    self.conv_bwd(c, xin, N, h, w, dy, P, Q, gnext, res=res, bnb=bnb, res_phase=res_phase,
                                  fin=(N * h * w, pb["bns"][-1], pb["ds_bn"] if pds else None))
                    g_fused = slots
                else:
                    self.conv_bwd(c, xin, N, h, w, dy, P, Q, gnext, res=res, res_phase=res_phase)
                    g_fused = None
            g = gnext
            gsel ^= 1
        # stem: fused max-pool backward + ReLU mask + BN backward (two passes, no 112x112 dz tensor)
        # -> window-mode weight gradient
        st, sbn = self.stem, self.stem_bn
        P0, Q0 = saved["P0"], saved["Q0"]
        slots = self._buf(("bnslots", st.cout, 2), self.n_slots * st.cout * 2, torch.float64)
        # BN-backward sums from the pooled output alone (ReLU mask = out > 0, BN input recovered from out)
        Cn.stem_pool_bwd_reduce_out(g, saved["x0"], sbn.coef, slots, N, P0, Q0, st.cout)
        self._bn_bwd_finish(slots, N * P0 * Q0, sbn)
        ldw = self.stem_pairs * 64
        if self._stem_fused_ok(Q0):
            # the stem weight gradient computes its dY tiles itself (max-pool backward + ReLU + BN-backward
            # apply from g / argmax / y0): the 112x112 dY is never written or re-read
            def stem_wg():
                tmp = self._buf("stem_dw", st.cout * ldw, torch.float32)
                key = (st.cout, self.stem_pairs, 1, 64, N * P0 * Q0, True)
                plan = self._plans.get(key)
                if plan is None:
                    plan = tuple(Cn.conv_wgrad_plan(st.cout, self.stem_pairs, 1, 64, N * P0 * Q0, self.wgrad_blocks,
                                                    True))[:2]
                    self._plans[key] = plan
                splits, pps = plan
                ws = self._buf("ws", splits * st.cout * ldw, torch.float32)
                Cn.conv_wgrad_stem_fused(saved["xp"], g, saved["idx"], saved["y0"], sbn.coef, sbn.bcoef, ws, N,
                                         saved["Hp"], saved["Wp"], self.stem_pairs, P0, Q0, st.st, 2, ldw, splits, pps)
                Cn.wgrad_reduce(ws, splits, st.cout, ldw, ldw, st.cout * ldw, tmp, ldw, 1.0, False)
                Cn.gather32(tmp, self.stem_gidx, self._g(st.slot))
                self.grad_ready(st.pid)
            # (round 5: on the compute stream instead, beside the side stream's last layer1 weight gradients, measured
            # 20.57 -> 20.74 ms/step, same box)
            self._side_wgrad((g, saved["xp"], saved["idx"], saved["y0"], sbn.coef, sbn.bcoef), stem_wg)
        else:
            dy0 = self._buf("dy0", N * P0 * Q0 * st.cout)
            Cn.stem_pool_bwd_apply(g, saved["idx"], saved["y0"], sbn.coef, sbn.bcoef, dy0, N, P0, Q0, st.cout)

            def stem_wg():
                tmp = self._buf("stem_dw", st.cout * ldw, torch.float32)
                self._wgrad(st.cout, saved["xp"], dy0, N, saved["Hp"], saved["Wp"], 64, self.stem_pairs, 1, P0, Q0,
                            st.st, 0, tmp, ldw, cs=4, win=True, dil=2)
                Cn.gather32(tmp, self.stem_gidx, self._g(st.slot))
                self.grad_ready(st.pid)
            self._side_wgrad((dy0, saved["xp"]), stem_wg)
        self._join_side()
