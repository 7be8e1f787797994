"""Native fp32 ResNet executor: the reference's own precision on our HIP kernels.

`distributed.py` and `dataparallel.py` train in plain fp32 (no autocast, `distributed.py:245-263`,
`dataparallel.py:211-222`) and every script validates in fp32 (`distributed_syncBN_amp.py:311-317`).  This
executor runs that precision end to end on the fp32 kernels of ``csrc/kernels/fp32.hip`` -- conv forward /
multi-phase backward-data / weight gradient on ``v_mfma_f32_16x16x4f32``, BatchNorm statistics through the
deterministic per-block rows, BN apply / backward, stem BN+ReLU+max-pool, average pool, cross-entropy -- with
fp32 activations and weights read straight from the fp32 master buffer (no 16-bit shadow).

Structure mirrors :class:`~.executor.ResNetExecutor` (torchvision-layout Basic / Bottleneck ResNets, flat
gradient buffer, per-parameter ``grad_ready`` for the DDP bucketer, SyncBN through the same fp64 statistic
all-reduce) without its 16-bit-specific fusions: BN-backward reductions are separate passes and the stem runs
as an im2col GEMM (K = 7*7*3 padded to 192), processed in image chunks so every operand stays within the
32-bit buffer offsets of the LDS-DMA loads.

Accuracy (measured in round 4 against an fp64 forward, ResNet-50): the forward activations track an fp64 forward exactly as closely as
PyTorch's own fp32 does (relative error 2e-7 after the stem, 7e-5 at the last block, both), and conv weight
gradients of the later layers match fp64 to ~5e-6.  Where a gradient differs more it is a discrete effect of
fp32 rounding itself -- a near-zero pre-activation landing on the other side of a ReLU than in fp64 -- which
tests/test_fp32_gpu.py judges against the fp64 gradients' own sensitivity to an input nudge of that size.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import torch

from ..ops import native
from .executor import ResNetExecutor, _BN, _Conv
from .resnet import BasicBlock, ResNet

STEM_K = 192  # im2col width of the 7x7x3 stem (147 columns, zero padded to a multiple of 64)


def fp32_supported(model) -> bool:
    """Models this executor runs: torchvision-layout ResNets, Wide-ResNets and ResNeXts (grouped convs as 64-channel
    slices, as the 16-bit executor)."""
    return isinstance(model, ResNet)


class ResNetExecutor32(ResNetExecutor):
    """fp32 counterpart of :class:`ResNetExecutor` (same public interface)."""

    def __init__(self, model: ResNet, flat, device: torch.device,
                 grad_ready: Optional[Callable[[int], None]] = None, syncbn_group=None,
                 syncbn_allreduce: Optional[Callable[[torch.Tensor], None]] = None, syncbn_world: int = 0,
                 wgrad_blocks: int = 2048):
        if not fp32_supported(model):
            raise NotImplementedError("native fp32 executor supports torchvision-style ResNets / ResNeXts")
        self.C = native.C
        self.n_slots = self.C.stat_slots()
        self.model = model
        self.flat = flat
        self.device = torch.device(device)
        self.dtype = torch.float32
        self._user_grad_ready = grad_ready or (lambda pid: None)
        self.side = None  # one stream: every kernel here is MFMA- or bandwidth-bound on its own
        self._on_side = False
        self._pending_reads = {}
        self.syncbn_group = syncbn_group
        self.syncbn = syncbn_allreduce is not None or syncbn_group is not None
        # the inherited bn_train_finalize / _pair use the forward-statistics hook when one is set; this executor
        # issues every SyncBN all-reduce through _sync_sum
        self._sync_sum_fwd = None
        if syncbn_allreduce is not None:
            self.syncbn_world = int(syncbn_world) if syncbn_world else 1
            self._sync_sum = syncbn_allreduce
        elif syncbn_group is not None:
            import torch.distributed as dist
            self.syncbn_world = dist.get_world_size(syncbn_group)
            self._sync_sum = lambda t: dist.all_reduce(t, group=syncbn_group)
        self.wgrad_blocks = wgrad_blocks
        from ..data.transforms import IMAGENET_MEAN, IMAGENET_STD
        self.mean = torch.tensor(IMAGENET_MEAN, device=self.device).view(1, 3, 1, 1)
        self.std = torch.tensor(IMAGENET_STD, device=self.device).view(1, 3, 1, 1)
        derived_maps: List[torch.Tensor] = []
        off = [0]
        gfwd_maps: list = []  # forward layouts of the grouped convs' 64-channel slices

        def conv(c):
            return _Conv(c, flat, derived_maps, off, gfwd_maps)

        st = model.conv1
        assert st.in_channels * st.kernel_size[0] * st.kernel_size[1] <= STEM_K, "stem too wide for the im2col GEMM"
        self.stem = conv(st)
        self.stem_bn = _BN(model.bn1, flat, self.device)
        self.blocks = []
        for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
            for blk in layer:
                kind = "basic" if isinstance(blk, BasicBlock) else "bottleneck"
                convs = [blk.conv1, blk.conv2] + ([blk.conv3] if kind == "bottleneck" else [])
                bns = [blk.bn1, blk.bn2] + ([blk.bn3] if kind == "bottleneck" else [])
                d = {"kind": kind, "convs": [conv(c) for c in convs], "bns": [_BN(b, flat, self.device) for b in bns],
                     "ds_conv": conv(blk.downsample[0]) if blk.downsample is not None else None,
                     "ds_bn": _BN(blk.downsample[1], flat, self.device) if blk.downsample is not None else None}
                self.blocks.append(d)
        for gc, j, gm in gfwd_maps:  # (one gather refreshes every layout: their order is free)
            gc.gfwd.append(off[0])
            derived_maps.append(gm)
            off[0] += gm.numel()
        # stem weight as a [64][STEM_K] GEMM operand (KRSC flattening == im2col column order), zero padded
        s = self.stem
        kk = s.R * s.S * s.cin
        o = torch.arange(s.cout).view(-1, 1)
        k = torch.arange(STEM_K).view(1, -1)
        m = torch.where(k < kk, s.slot.offset + o * kk + k, torch.full_like(o * k, -1))
        self.stem_w_off = off[0]
        derived_maps.append(m.reshape(-1).to(torch.int32))
        off[0] += m.numel()
        # window-mode stem (default; PDT_FP32_STEM_WIN=0: the im2col GEMM): [64][R][32] over the zero-padded NHWC4 image, column s * 4 + c of kernel
        # row r (s = 7 and c = 3 zero) -- no im2col buffer in the forward pass
        self.stem_win = os.environ.get("PDT_FP32_STEM_WIN", "1") == "1" and s.S <= 7 and s.cin <= 3
        if self.stem_win:
            r = torch.arange(s.R).view(1, -1, 1)
            j = torch.arange(32).view(1, 1, -1)
            o3 = torch.arange(s.cout).view(-1, 1, 1)
            sj, cj = j // 4, j % 4
            mw = torch.where((sj < s.S) & (cj < s.cin), s.slot.offset + ((o3 * s.R + r) * s.S + sj) * s.cin + cj,
                             torch.full_like(o3 * r * j, -1))
            self.stem_win_off = off[0]
            derived_maps.append(mw.reshape(-1).to(torch.int32))
            off[0] += mw.numel()
            # its weight gradient comes out as [64][kernel-row pair t][row 2t: 8 px x 4 ch | row 2t+1: same] (wgrad32_stem)
            self.stem_pairs = (s.R + 1) // 2
            kk_, rr, ss, cc = torch.meshgrid(torch.arange(s.cout), torch.arange(s.R), torch.arange(s.S),
                                             torch.arange(s.cin), indexing="ij")
            self.stem_gidx_win = (kk_ * (self.stem_pairs * 64) + (rr // 2) * 64 + (rr % 2) * 32 + ss * 4 + cc).reshape(
                -1).to(torch.int32).to(self.device)
        # stem weight gradient: [64][STEM_K] GEMM result -> KRSC slot
        self.stem_gidx = (torch.arange(s.cout).view(-1, 1) * STEM_K + torch.arange(kk).view(1, -1)).reshape(-1).to(
            torch.int32).to(self.device)
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
        self.derived_idx = torch.cat([x.to(torch.int32) for x in derived_maps]).to(self.device)
        self.derived = torch.zeros(off[0], dtype=torch.float32, device=self.device)
        for b in self.blocks:
            for c in b["convs"]:
                if c.groups > 1:
                    c.gidx = c.gidx.to(self.device)
        self._bufs = {}
        self._plans = {}
        self._tiles = {}
        self.update_derived()

    # ------------------------------------------------------------------------------------------ helpers
    def update_derived(self) -> None:
        """Derived fp32 weight layouts (dgrad phase weights, padded stem / fc matrices) from the master."""
        self.C.gather32(self.flat.data, self.derived_idx, self.derived)

    def _wait_derived(self) -> None:
        pass

    def _w32(self, c: _Conv) -> torch.Tensor:
        s = c.slot
        return self.flat.data[s.offset:s.offset + s.numel]

    @staticmethod
    def _bn_tile(n: int) -> int:
        return 128 if n % 128 == 0 else 64

    _WIDE = True
    # 64-channel GEMMs (layer1, the stem): rows per tile (128: 4 waves of 64x32; round-3 sweep over 128 / 256 / 512)
    _BM64 = 128

    def _tile32(self, n: int, m: int):
        """(BM, BN) of the fp32 implicit GEMM: 8-wave 256-row tiles (256x256 / 256x128, twice / 1.3x the FLOP per
        staged byte of 128x128) when the GEMM has enough rows to fill the chip, else the 4-wave 128-row tiles.
        (Round 3: the 128-row-only table measured slower.)"""
        if self._WIDE and m >= 256 * 256:
            if n % 256 == 0:
                return 256, 256
            if n % 128 == 0:
                return 256, 128
            if n == 64 and self._BM64 in (256, 512):
                return self._BM64, 64
        return 128, self._bn_tile(n)

    # shipped per-conv fp32 tiles (models/tuned_tiles32_mi355x.json; PDT_FP32_TUNED=0 ignores them)
    from .tuned import ARITY32, TABLE32, load_table
    _TUNED32 = load_table(TABLE32, ARITY32) if os.environ.get("PDT_FP32_TUNED", "1") == "1" else {}

    def _tile32c(self, kind: str, c: _Conv, N: int, H: int, n: int, m: int):
        return self._TUNED32.get((kind, N, H, c.cin, c.cout, c.R, c.st)) or self._tile32(n, m)

    # Grouped convs (ResNeXt) in fp32: the 16-bit executor's 64-channel slices with block-diagonal weights (_Conv
    # _init_grouped), each slice gathered into a dense [pixels][64] operand and run on the dense fp32 kernels; outputs,
    # statistics columns and the weight gradient's diagonal blocks are scattered back.  (The reference precision path:
    # MIOpen's fp16 grouped conv ran this model at 1239 ms per step, so even the gather copies are far ahead.)
    def _slice(self, key, t, rows: int, width: int, j: int):
        """Dense copy of channel slice j of a [rows][width] tensor."""
        s = self._buf(key, rows * self._GS, torch.float32)
        s.view(rows, self._GS).copy_(t.view(rows, width)[:, j * self._GS:(j + 1) * self._GS])
        return s

    _GS = _Conv.GSLICE

    def _gconv_fwd32(self, c: _Conv, x, N, H, W, y, stats: bool):
        P, Q, S_ = *c.out_hw(H, W), self._GS
        sp = self._buf(("stats", c.cout), self.n_slots * c.cout * 2, torch.float64) if stats else None
        ys = self._buf("g32_y", N * P * Q * S_, torch.float32)
        sps = self._buf("g32_st", self.n_slots * S_ * 2, torch.float64) if stats else None
        n = S_ * c.R * c.S * S_
        tile = self._tile32(S_, N * P * Q)
        for j in range(c.nslice):
            xs = self._slice("g32_x", x, N * H * W, c.cin, j)
            self.C.conv32_fwd(xs, self.derived[c.gfwd[j]:c.gfwd[j] + n], ys, None, sps, N, H, W, S_, S_, c.R, c.S, P,
                              Q, c.st, c.pad, *tile)
            y.view(N * P * Q, c.cout)[:, j * S_:(j + 1) * S_].copy_(ys.view(-1, S_))
            if stats:
                sp.view(self.n_slots, c.cout, 2)[:, j * S_:(j + 1) * S_].copy_(sps.view(self.n_slots, S_, 2))
        return P, Q, sp

    def _gdgrad32(self, c: _Conv, dy, N, H, W, P, Q, dx):
        S_ = self._GS
        dxs = self._buf("g32_dx", N * H * W * S_, torch.float32)
        tile = self._tile32(S_, N * P * Q)
        for j in range(c.nslice):
            dys = self._slice("g32_dy", dy, N * P * Q, c.cout, j)
            phases = [p for p in c.gphases[j] if H - p[0] > 0 and W - p[1] > 0]
            self.C.conv32_dgrad(dys, self.derived, dxs, None, N, P, Q, S_, S_, H, W, c.st, phases, *tile)
            dx.view(N * H * W, c.cin)[:, j * S_:(j + 1) * S_].copy_(dxs.view(-1, S_))

    def _gwgrad32(self, c: _Conv, x, dy, N, H, W, P, Q):
        S_ = self._GS
        ldw = c.R * c.S * S_
        tmp = self._buf("g32_dw", c.nslice * S_ * ldw, torch.float32)
        for j in range(c.nslice):
            xs = self._slice("g32_x", x, N * H * W, c.cin, j)
            dys = self._slice("g32_dy", dy, N * P * Q, c.cout, j)
            self._wgrad(S_, xs, dys, N, H, W, S_, c.R, c.S, P, Q, c.st, c.pad, tmp[j * S_ * ldw:(j + 1) * S_ * ldw], ldw)
        self.C.gather32(tmp, c.gidx, self._g(c.slot))  # the diagonal blocks = the grouped weight gradient

    def _conv_fwd(self, c: _Conv, x, N, H, W, y, stats: bool):
        if c.groups > 1:
            return self._gconv_fwd32(c, x, N, H, W, y, stats)
        P, Q = c.out_hw(H, W)
        sp = self._buf(("stats", c.cout), self.n_slots * c.cout * 2, torch.float64) if stats else None
        tile = self._tile32c("fwd", c, N, H, c.cout, N * P * Q)
        self.C.conv32_fwd(x, self._w32(c), y, None, sp, N, H, W, c.cin, c.cout, c.R, c.S, P, Q, c.st, c.pad, *tile)
        return P, Q, sp

    # (the inner BatchNorms' BN + ReLU applied inside the consumer conv's fp32 kernels -- round 4's PDT_FP32_PRE --
    # measured 126.1 -> 129.7 ms/step, the fused kernels 14-21 % slower than the 1.2 ms of bn_apply32 passes they
    # remove, and was deleted in round 5; profiles/r4_fp32_pre.md)

    def _dgrad(self, c: _Conv, dy, N, H, W, P, Q, dx, res=None, bnb=None):
        """``bnb = (mref, y1, coef, slots)``: the consumer BatchNorm's backward reduce fused into the epilogue (dx then
        holds dz = dx * (mref > 0) and the slots receive sum dz, sum dz * xhat -- no separate bn_bwd_reduce32 pass)."""
        # every sub-pixel phase of the stride in one launch; a phase without taps (odd phases of a 1x1/2 conv)
        # runs zero K-steps and writes zeros (+ the residual)
        phases = [[ph, pw, T, U, ioff_h, ioff_w, doff] for (ph, pw, T, U, ioff_h, ioff_w, doff, dn) in c.phases
                  if H - ph > 0 and W - pw > 0]
        self.C.conv32_dgrad(dy, self.derived, dx, res, N, P, Q, c.cout, c.cin, H, W, c.st, phases,
                            *self._tile32c("dgrad", c, N, H, c.cin, N * P * Q), *(bnb or ()))

    _FUSE_BN = os.environ.get("PDT_FP32_FUSE_BN", "1") == "1"

    _HALO = True
    # stem backward tail: max-pool backward + ReLU mask recomputed inside the BN-backward reduce and apply (no dz
    # tensor); PDT_FP32_STEM_FUSE=0: maxpool_bwd_relu32 + bn_bwd_reduce32 + bn_bwd_apply32 over a stored dz
    _FUSE_STEM = os.environ.get("PDT_FP32_STEM_FUSE", "1") == "1"
    # stem weight gradient: every kernel-row pair per block (dY staged once, not once per pair); 0: one block per pair
    _STEM4 = True
    # ... and its dY computed inside that kernel from the pooled gradient, argmax, conv output and BN coefficients (the
    # apply pass and the fp32 dY tensor disappear); PDT_FP32_STEM_WG_FUSE=0: stem_pool_bwd_apply32 + the plain kernel
    _STEM_WG_FUSE = os.environ.get("PDT_FP32_STEM_WG_FUSE", "1") == "1"
    # stem BN-backward sums over the pooled output (mask out > 0, BN input recovered from out) instead of the window
    # gather over the 112x112 conv output; PDT_FP32_STEM_REDUCE_OUT=0: stem_pool_bwd_reduce32
    _STEM_REDUCE_OUT = os.environ.get("PDT_FP32_STEM_REDUCE_OUT", "1") == "1"

    def _wgrad_tile(self, cout, R, S, C, H, W, P, Q, st, pad) -> int:
        # 3x3 / s1 / p1 over 64-channel blocks with wide rows (layer1): the halo kernel, all three taps of a kernel
        # row per block (48 FLOP per staged byte); else 128 x 128 / 8-wave tiles when both channel counts allow
        # (32 FLOP/B), else 64 x 64 (16 FLOP/B)
        if (self._HALO and R == 3 and S == 3 and st == 1 and pad == 1 and P == H and Q == W and 28 <= Q <= 62
                and C == 64 and cout % 64 == 0):
            return 3
        return 128 if (self._WIDE and C % 128 == 0 and cout % 128 == 0) else 64

    def _wgrad(self, cout, x, dy, N, H, W, C, R, S, P, Q, st, pad, gout, ldo, rows=None, cols=None,
               accumulate=False):
        ldw = R * S * C
        npix = N * P * Q
        tile = self._wgrad_tile(cout, R, S, C, H, W, P, Q, st, pad)
        key = (cout, R, S, C, npix, tile)
        plan = self._plans.get(key)
        if plan is None:
            if tile == 3:  # splits over the N * P output rows; 3 kernel rows x channel blocks per split
                per_split = 3 * (cout // 64) * (C // 64)
                splits = max(1, min(1024 // per_split, N * P))
                pps = (N * P + splits - 1) // splits
                splits = (N * P + pps - 1) // pps
            else:
                per_split = (cout // tile) * R * S * (C // tile)
                target = self.wgrad_blocks if tile == 64 else self.wgrad_blocks // 2  # 2 wide blocks per CU
                splits = max(1, min(target // max(per_split, 1), (npix + 63) // 64))
                pps = ((npix + splits - 1) // splits + 63) // 64 * 64
                splits = (npix + pps - 1) // pps
            plan = self._plans[key] = (splits, pps)
        splits, pps = plan
        ws = self._buf("ws", splits * cout * ldw, torch.float32)
        self.C.wgrad32(x, dy, ws, N, H, W, C, cout, R, S, P, Q, st, pad, ldw, splits, pps, tile)
        self.C.wgrad_reduce(ws, splits, rows or cout, cols or ldw, ldw, cout * ldw, gout, ldo, 1.0, accumulate)

    def _stem_chunk(self, N: int) -> int:
        # im2col rows of one chunk stay < 2^30 fp32 elements (32-bit LDS-DMA offsets)
        P0, Q0 = self.stem.out_hw(self._HW[0], self._HW[1])
        return max(1, min(N, ((1 << 30) - 1) // (P0 * Q0 * STEM_K)))

    def bn_reduce(self, bn1: _BN, g, mref, y1, count, bn2: Optional[_BN] = None, y2=None):
        C = bn1.C
        rows = g.numel() // C
        K = 4 if bn2 is not None else 2
        slots = self._buf(("bnslots", C, K), self.n_slots * C * K, torch.float64)
        blocks = self.C.bn_bwd_reduce32_blocks(rows, C)
        self.C.bn_bwd_reduce32(g, mref, y1, bn1.coef, y2, bn2.coef if bn2 is not None else None, slots, blocks, rows,
                               C)
        self._bn_bwd_finish(slots, count, bn1, bn2)

    # ------------------------------------------------------------------------------------------ forward
    def _forward(self, images: torch.Tensor, train: bool):
        Cn = self.C
        N, _, H, W = images.shape
        if images.dtype == torch.uint8:  # raw pixels: ImageNet normalisation on the device
            x32 = ((images.float() / 255.0 - self.mean) / self.std).contiguous()
        else:
            x32 = images.float().contiguous()
        self._HW = (H, W)
        st = self.stem
        P0, Q0 = st.out_hw(H, W)
        y0 = self._buf("y0", N * P0 * Q0 * st.cout, torch.float32)
        wst = self.derived[self.stem_w_off:self.stem_w_off + st.cout * STEM_K]
        ch = self._stem_chunk(N)
        sp = None
        if train:
            sp = self._buf(("stats", st.cout), self.n_slots * st.cout * 2, torch.float64)
            sp.zero_()
        if self.stem_win:
            Hp = max(H + 2 * st.pad, (P0 - 1) * st.st + 2 * ((st.R + 1) // 2))  # + the pair-mode row R (weight 0)
            Wp = max(W + 2 * st.pad, (Q0 - 1) * st.st + 8)
            xp = self._buf("stem_in", N * Hp * Wp * 4, torch.float32)
            Cn.stem_pack32(x32, xp, N, 3, H, W, st.pad, Hp, Wp)
            self._stem_xp = (xp, Hp, Wp)
            wwin = self.derived[self.stem_win_off:self.stem_win_off + st.cout * st.R * 32]
            Cn.conv32_stem_fwd(xp, wwin, y0, sp, N, Hp, Wp, st.R, P0, Q0, st.st, st.cout,
                               *self._tile32(st.cout, N * P0 * Q0))
            ch = N + 1  # no im2col chunks
        for n0 in range(0, N if not self.stem_win else 0, ch):
            n1 = min(N, n0 + ch)
            cols = self._buf("stem_cols", (n1 - n0) * P0 * Q0 * STEM_K, torch.float32)
            Cn.im2col32(x32[n0:n1], cols, n1 - n0, 3, H, W, st.R, st.S, st.st, st.pad, STEM_K)
            spc = self._buf("stats_chunk", self.n_slots * st.cout * 2, torch.float64) if train else None
            Cn.conv32_fwd(cols, wst, y0[n0 * P0 * Q0 * st.cout:n1 * P0 * Q0 * st.cout], None, spc,
                          (n1 - n0) * P0 * Q0, 1, 1, STEM_K, st.cout, 1, 1, 1, 1, 1, 0,
                          *self._tile32(st.cout, (n1 - n0) * P0 * Q0))
            if train:
                sp.add_(spc)  # chunks in a fixed order: deterministic
        if train:
            self.bn_train_finalize(self.stem_bn, sp, 0, N * P0 * Q0)
        else:
            self.bn_eval(self.stem_bn)
        H1, W1 = (P0 - 1) // 2 + 1, (Q0 - 1) // 2 + 1
        x = self._buf("act_in", N * H1 * W1 * st.cout, torch.float32)
        idx = self._buf("mp_idx", N * H1 * W1 * st.cout, torch.uint8)
        Cn.bn_relu_maxpool32(y0, self.stem_bn.coef, x, idx, N, P0, Q0, st.cout)
        saved = {"N": N, "H": H, "W": W, "x32": x32, "y0": y0, "P0": P0, "Q0": Q0, "idx": idx, "x0": x, "H1": H1,
                 "W1": W1}
        if self.stem_win:
            saved["xp"], saved["Hp"], saved["Wp"] = self._stem_xp
        Hc, Wc, Cc = H1, W1, st.cout
        recs = []
        for bi, b in enumerate(self.blocks):
            rec = {"x": x, "H": Hc, "W": Wc, "C": Cc, "ys": [], "as": [], "hw": []}
            cur, h, w = x, Hc, Wc
            for ci, (c, bn) in enumerate(zip(b["convs"], b["bns"])):
                P, Q = c.out_hw(h, w)
                y = self._buf(("y", bi, ci), N * P * Q * c.cout, torch.float32)
                _, _, sp = self._conv_fwd(c, cur, N, h, w, y, train)
                if train:
                    self.bn_train_finalize(bn, sp, 0, N * P * Q)
                else:
                    self.bn_eval(bn)
                rec["ys"].append(y)
                rec["hw"].append((h, w, P, Q))
                if ci < len(b["convs"]) - 1:
                    a = self._buf(("a", bi, ci), y.numel(), torch.float32)
                    Cn.bn_apply32(y, bn.coef, None, None, a, c.cout, 0, True)
                    rec["as"].append(a)
                    cur = a
                h, w = P, Q
            cl, bnl = b["convs"][-1], b["bns"][-1]
            out = self._buf(("out", bi), N * h * w * cl.cout, torch.float32)
            if b["ds_conv"] is not None:
                dc, dbn = b["ds_conv"], b["ds_bn"]
                yd = self._buf(("yd", bi), N * h * w * dc.cout, torch.float32)
                _, _, sp = self._conv_fwd(dc, x, N, Hc, Wc, yd, train)
                if train:
                    self.bn_train_finalize(dbn, sp, 0, N * h * w)
                else:
                    self.bn_eval(dbn)
                Cn.bn_apply32(rec["ys"][-1], bnl.coef, yd, dbn.coef, out, cl.cout, 2, True)
                rec["yd"] = yd
            else:
                Cn.bn_apply32(rec["ys"][-1], bnl.coef, x, None, out, cl.cout, 1, True)
            rec["out"] = out
            recs.append(rec)
            x, Hc, Wc, Cc = out, h, w, cl.cout
        feat = self._buf("feat", N * self.feat, torch.float32)
        Cn.avgpool32_fwd(x, feat, N, Hc * Wc, Cc, self.feat)
        logits = self._buf("logits32", N * self.ncls_pad, torch.float32)
        wfc = self.derived[self.fc_w_off:self.fc_w_off + self.ncls_pad * self.feat]
        Cn.conv32_fwd(feat, wfc, logits, None, None, N, 1, 1, self.feat, self.ncls_pad, 1, 1, 1, 1, 1, 0, 128, 128)
        saved.update(blocks=recs, feat=feat, logits=logits, Hc=Hc, Wc=Wc, Cc=Cc)
        return saved

    def _loss(self, saved, target, dlogits, loss_scale, grad_div):
        N = saved["N"]
        out = torch.empty(N, self.ncls, dtype=torch.float32, device=self.device)
        rl = self._buf("row_loss", N, torch.float32)
        rc = self._buf("row_correct", N, torch.float32)
        self.C.xent32(saved["logits"], self.ncls_pad, self._p(self.fcb_slot), target, N, self.ncls, out, dlogits,
                      loss_scale, float(grad_div), rl, rc)
        met = torch.empty(2, dtype=torch.float32, device=self.device)
        self.C.metrics(rl, rc, N, met)
        return out, met

    @torch.no_grad()
    def train_step(self, images, target, loss_scale: Optional[torch.Tensor] = None, grad_div: Optional[float] = None):
        saved = self._forward(images, train=True)
        N = saved["N"]
        dlog = self._buf("dlogits32", N * self.ncls_pad, torch.float32)
        logits, met = self._loss(saved, target, dlog, loss_scale, grad_div or N)
        self._backward(saved, dlog)
        return logits, met

    # ------------------------------------------------------------------------------------------ backward
    def _backward(self, saved, dlog):
        Cn = self.C
        N = saved["N"]
        Cn.colsum32(dlog, N, self.ncls_pad, self.ncls, self._g(self.fcb_slot), 1.0)
        self.grad_ready(self.fcb_slot.index)
        self._wgrad(self.ncls_pad, saved["feat"], dlog, N, 1, 1, self.feat, 1, 1, 1, 1, 1, 0, self._g(self.fc_slot),
                    self.feat, rows=self.ncls, cols=self.feat)
        self.grad_ready(self.fc_slot.index)
        dfeat = self._buf("dfeat", N * self.feat, torch.float32)
        wt = self.derived[self.fc_wt_off:self.fc_wt_off + self.ncls_pad * self.feat]
        Cn.conv32_fwd(dlog, wt, dfeat, None, None, N, 1, 1, self.ncls_pad, self.feat, 1, 1, 1, 1, 1, 0, 128,
                      self._bn_tile(self.feat))
        Hc, Wc, Cc = saved["Hc"], saved["Wc"], saved["Cc"]
        g = self._buf("g_a", N * Hc * Wc * Cc, torch.float32)
        Cn.avgpool32_bwd(dfeat, g, N, Hc * Wc, Cc, self.feat)
        gsel = 0
        g_fused = None  # this block's output-BN backward sums, reduced by the previous backward-data epilogue
        for bi in range(len(self.blocks) - 1, -1, -1):
            b, rec = self.blocks[bi], saved["blocks"][bi]
            convs, bns = b["convs"], b["bns"]
            h_last, w_last = rec["hw"][-1][2], rec["hw"][-1][3]
            x, Hin, Win, Cin = rec["x"], rec["H"], rec["W"], rec["C"]
            ds = b["ds_conv"] is not None
            dsbn = b["ds_bn"] if ds else None
            # block output: dz = g * relu'(out); BN backward of the last BN (+ the downsample BN sharing dz)
            if g_fused is not None:  # g already holds dz
                self._bn_bwd_finish(g_fused, N * h_last * w_last, bns[-1], dsbn)
                mref = None
            else:
                self.bn_reduce(bns[-1], g, rec["out"], rec["ys"][-1], N * h_last * w_last, dsbn,
                               rec["yd"] if ds else None)
                mref = rec["out"]
            dy = self._buf(("dy", 0), rec["ys"][-1].numel(), torch.float32)
            gnext = self._buf("g_b" if gsel == 0 else "g_a", N * Hin * Win * Cin, torch.float32)
            if ds:
                dyd = self._buf("dyd", rec["yd"].numel(), torch.float32)
                Cn.bn_bwd_apply32(g, mref, rec["ys"][-1], bns[-1].bcoef, dy, rec["yd"], dsbn.bcoef, dyd, None,
                                  convs[-1].cout)
                dc = b["ds_conv"]
                P, Q = dc.out_hw(Hin, Win)
                self._wgrad(dc.cout, x, dyd, N, Hin, Win, Cin, dc.R, dc.S, P, Q, dc.st, dc.pad, self._g(dc.slot),
                            dc.R * dc.S * Cin)
                self.grad_ready(dc.pid)
                self._dgrad(dc, dyd, N, Hin, Win, P, Q, gnext)
                res = gnext
            elif mref is None:  # g is dz already: it is the identity branch's gradient too
                Cn.bn_bwd_apply32(g, None, rec["ys"][-1], bns[-1].bcoef, dy, None, None, None, None, convs[-1].cout)
                res = g
            else:
                dz = self._buf("dz_id", g.numel(), torch.float32)
                Cn.bn_bwd_apply32(g, rec["out"], rec["ys"][-1], bns[-1].bcoef, dy, None, None, None, dz,
                                  convs[-1].cout)
                res = dz
            for ci in range(len(convs) - 1, -1, -1):
                c = convs[ci]
                h, w, P, Q = rec["hw"][ci]
                xin = rec["as"][ci - 1] if ci > 0 else x
                if c.groups > 1:
                    self._gwgrad32(c, xin, dy, N, h, w, P, Q)
                else:
                    self._wgrad(c.cout, xin, dy, N, h, w, c.cin, c.R, c.S, P, Q, c.st, c.pad, self._g(c.slot),
                                c.R * c.S * c.cin)
                self.grad_ready(c.pid)
                if ci > 0:
                    da = self._buf("da", N * h * w * c.cin, torch.float32)
                    bnp, yp, ap = bns[ci - 1], rec["ys"][ci - 1], rec["as"][ci - 1]
                    if c.groups > 1:  # grouped (a block-internal conv): slice dgrads, then the separate BN reduce
                        self._gdgrad32(c, dy, N, h, w, P, Q, da)
                        self.bn_reduce(bnp, da, ap, yp, N * h * w)
                        mref = ap
                    elif self._FUSE_BN:  # dgrad epilogue writes dz and reduces the inner BN's backward sums (ReLU
                        # mask from ap)
                        slots = self._buf(("bnslots", c.cin, 2), self.n_slots * c.cin * 2, torch.float64)
                        self._dgrad(c, dy, N, h, w, P, Q, da, bnb=(ap, yp, bnp.coef, slots))
                        self._bn_bwd_finish(slots, N * h * w, bnp)
                        mref = None
                    else:
                        self._dgrad(c, dy, N, h, w, P, Q, da)
                        self.bn_reduce(bnp, da, ap, yp, N * h * w)
                        mref = ap
                    dyp = self._buf(("dy", (len(convs) - ci) % 2 + 1), yp.numel(), torch.float32)
                    Cn.bn_bwd_apply32(da, mref, yp, bnp.bcoef, dyp, None, None, None, None, c.cin)
                    dy = dyp
                elif self._FUSE_BN and bi > 0:
                    # gnext is the previous block's output gradient: reduce that block's output-BN backward sums
                    # (ReLU mask from its output, one or two BN branches) in this dgrad's epilogue
                    pb, prec = self.blocks[bi - 1], saved["blocks"][bi - 1]
                    pds = pb["ds_conv"] is not None
                    K = 4 if pds else 2
                    slots = self._buf(("bnslots", c.cin, K), self.n_slots * c.cin * K, torch.float64)
                    bnb = (prec["out"], prec["ys"][-1], pb["bns"][-1].coef, slots) + (
                        (prec["yd"], pb["ds_bn"].coef) if pds else ())
                    self._dgrad(c, dy, N, h, w, P, Q, gnext, res=res, bnb=bnb)
                    g_fused = slots
                else:
                    self._dgrad(c, dy, N, h, w, P, Q, gnext, res=res)
                    g_fused = None
            g = gnext
            gsel ^= 1
        # stem: max-pool backward + ReLU mask (from the BN input) -> BN backward -> im2col weight gradient
        st, sbn = self.stem, self.stem_bn
        P0, Q0, H, W = saved["P0"], saved["Q0"], saved["H"], saved["W"]
        dz0 = None
        if self._FUSE_STEM:  # dz recomputed by the reduce and the apply: never stored
            rows = N * P0 * Q0
            slots = self._buf(("bnslots", st.cout, 2), self.n_slots * st.cout * 2, torch.float64)
            if self._STEM_REDUCE_OUT:
                prow = saved["x0"].numel() // st.cout
                Cn.stem_pool_bwd_reduce_out32(g, saved["x0"], sbn.coef, slots, max(1, min(2048, prow // 64)), st.cout)
            else:
                # 4x the blocks of a plain reduce: the per-pixel window gather is latency-bound, not a stream
                blocks = max(1, min(4096, rows // 256))
                Cn.stem_pool_bwd_reduce32(g, saved["idx"], saved["y0"], sbn.coef, slots, blocks, N, P0, Q0, st.cout)
            self._bn_bwd_finish(slots, rows, sbn, None)
            wg_fused = (self.stem_win and self._STEM4 and self._STEM_WG_FUSE and self.stem_pairs == 4
                        and st.cout == 64)
            if not wg_fused:  # (fused: no 3.85 GB dY buffer at ResNet-18 B = 1200)
                dy0 = dz0 = self._buf("dz0", saved["y0"].numel(), torch.float32)
                Cn.stem_pool_bwd_apply32(g, saved["idx"], saved["y0"], sbn.coef, sbn.bcoef, dy0, N, P0, Q0, st.cout)
        else:
            wg_fused = False
            dz0 = self._buf("dz0", saved["y0"].numel(), torch.float32)
            Cn.maxpool_bwd_relu32(g, saved["idx"], saved["y0"], sbn.coef, dz0, N, P0, Q0, st.cout)
            self.bn_reduce(sbn, dz0, None, saved["y0"], N * P0 * Q0)
            dy0 = dz0  # in place: each element read then written by the same thread
            Cn.bn_bwd_apply32(dz0, None, saved["y0"], sbn.bcoef, dy0, None, None, None, None, st.cout)
        if self.stem_win:  # window-pair weight gradient straight from the padded NHWC4 image (no im2col)
            npix = N * P0 * Q0
            key = ("stem_win", npix)
            plan = self._plans.get(key)
            if plan is None:
                per_split = (st.cout // 64) * self.stem_pairs
                splits = max(1, min(self.wgrad_blocks // per_split, (npix + 63) // 64))
                pps = ((npix + splits - 1) // splits + 63) // 64 * 64
                plan = self._plans[key] = ((npix + pps - 1) // pps, pps)
            splits, pps = plan
            ldw = self.stem_pairs * 64
            ws = self._buf("ws", splits * st.cout * ldw, torch.float32)
            if wg_fused:
                Cn.wgrad32_stem_fused(saved["xp"], g, saved["idx"], saved["y0"], sbn.coef, sbn.bcoef, ws, N,
                                      saved["Hp"], saved["Wp"], P0, Q0, st.st, splits, pps)
            else:
                Cn.wgrad32_stem(saved["xp"], dy0, ws, N, saved["Hp"], saved["Wp"], self.stem_pairs, st.cout, P0, Q0,
                                st.st, splits, pps, 1 if (self._STEM4 and self.stem_pairs == 4) else 0)
            tmp = self._buf("stem_dw", st.cout * ldw, torch.float32)
            Cn.wgrad_reduce(ws, splits, st.cout, ldw, ldw, st.cout * ldw, tmp, ldw, 1.0, False)
            Cn.gather32(tmp, self.stem_gidx_win, self._g(st.slot))
            self.grad_ready(st.pid)
            return
        tmp = self._buf("stem_dw", st.cout * STEM_K, torch.float32)
        ch = self._stem_chunk(N)
        for i, n0 in enumerate(range(0, N, ch)):
            n1 = min(N, n0 + ch)
            cols = self._buf("stem_cols", (n1 - n0) * P0 * Q0 * STEM_K, torch.float32)
            Cn.im2col32(saved["x32"][n0:n1], cols, n1 - n0, 3, H, W, st.R, st.S, st.st, st.pad, STEM_K)
            npix = (n1 - n0) * P0 * Q0
            self._wgrad(st.cout, cols, dy0[n0 * P0 * Q0 * st.cout:n1 * P0 * Q0 * st.cout], npix, 1, 1, STEM_K, 1, 1,
                        1, 1, 1, 0, tmp, STEM_K, accumulate=i > 0)
        Cn.gather32(tmp, self.stem_gidx, self._g(st.slot))
        self.grad_ready(st.pid)
