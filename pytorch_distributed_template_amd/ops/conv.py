"""Functional NHWC convolution ops over the native implicit-GEMM kernels.

Tensors are NHWC 16-bit activations (``[N, H, W, C]`` contiguous) and KRSC weights
(``[Cout, kh, kw, Cin]`` contiguous, i.e. a ``channels_last`` PyTorch conv weight's storage).

* :func:`conv_fwd`    forward conv (optionally with BatchNorm partial statistics)
* :func:`conv_dgrad`  gradient w.r.t. the input, one launch per sub-pixel phase of the stride
* :func:`conv_wgrad`  gradient w.r.t. the weight (fp32), split-K over pixels

These wrappers allocate their outputs; the ResNet executor calls the same kernels on preallocated
buffers.  They are the unit-test surface of the kernels (tests/test_kernels_gpu.py).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import native


# shortest reduction that goes to the ping-pong kernel: tools/conv_bench.py --r50 (forward + BN statistics) measured
# it ahead of the 128x128 kernel from two K-steps on (ResNet-50 1x1 convs 128->512: 278 vs 251 TF/s, 256->1024:
# 452 vs 392; the round-1 table used 512)
_PP_MIN_K = 128


# a 256 x 128 tile needs this many tiles (two workgroups per CU: 512 resident) to beat the 128 x 128 one; below it
# the larger tile leaves CUs idle (e.g. ResNet-18 layer4 at 150 images/GPU)
_WIDE128_MIN_TILES = 1024


def conv_tile(cout: int, kdim: int = 0, m: int = 0) -> Tuple[int, int]:
    """(BM, BN) tile of the implicit-GEMM kernel for a given GEMM-N (output channels), GEMM-K (reduction length
    ``Cin*R*S``; 0 = unknown) and GEMM-M (output pixels; 0 = unknown).

    Long reductions over >= 256 channels go to the 8-wave ping-pong kernel (256x256, one workgroup per
    CU, counted-vmcnt DMA pipeline: +10-25 % over the 2-stage 128x128 kernel on ResNet layer3/4 shapes,
    tools/conv_bench.py); short ones (1x1 convs: 1-4 K-steps) stay on the 2-stage kernel, whose
    prologue/epilogue is cheaper.  128-channel GEMMs with enough pixels take the 256x128 3-stage tile (4 waves of
    the ping-pong wave tile, 2 workgroups per CU; conv_fwd.hip launch_tile)."""
    if cout % 256 == 0 and kdim >= _PP_MIN_K and kdim % 64 == 0:
        return 256, 256
    if cout % 128 == 0:
        if m and (m + 255) // 256 * (cout // 128) >= _WIDE128_MIN_TILES:
            return 256, 128
        return 128, 128
    return 256, 64


def dgrad_phases(R: int, S: int, stride: int, pad: int) -> List[Tuple[int, int, List[int], List[int], int, int]]:
    """Sub-pixel decomposition of a strided conv's backward-data pass.

    For output phase (ph, pw) of dX (rows h = stride*i + ph), only taps r = r0 + stride*t contribute,
    with dY row ``i + ioff_h - t``.  Returns ``(ph, pw, rs, ss, ioff_h, ioff_w)`` per phase; ``rs``/``ss``
    are the contributing tap indices (possibly empty: e.g. odd phases of a 1x1 stride-2 conv).
    """
    out = []
    for ph in range(stride):
        for pw in range(stride):
            r0, s0 = (ph + pad) % stride, (pw + pad) % stride
            rs = list(range(r0, R, stride))
            ss = list(range(s0, S, stride))
            out.append((ph, pw, rs, ss, (ph + pad - r0) // stride, (pw + pad - s0) // stride))
    return out


def dgrad_weight_index(cout: int, cin: int, R: int, S: int, rs: List[int], ss: List[int]) -> torch.Tensor:
    """Index map (into a KRSC weight) of the phase weight ``Wt[c][t][u][k] = W[k][rs[t]][ss[u]][c]``."""
    if not rs or not ss:
        return torch.empty(0, dtype=torch.long)
    c = torch.arange(cin).view(-1, 1, 1, 1)
    t = torch.tensor(rs).view(1, -1, 1, 1)
    u = torch.tensor(ss).view(1, 1, -1, 1)
    k = torch.arange(cout).view(1, 1, 1, -1)
    return (((k * R + t) * S + u) * cin + c).reshape(-1)


def out_hw(H: int, W: int, R: int, S: int, stride: int, pad: int) -> Tuple[int, int]:
    return (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1


def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride: int = 1, pad: int = 0, stats: bool = False,
             residual: Optional[torch.Tensor] = None, tile: Optional[Tuple[int, int, int]] = None):
    """y = conv(x, w) in NHWC/KRSC.  Returns ``y`` or ``(y, (sum, sumsq) per channel)`` with stats.
    ``tile`` = (BM, BN, BK) overrides the per-shape table (tests / sweeps)."""
    N, H, W, C = x.shape
    K, R, S, C2 = w.shape
    assert C == C2
    P, Q = out_hw(H, W, R, S, stride, pad)
    y = torch.empty(N, P, Q, K, dtype=x.dtype, device=x.device)
    bm, bn = conv_tile(K, C * R * S, N * P * Q)
    bk = 64 if C % 64 == 0 else 32
    if tile is not None:
        bm, bn, bk = tile
    sp = None
    if stats:
        sp = torch.empty(native.C.stat_slots() * K * 2, dtype=torch.float64, device=x.device)
    native.C.conv_fwd(x, w, y, residual, sp, N, H, W, C, K, R, S, P, Q, stride, stride, -pad, -pad, 1, 1,
                      P, Q, 1, 1, 0, 0, bm, bn, bk, 0)
    if not stats:
        return y
    sums = torch.empty(2 * K, dtype=torch.float64, device=x.device)
    native.C.bn_slot_sum(sp, K, 2, sums)
    return y, (sums[:K], sums[K:])


def pack_relu_mask(out: torch.Tensor) -> torch.Tensor:
    """ReLU bitmask of a 16-bit activation: bit e of byte v is ``out.flatten()[8v + e] > 0`` (the layout
    ``bn_apply(..., mask)`` writes and the backward kernels read)."""
    bits = (out.reshape(-1, 8) > 0).to(torch.int32)
    w = (1 << torch.arange(8, device=out.device, dtype=torch.int32))
    return (bits * w).sum(1).to(torch.uint8)


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, H: int, W: int, stride: int = 1, pad: int = 0,
               residual: Optional[torch.Tensor] = None, bnb: Optional[tuple] = None,
               tile: Optional[Tuple[int, int, int]] = None, res_phase: int = -1) -> torch.Tensor:
    """dX (NHWC, [N, H, W, Cin]) of ``y = conv(x, w)`` given dY ([N, P, Q, Cout]).

    ``bnb = (mode, y1, coef1, y2, coef2, out_mask, slots)`` fuses the consuming BatchNorm's backward
    reduce into the epilogue (the result is then dz = dX * relu'; sums land in ``slots``); ``out_mask`` is
    the block output's ReLU bitmask (:func:`pack_relu_mask`, modes 2/3).  ``res_phase >= 0``: ``residual`` is
    compact ([N, ceil(H/stride), ceil(W/stride), Cin]) and added on that sub-pixel phase only (index into the
    phases kept for this launch), e.g. a 1x1/2 downsample's data gradient added to a 3x3/2 one."""
    N, P, Q, K = dy.shape
    K2, R, S, C = w.shape
    assert K == K2
    dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
    bm, bn = conv_tile(C, K * R * S, N * H * W)
    bk = 64 if K % 64 == 0 else 32
    if tile is not None:
        bm, bn, bk = tile
    wflat = w.reshape(-1)
    pieces, phases, off = [], [], 0
    for ph, pw, rs, ss, ioff_h, ioff_w in dgrad_phases(R, S, stride, pad):
        if H - ph <= 0 or W - pw <= 0:
            continue
        idx = dgrad_weight_index(K, C, R, S, rs, ss).to(w.device)
        if idx.numel():
            pieces.append(wflat[idx])
        phases.append([ph, pw, len(rs), len(ss), ioff_h, ioff_w, off])
        off += idx.numel()
    wt = torch.cat(pieces).contiguous() if pieces else torch.zeros(1, dtype=w.dtype, device=w.device)
    if bnb is None and res_phase < 0:
        native.C.conv_dgrad(dy, wt, dx, residual, N, P, Q, K, C, H, W, stride, phases, bm, bn, bk)
    else:
        native.C.conv_dgrad_bn(dy, wt, dx, residual, N, P, Q, K, C, H, W, stride, phases, bm, bn, bk,
                               *(bnb or (0, None, None, None, None, None, None)), res_phase)
    return dx


def conv_wgrad(x: torch.Tensor, dy: torch.Tensor, R: int, S: int, stride: int = 1, pad: int = 0,
               target_blocks: int = 2048) -> torch.Tensor:
    """dW (fp32, KRSC [Cout, R, S, Cin]) of ``y = conv(x, w)``."""
    N, H, W, C = x.shape
    _, P, Q, K = dy.shape
    splits, pps, _ = native.C.conv_wgrad_plan(K, R, S, C, N * P * Q, target_blocks, False)
    ldw = R * S * C
    ws = torch.empty(splits * K * ldw, dtype=torch.float32, device=x.device)
    native.C.conv_wgrad(x, dy, ws, N, H, W, C, K, R, S, P, Q, stride, stride, pad, pad, 1, 1, ldw, splits, pps, 0,
                        False)
    out = torch.empty(K * ldw, dtype=torch.float32, device=x.device)
    native.C.wgrad_reduce(ws, splits, K, ldw, ldw, K * ldw, out, ldw, 1.0, False)
    return out.view(K, R, S, C)
