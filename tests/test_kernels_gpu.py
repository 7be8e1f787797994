"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references (run on an MI355X)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _rand16(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


CONV_CASES = [
    # N, H, W, C, K, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 15, 13, 64, 128, 3, 2, 1),
    (3, 14, 14, 128, 256, 1, 2, 0),
    (2, 7, 7, 256, 64, 1, 1, 0),
    (2, 12, 12, 64, 256, 1, 1, 0),  # one K-step forward (single-buffer variant)
    (3, 14, 14, 64, 128, 1, 2, 0),  # one K-step strided 1x1
    (1, 9, 9, 128, 128, 3, 1, 1),
    (2, 8, 8, 512, 512, 3, 1, 1),
    (2, 8, 56, 64, 64, 3, 1, 1),   # ResNet layer1 geometry -> halo-reuse kernel (conv_l1.hip)
    (2, 9, 56, 64, 64, 3, 1, 1),   # layer1 geometry with H % 4 != 0 -> generic kernel (conv_l1 takes whole row tiles)
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_fwd_and_stats(case, dtype):
    from pytorch_distributed_template_amd.ops import conv
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(0)
    x = _rand16(N, H, W, C, dtype=dtype)
    w = _rand16(K, R, R, C, dtype=dtype, scale=(1.0 / (C * R * R)) ** 0.5)
    y, (s, ss) = conv.conv_fwd(x, w, st, pad, stats=True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=st, padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, K)
    assert torch.allclose(s.float(), yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(ss.float(), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(case):
    from pytorch_distributed_template_amd.ops import conv
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(1)
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    dy = _rand16(N, P, Q, K)
    w = _rand16(K, R, R, C, scale=(1.0 / (K * R * R)) ** 0.5)
    res = _rand16(N, H, W, C)
    dx = conv.conv_dgrad(dy, w, H, W, st, pad, residual=res)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     stride=st, padding=pad).permute(0, 2, 3, 1) + res.float()
    assert _rel(dx, ref) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_wgrad(case, dtype):
    from pytorch_distributed_template_amd.ops import conv
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(2)
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    x = _rand16(N, H, W, C, dtype=dtype)
    dy = _rand16(N, P, Q, K, dtype=dtype)
    dw = conv.conv_wgrad(x, dy, R, R, st, pad, target_blocks=64)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, R), dy.float().permute(0, 3, 1, 2),
                                      stride=st, padding=pad).permute(0, 2, 3, 1)
    assert _rel(dw, ref) < 2e-3


@pytest.mark.parametrize("case", [(2, 15, 13, 64, 256, 3, 2, 1), (4, 14, 14, 64, 128, 3, 1, 1),
                                  (3, 14, 14, 64, 128, 1, 2, 0), (2, 9, 9, 64, 384, 1, 1, 0),
                                  (2, 28, 28, 64, 128, 3, 2, 1), (3, 6, 6, 64, 128, 3, 2, 1)])
@pytest.mark.parametrize("target", [64, 2048])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_wgrad_two_tap_pair_tile(case, target, dtype):
    """C == 64, Kout % 128 == 0 runs the 128x128 wgrad kernel with its c side split over two taps (an odd tap count
    leaves the last tile's second half dead): every tap's dW against torch fp32, few and many splits."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K, R, st, pad = case
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    assert native.C.conv_wgrad_plan(K, R, R, C, N * P * Q, target, False)[2] == 128
    torch.manual_seed(12)
    x = _rand16(N, H, W, C, dtype=dtype)
    dy = _rand16(N, P, Q, K, dtype=dtype)
    dw = conv.conv_wgrad(x, dy, R, R, st, pad, target_blocks=target)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, R), dy.float().permute(0, 3, 1, 2),
                                      stride=st, padding=pad).permute(0, 2, 3, 1)
    for t in range(R * R):  # per tap: a dead or misplaced half shows up as one tap's block
        assert _rel(dw.reshape(K, R * R, C)[:, t], ref.reshape(K, R * R, C)[:, t]) < 2e-3, t


@pytest.mark.parametrize("case", [(2, 14, 14, 128, 128, 3, 1, 1), (2, 15, 13, 128, 256, 3, 2, 1),
                                  (3, 9, 9, 256, 128, 1, 1, 0), (2, 10, 10, 128, 128, 1, 2, 0),
                                  (1, 7, 7, 384, 128, 3, 1, 1), (2, 28, 28, 128, 128, 3, 1, 1),
                                  (3, 6, 6, 128, 128, 3, 2, 1)])
@pytest.mark.parametrize("target", [64, 2048])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_wgrad_wide_tile(case, target, dtype):
    """C % 128 == 0 and Kout % 128 == 0 below 256 x 256: the wide 256 (two 128-wide column blocks of dW) x 128 kernel
    with its 3-deep counted-wait DMA ring.  Every column block against torch fp32 (an odd block count leaves the last
    tile's second half dead), few and many splits (a split of one K-step drains the ring at once); image and row
    wraps inside a K-step (7 x 7, 5 x 5 outputs) and a 3-wide output (the 128 x 128 fallback)."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K, R, st, pad = case
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    assert native.C.conv_wgrad_plan(K, R, R, C, N * P * Q, target, False)[2] == 2  # kWgradWide
    torch.manual_seed(14)
    x = _rand16(N, H, W, C, dtype=dtype)
    dy = _rand16(N, P, Q, K, dtype=dtype)
    dw = conv.conv_wgrad(x, dy, R, R, st, pad, target_blocks=target)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, R), dy.float().permute(0, 3, 1, 2),
                                      stride=st, padding=pad).permute(0, 2, 3, 1)
    nb = R * R * C // 128
    for b in range(nb):
        assert _rel(dw.reshape(K, nb, 128)[:, b], ref.reshape(K, nb, 128)[:, b]) < 2e-3, b


def test_conv_wgrad_many_splits():
    from pytorch_distributed_template_amd.ops import conv
    torch.manual_seed(3)
    x = _rand16(16, 28, 28, 64)
    dy = _rand16(16, 28, 28, 64)
    dw = conv.conv_wgrad(x, dy, 3, 3, 1, 1, target_blocks=4096)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      stride=1, padding=1).permute(0, 2, 3, 1)
    assert _rel(dw, ref) < 2e-3


def test_sgd_matches_torch():
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(4)
    n = 10007
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    buf = torch.zeros(n, device=DEV)
    sh = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ref_p = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([ref_p], lr=0.1, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        ref_p.grad = g * 0.5
        opt.step()
        native.C.sgd(p, g, buf, sh, None, 0.1, 0.9, 1e-4, 0.5, None, None, step == 0)
    assert torch.allclose(p, ref_p.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(sh, p.to(torch.bfloat16))


def test_sgd_skips_on_inf():
    from pytorch_distributed_template_amd.ops import native
    p = torch.ones(100, device=DEV)
    g = torch.ones(100, device=DEV)
    g[7] = float("inf")
    found = torch.zeros(1, device=DEV)
    native.C.nonfinite_check(g, found)
    assert found.item() == 1.0
    buf = torch.zeros(100, device=DEV)
    native.C.sgd(p, g, buf, None, None, 0.1, 0.9, 0.0, 1.0, None, found, True)
    assert torch.equal(p, torch.ones(100, device=DEV))


def test_xent_matches_torch():
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(5)
    B, ncls, ld = 37, 1000, 1024
    logits = torch.zeros(B, ld, device=DEV, dtype=torch.bfloat16)
    logits[:, :ncls] = (torch.randn(B, ncls, device=DEV) * 3).to(torch.bfloat16)
    bias = torch.randn(ncls, device=DEV) * 0.1
    tgt = torch.randint(0, ncls, (B,), device=DEV)
    out = torch.empty(B, ncls, device=DEV)
    d = torch.empty(B, ld, device=DEV, dtype=torch.bfloat16)
    rl = torch.empty(B, device=DEV)
    rc = torch.empty(B, device=DEV)
    scale = torch.full((1,), 8.0, device=DEV)
    native.C.xent(logits, ld, bias, tgt, B, ncls, out, d, scale, float(B), rl, rc)
    met = torch.empty(2, device=DEV)
    native.C.metrics(rl, rc, B, met)
    ref_in = (logits[:, :ncls].float() + bias).requires_grad_(True)
    loss = F.cross_entropy(ref_in, tgt)
    loss.backward()
    assert torch.allclose(out, ref_in.detach(), atol=1e-5)
    assert abs(met[0].item() - loss.item()) < 1e-4
    acc = (ref_in.detach().argmax(1) == tgt).float().mean().item()
    assert abs(met[1].item() - acc) < 1e-6
    assert _rel(d[:, :ncls], ref_in.grad * 8.0) < 1e-2
    assert d[:, ncls:].abs().max().item() == 0


@pytest.mark.parametrize("pad,N,H,W,C", [(1, 2, 12, 11, 64), (0, 2, 13, 11, 64), (0, 3, 27, 27, 192),
                                         (0, 2, 55, 55, 64)])
def test_bn_relu_maxpool_and_backward(pad, N, H, W, C):
    """MaxPool(3, 2, pad) over relu(a*y + b), forward with argmax and the gather-form backward with the ReLU mask,
    against torch: pad 1 is the ResNet stem's, pad 0 AlexNet's (27 -> 13, 55 -> 27 and an odd width)."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(6)
    y = _rand16(N, H, W, C)
    # mixed-sign BN scales: the kernel pools the raw input (sign-flipped where the scale is negative)
    sign = torch.where(torch.rand(C, device=DEV) < 0.5, -1.0, 1.0)
    coef = torch.cat([(torch.rand(C, device=DEV) + 0.5) * sign, torch.randn(C, device=DEV) * 0.1,
                      torch.zeros(2 * C, device=DEV)])
    OH, OW = (H + 2 * pad - 3) // 2 + 1, (W + 2 * pad - 3) // 2 + 1
    out = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=DEV)
    idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=DEV)
    native.C.bn_relu_maxpool(y, coef, out, idx, N, H, W, C, pad=pad)
    a = torch.relu(y.float() * coef[:C] + coef[C:2 * C]).permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(a, 3, 2, pad)
    assert _rel(out.permute(0, 3, 1, 2), ref) < 1e-2
    # windows whose maximum is the ReLU's zero carry the dead argmax 255 (no gradient); the others a window position
    dead = out.float() == 0
    assert dead.any() and (~dead).any()
    assert torch.equal(idx == 255, dead) and bool((idx[~dead] < 9).all())
    dp = _rand16(N, OH, OW, C)
    ref.backward(dp.float().permute(0, 3, 1, 2))
    dz = torch.empty_like(y)
    native.C.maxpool_bwd_relu(dp, idx, y, coef, dz, N, H, W, C, pad=pad)
    refdz = a.grad * (a.detach() > 0)
    assert _rel(dz.permute(0, 3, 1, 2), refdz) < 1e-2


def test_stem_window_mode_fwd_and_wgrad():
    """7x7/2 pad-3 stem via the zero-padded NHWC4 image (no im2col) vs F.conv2d / conv2d_weight."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(7)
    N, H, W, K = 2, 30, 26, 64
    x = torch.randn(N, 3, H, W, device=DEV)
    w = torch.randn(K, 3, 7, 7, device=DEV) * 0.05
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = max(H + 6, 2 * (P - 1) + 8), max(W + 6, 2 * (Q - 1) + 8)
    xp = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device=DEV)
    native.C.stem_pack(x, xp, N, 3, H, W, 3, Hp, Wp)
    wk = w.permute(0, 2, 3, 1)  # K, r, s, c
    wwin = torch.zeros(K, 7, 8, 4, device=DEV)
    wwin[:, :, :7, :3] = wk
    wwin = wwin.reshape(K, 7 * 32).to(torch.bfloat16).contiguous()
    y = torch.empty(N * P * Q * K, dtype=torch.bfloat16, device=DEV)
    native.C.conv_fwd(xp, wwin, y, None, None, N, Hp, Wp, 32, K, 7, 1, P, Q, 2, 2, 0, 0, 1, 0, P, Q, 1, 1, 0, 0,
                      256, 64, 32, 4)
    xr = x.to(torch.bfloat16).float()
    ref = F.conv2d(xr, wk.to(torch.bfloat16).float().permute(0, 3, 1, 2), stride=2, padding=3)
    assert _rel(y.view(N, P, Q, K).permute(0, 3, 1, 2), ref) < 1e-2
    # window-pair mode: one 64-wide K step covers kernel rows (2p, 2p+1); 4 steps with BK=64
    wpair = torch.zeros(K, 8, 8, 4, device=DEV)
    wpair[:, :7, :7, :3] = wk
    wpair = wpair.reshape(K, 4 * 64).to(torch.bfloat16).contiguous()
    for bm, bn in ((256, 64), (128, 64)):
        y2 = torch.empty_like(y)
        native.C.conv_fwd(xp, wpair, y2, None, None, N, Hp, Wp, 64, K, 4, 1, P, Q, 2, 2, 0, 0, 2, 0, P, Q, 1, 1, 0, 0,
                          bm, bn, 64, 4)
        assert _rel(y2.view(N, P, Q, K).permute(0, 3, 1, 2), ref) < 1e-2
        # dedicated persistent stem kernel (register-fed B fragments, resident weights) with BN stats
        ys = torch.empty_like(y)
        stats = torch.zeros(native.C.stat_slots() * K * 2, dtype=torch.float64, device=DEV)
        native.C.stem_fwd(xp, wwin, ys, stats, N, Hp, Wp, P, Q, 2)
        assert _rel(ys.view(N, P, Q, K).permute(0, 3, 1, 2), ref) < 1e-2
        st = stats.view(-1, K, 2).sum(0)
        yf = ys.view(-1, K).float()
        assert torch.allclose(st[:, 0].float(), yf.sum(0), rtol=1e-4, atol=1e-2)
        assert torch.allclose(st[:, 1].float(), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)
    # weight gradient in window mode, then the KRSC scatter
    dy = _rand16(N, P, Q, K)
    pairs = 4
    splits, pps, _ = native.C.conv_wgrad_plan(K, pairs, 1, 64, N * P * Q, 64, True)
    ws = torch.empty(splits * K * pairs * 64, device=DEV)
    native.C.conv_wgrad(xp, dy, ws, N, Hp, Wp, 64, K, pairs, 1, P, Q, 2, 2, 0, 0, 2, 2, pairs * 64, splits, pps, 4, True)
    tmp = torch.empty(K * pairs * 64, device=DEV)
    native.C.wgrad_reduce(ws, splits, K, pairs * 64, pairs * 64, K * pairs * 64, tmp, pairs * 64, 1.0, False)
    kk = torch.arange(K).view(-1, 1, 1, 1)
    rr = torch.arange(7).view(1, -1, 1, 1)
    ss = torch.arange(7).view(1, 1, -1, 1)
    cc = torch.arange(3).view(1, 1, 1, -1)
    gidx = (kk * (pairs * 64) + (rr // 2) * 64 + (rr % 2) * 32 + ss * 4 + cc).reshape(-1).to(torch.int32).to(DEV)
    dw = torch.empty(K * 7 * 7 * 3, device=DEV)
    native.C.gather32(tmp, gidx, dw)
    refw = torch.nn.grad.conv2d_weight(xr, (K, 3, 7, 7), dy.float().permute(0, 3, 1, 2), stride=2, padding=3)
    assert _rel(dw.view(K, 7, 7, 3).permute(0, 3, 1, 2), refw) < 2e-3


def test_stem_pool_backward_fused():
    """Fused max-pool bwd + ReLU + BN bwd (reduce pass over argmax elements, apply pass) vs autograd fp32."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(8)
    N, H, W, C = 3, 14, 13, 64
    y = _rand16(N, H, W, C)
    yf = y.float()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.2
    mean = yf.mean((0, 1, 2))
    var = yf.var((0, 1, 2), unbiased=False)
    invstd = torch.rsqrt(var + 1e-5)
    scale = gamma * invstd
    coef = torch.cat([scale, beta - mean * scale, mean, invstd]).contiguous()
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=DEV)
    idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=DEV)
    native.C.bn_relu_maxpool(y, coef, out, idx, N, H, W, C)
    dp = _rand16(N, OH, OW, C)
    # reference: BN (batch stats) -> ReLU -> maxpool in fp32 autograd
    xin = yf.permute(0, 3, 1, 2).clone().requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    z = F.batch_norm(xin, None, None, g_, b_, training=True, eps=1e-5)
    F.max_pool2d(torch.relu(z), 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    slots = torch.zeros(native.C.stat_slots() * C * 2, dtype=torch.float64, device=DEV)
    native.C.stem_pool_bwd_reduce(dp, idx, y, coef, slots, N, H, W, C)
    sums = torch.empty(2 * C, dtype=torch.float64, device=DEV)
    native.C.bn_slot_sum(slots, C, 2, sums)
    dgamma = torch.empty(C, device=DEV)
    dbeta = torch.empty(C, device=DEV)
    bcoef = torch.empty(3 * C, device=DEV)
    native.C.bn_bwd_finalize(sums, float(N * H * W), coef, gamma, dgamma, dbeta, 1.0, bcoef)
    assert _rel(dgamma, g_.grad) < 1e-2 and _rel(dbeta, b_.grad) < 1e-2
    # the same sums from the pooled output alone
    slots2 = torch.zeros_like(slots)
    native.C.stem_pool_bwd_reduce_out(dp, out, coef, slots2, N, H, W, C)
    sums2 = torch.empty(2 * C, dtype=torch.float64, device=DEV)
    native.C.bn_slot_sum(slots2, C, 2, sums2)
    assert torch.allclose(sums2[:C], sums[:C], rtol=1e-4, atol=1e-3)
    assert torch.allclose(sums2[C:], sums[C:], rtol=2e-2, atol=2e-2)
    dy = torch.empty_like(y)
    native.C.stem_pool_bwd_apply(dp, idx, y, coef, bcoef, dy, N, H, W, C)
    assert _rel(dy.permute(0, 3, 1, 2), xin.grad) < 2e-2


@pytest.mark.parametrize("geom", [(2, 29, 28), (3, 28, 36), (2, 64, 64), (2, 224, 224)])
def test_stem_wgrad_fused_dy(geom):
    """Stem weight gradient with dY computed in-kernel (max-pool bwd + ReLU + BN-bwd apply) vs the two-pass
    path (stem_pool_bwd_apply -> window-mode conv_wgrad) and vs an fp32 autograd reference.  The second
    geometry has an even conv-output height and a pooled width whose last window column is out of range
    for the last pixel pair (boundary windows), both have a partial last K-step; those two run the 2x2-quad kernel,
    the 64 and 224 px ones (conv output a multiple of 4 x 16) the raw-image-row kernel."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(9)
    N, H, W = geom
    K = C = 64
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = max(H + 6, 2 * (P - 1) + 8), max(W + 6, 2 * (Q - 1) + 8)
    x = torch.randn(N, 3, H, W, device=DEV)
    xp = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device=DEV)
    native.C.stem_pack(x, xp, N, 3, H, W, 3, Hp, Wp)
    y = _rand16(N, P, Q, C)  # stands in for the stem conv output
    yf = y.float()
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.2
    mean = yf.mean((0, 1, 2))
    invstd = torch.rsqrt(yf.var((0, 1, 2), unbiased=False) + 1e-5)
    scale = gamma * invstd
    coef = torch.cat([scale, beta - mean * scale, mean, invstd]).contiguous()
    OH, OW = (P - 1) // 2 + 1, (Q - 1) // 2 + 1
    out = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=DEV)
    idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=DEV)
    native.C.bn_relu_maxpool(y, coef, out, idx, N, P, Q, C)
    dp = _rand16(N, OH, OW, C)
    slots = torch.zeros(native.C.stat_slots() * C * 2, dtype=torch.float64, device=DEV)
    native.C.stem_pool_bwd_reduce_out(dp, out, coef, slots, N, P, Q, C)
    sums = torch.empty(2 * C, dtype=torch.float64, device=DEV)
    native.C.bn_slot_sum(slots, C, 2, sums)
    dgamma, dbeta, bcoef = torch.empty(C, device=DEV), torch.empty(C, device=DEV), torch.empty(3 * C, device=DEV)
    native.C.bn_bwd_finalize(sums, float(N * P * Q), coef, gamma, dgamma, dbeta, 1.0, bcoef)
    pairs, ldw = 4, 256
    splits, pps, _ = native.C.conv_wgrad_plan(K, pairs, 1, 64, N * P * Q, 64, True)
    # two-pass path
    dy = torch.empty_like(y)
    native.C.stem_pool_bwd_apply(dp, idx, y, coef, bcoef, dy, N, P, Q, C)
    ws = torch.empty(splits * K * ldw, device=DEV)
    native.C.conv_wgrad(xp, dy, ws, N, Hp, Wp, 64, K, pairs, 1, P, Q, 2, 2, 0, 0, 2, 2, ldw, splits, pps, 4, True)
    t1 = torch.empty(K * ldw, device=DEV)
    native.C.wgrad_reduce(ws, splits, K, ldw, ldw, K * ldw, t1, ldw, 1.0, False)
    # fused path
    ws2 = torch.full_like(ws, float("nan"))
    native.C.conv_wgrad_stem_fused(xp, dp, idx, y, coef, bcoef, ws2, N, Hp, Wp, pairs, P, Q, 2, 2, ldw, splits, pps)
    t2 = torch.empty(K * ldw, device=DEV)
    native.C.wgrad_reduce(ws2, splits, K, ldw, ldw, K * ldw, t2, ldw, 1.0, False)
    torch.cuda.synchronize()
    assert torch.isfinite(t2).all()
    assert _rel(t2, t1) < 2e-3
    # fp32 reference: autograd through BN -> ReLU -> max-pool gives dY, conv2d_weight gives dW
    xin = yf.permute(0, 3, 1, 2).clone().requires_grad_(True)
    z = F.batch_norm(xin, None, None, gamma, beta, training=True, eps=1e-5)
    F.max_pool2d(torch.relu(z), 3, 2, 1).backward(dp.float().permute(0, 3, 1, 2))
    xr = x.to(torch.bfloat16).float()
    refw = torch.nn.grad.conv2d_weight(xr, (K, 3, 7, 7), xin.grad, stride=2, padding=3)
    kk = torch.arange(K).view(-1, 1, 1, 1)
    rr = torch.arange(7).view(1, -1, 1, 1)
    ss = torch.arange(7).view(1, 1, -1, 1)
    cc = torch.arange(3).view(1, 1, 1, -1)
    gidx = (kk * ldw + (rr // 2) * 64 + (rr % 2) * 32 + ss * 4 + cc).reshape(-1).to(torch.int32).to(DEV)
    dw = torch.empty(K * 7 * 7 * 3, device=DEV)
    native.C.gather32(t2, gidx, dw)
    assert _rel(dw.view(K, 7, 7, 3).permute(0, 3, 1, 2), refw) < 3e-2


def test_stem_kernel_persistent_tiles():
    """Stem kernel with more tiles than blocks (persistent loop + next-tile prefetch) vs F.conv2d."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(9)
    N, H, W, K = 24, 112, 112, 64
    x = torch.randn(N, 3, H, W, device=DEV)
    w = torch.randn(K, 3, 7, 7, device=DEV) * 0.05
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = max(H + 6, 2 * (P - 1) + 8), max(W + 6, 2 * (Q - 1) + 8)
    xp = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device=DEV)
    native.C.stem_pack(x, xp, N, 3, H, W, 3, Hp, Wp)
    wk = w.permute(0, 2, 3, 1)
    wwin = torch.zeros(K, 7, 8, 4, device=DEV)
    wwin[:, :, :7, :3] = wk
    wwin = wwin.reshape(K, 7 * 32).to(torch.bfloat16).contiguous()
    ys = torch.empty(N * P * Q * K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(native.C.stat_slots() * K * 2, dtype=torch.float64, device=DEV)
    native.C.stem_fwd(xp, wwin, ys, stats, N, Hp, Wp, P, Q, 1)
    ref = F.conv2d(x.to(torch.bfloat16).float(), wk.to(torch.bfloat16).float().permute(0, 3, 1, 2), stride=2,
                   padding=3)
    assert _rel(ys.view(N, P, Q, K).permute(0, 3, 1, 2), ref) < 1e-2
    st = stats.view(-1, K, 2).sum(0)
    yf = ys.view(-1, K).double()
    assert torch.allclose(st[:, 0], yf.sum(0), rtol=1e-4, atol=1e-1)
    assert torch.allclose(st[:, 1], (yf * yf).sum(0), rtol=1e-4, atol=1e-1)


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("case", [(2, 14, 14, 64, 64, 3, 1, 1), (2, 15, 13, 128, 128, 3, 2, 1), (3, 14, 14, 256, 128, 1, 2, 0),
                                  (3, 10, 56, 64, 64, 3, 1, 1), (3, 12, 56, 64, 64, 3, 1, 1),
                                  (2, 10, 10, 256, 64, 1, 1, 0)])
def test_conv_dgrad_fused_bn_backward(case, mode):
    """dgrad epilogue with the consumer BN's backward reduce (ReLU mask + sum dz, sum dz*xhat) vs torch."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(11)
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    dy = _rand16(N, P, Q, K)
    w = _rand16(K, R, R, C, scale=(1.0 / (K * R * R)) ** 0.5)
    res = _rand16(N, H, W, C) if mode > 1 else None
    plain = conv.conv_dgrad(dy, w, H, W, st, pad, residual=res).float()

    def coef_for(y):
        yf = y.float().view(-1, C)
        mean, var = yf.mean(0), yf.var(0, unbiased=False)
        invstd = torch.rsqrt(var + 1e-5)
        scale = torch.rand(C, device=DEV) + 0.5
        shift = torch.randn(C, device=DEV) * 0.3
        return torch.cat([scale, shift, mean, invstd]).contiguous(), mean, invstd

    y1 = _rand16(N, H, W, C)
    coef1, m1, i1 = coef_for(y1)
    y2 = _rand16(N, H, W, C) if mode == 3 else None
    coef2, m2, i2 = coef_for(y2) if mode == 3 else (None, None, None)
    out = torch.relu(_rand16(N, H, W, C)).to(torch.bfloat16) if mode > 1 else None
    K_ = 4 if mode == 3 else 2
    slots = torch.zeros(native.C.stat_slots() * C * K_, dtype=torch.float64, device=DEV)
    om = conv.pack_relu_mask(out) if mode > 1 else None
    dz = conv.conv_dgrad(dy, w, H, W, st, pad, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots))
    if mode == 1:
        mask = (y1.float() * coef1[:C] + coef1[C:2 * C]) > 0
    else:
        mask = out.float() > 0
    ref_dz = plain * mask
    assert _rel(dz, ref_dz) < 1e-2
    sums = slots.view(-1, C, K_).sum(0)
    dzf = dz.float().view(-1, C).double()
    x1 = ((y1.float() - m1) * i1).view(-1, C).double()
    assert torch.allclose(sums[:, 0], dzf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sums[:, 1], (dzf * x1).sum(0), rtol=1e-3, atol=1e-2)
    if mode == 3:
        x2 = ((y2.float() - m2) * i2).view(-1, C).double()
        assert torch.allclose(sums[:, 2], dzf.sum(0), rtol=1e-3, atol=1e-2)
        assert torch.allclose(sums[:, 3], (dzf * x2).sum(0), rtol=1e-3, atol=1e-2)


def test_wgrad_3x3c64_all_taps():
    """Layer1 weight-gradient kernel (9 taps per block, staged 4-row tiles, persistent) vs conv2d_weight."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(12)
    N, H, W = 5, 22, 56   # H not a multiple of 4: partial last row tile
    x = _rand16(N, H, W, 64)
    dy = _rand16(N, H, W, 64)
    blocks = native.C.wgrad_blocks_3x3c64()
    ws = torch.empty(blocks * 64 * 576, device=DEV)
    assert native.C.conv_wgrad_3x3c64(x, dy, ws, N, H, W) == blocks
    out = torch.empty(64 * 576, device=DEV)
    native.C.wgrad_reduce(ws, blocks, 64, 576, 576, 64 * 576, out, 576, 1.0, False)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      stride=1, padding=1)
    assert _rel(out.view(64, 3, 3, 64).permute(0, 3, 1, 2), ref) < 2e-3


TILES = [(128, 128, 64), (256, 64, 64), (128, 64, 64), (64, 128, 64), (256, 128, 64), (256, 256, 32),
         (128, 128, 32), (256, 64, 32), (128, 64, 32), (256, 256, 64), (512, 128, 64), (256, 128, 32)]
PP_TILES = [(256, 256, 64), (512, 128, 64)]  # 8-wave ping-pong kernel (conv_pp_kernel)


@pytest.mark.parametrize("tile", TILES)
def test_conv_tile_configs(tile):
    """Every compiled tile config (ring depth, wave count) on a strided 3x3 with stats and a residual dgrad."""
    from pytorch_distributed_template_amd.ops import conv
    bm, bn, bk = tile
    N, H, W, C, K = 2, 15, 13, 256, 256
    torch.manual_seed(13)
    x = _rand16(N, H, W, C)
    w = _rand16(K, 3, 3, C, scale=(1.0 / (C * 9)) ** 0.5)
    y, (s, ss) = conv.conv_fwd(x, w, 2, 1, stats=True, tile=tile)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2, padding=1)
    assert _rel(y, ref.permute(0, 2, 3, 1)) < 1e-2
    yf = y.float().reshape(-1, K)
    assert torch.allclose(s.float(), yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(ss.float(), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    P, Q = y.shape[1], y.shape[2]
    dy = _rand16(N, P, Q, K)
    res = _rand16(N, H, W, C)
    dx = conv.conv_dgrad(dy, w, H, W, 2, 1, residual=res, tile=tile)
    refx = torch.nn.grad.conv2d_input((N, C, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=1).permute(0, 2, 3, 1) + res.float()
    assert _rel(dx, refx) < 1e-2


@pytest.mark.parametrize("geom", [(3, 17, 224, 3, 0), (2, 9, 24, 3, 2), (2, 7, 20, 3, 1), (1, 5, 18, 3, 2)])
def test_stem_pack_matches_torch(geom):
    """fp32 NCHW -> zero-padded bf16 NHWC4 (row-tiled kernel for W % 4 == 0 and even Wp, per-pixel kernel otherwise)
    equals torch's pad + permute + cast exactly, padding and channel 3 zero."""
    from pytorch_distributed_template_amd.ops import native
    N, H, W, pad, ex = geom
    Hp, Wp = H + 2 * pad, W + 2 * pad + ex
    torch.manual_seed(13)
    x = torch.randn(N, 3, H, W, device=DEV)
    out = torch.full((N * Hp * Wp * 4,), float("nan"), dtype=torch.bfloat16, device=DEV)
    native.C.stem_pack(x, out, N, 3, H, W, pad, Hp, Wp)
    ref = torch.zeros(N, Hp, Wp, 4, device=DEV)
    ref[:, pad:pad + H, pad:pad + W, :3] = x.permute(0, 2, 3, 1)
    assert torch.equal(out.view(N, Hp, Wp, 4), ref.to(torch.bfloat16))


def test_stem_pack_u8_fused_normalize():
    """uint8 pixels normalised inside the stem packing == host-style Normalize then packing."""
    from pytorch_distributed_template_amd.data.transforms import IMAGENET_MEAN, IMAGENET_STD, normalize_on_device
    from pytorch_distributed_template_amd.ops import native
    N, H, W, pad = 3, 20, 18, 3
    Hp, Wp = H + 2 * pad + 2, W + 2 * pad + 2
    x8 = torch.randint(0, 256, (N, 3, H, W), device=DEV, dtype=torch.uint8)
    ref = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device=DEV)
    native.C.stem_pack(normalize_on_device(x8).contiguous(), ref, N, 3, H, W, pad, Hp, Wp)
    out = torch.empty_like(ref)
    std = torch.tensor(IMAGENET_STD)
    scale = (1.0 / (255.0 * std)).to(DEV)
    shift = (-torch.tensor(IMAGENET_MEAN) / std).to(DEV)
    native.C.stem_pack_u8(x8, out, N, 3, H, W, pad, Hp, Wp, scale, shift)
    assert (out.float() - ref.float()).abs().max().item() < 2e-2
    assert out.view(N, Hp, Wp, 4)[:, :, :, 3].abs().max().item() == 0  # 4th channel and padding stay zero


@pytest.mark.parametrize("resmode", [1, 2])
def test_bn_apply_relu_bitmask_and_masked_backward(resmode):
    """bn_apply writes the block output's ReLU bitmask; bn_bwd_reduce / bn_bwd_apply mask with it."""
    from pytorch_distributed_template_amd.ops import conv, native
    torch.manual_seed(5)
    rows, C = 3000, 128
    y = _rand16(rows, C)
    res = _rand16(rows, C)
    coef = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3,
                      torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5]).contiguous()
    rcoef = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3]).contiguous()
    out = torch.empty_like(y)
    mask = torch.empty(rows * C // 8, dtype=torch.uint8, device=DEV)
    native.C.bn_apply(y, coef, res, rcoef if resmode == 2 else None, out, C, resmode, True, mask)
    r = res.float() if resmode == 1 else res.float() * rcoef[:C] + rcoef[C:]
    ref = torch.relu(y.float() * coef[:C] + coef[C:2 * C] + r)
    assert _rel(out, ref) < 1e-2
    assert torch.equal(mask, conv.pack_relu_mask(out))
    g = _rand16(rows, C)
    dz_ref = g.float() * (out.float() > 0)
    slots = torch.zeros(native.C.stat_slots() * C * 2, dtype=torch.float64, device=DEV)
    native.C.bn_bwd_reduce(g, mask, y, coef, None, None, slots, native.C.bn_bwd_reduce_blocks(rows, C), rows, C)
    sums = slots.view(-1, C, 2).sum(0)
    xhat = (y.float() - coef[2 * C:3 * C]) * coef[3 * C:]
    assert torch.allclose(sums[:, 0], dz_ref.double().sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sums[:, 1], (dz_ref * xhat).double().sum(0), rtol=1e-3, atol=1e-2)
    b1 = torch.randn(3 * C, device=DEV)
    dy1 = torch.empty_like(y)
    dz = torch.empty_like(y)
    native.C.bn_bwd_apply(g, mask, y, b1, dy1, None, None, None, dz, C)
    assert torch.equal(dz.float(), dz_ref.to(dz.dtype).float())
    ref1 = b1[:C] * dz_ref + b1[C:2 * C] * y.float() + b1[2 * C:]
    assert _rel(dy1, ref1) < 1e-2


@pytest.mark.parametrize("tile", PP_TILES + [(256, 128, 32)])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_conv_pp_long_k_and_fused_bn_backward(tile, mode):
    """Ping-pong kernel (and the 4-wave 256x128 3-stage tile, same wave tile) over many K-steps and several
    (partial) M tiles: forward with stats, and backward-data with every fused BN-backward epilogue (mode 0 = plain
    dgrad with residual)."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K = 5, 14, 14, 256, 256
    torch.manual_seed(21 + mode)
    x = _rand16(N, H, W, C)
    w = _rand16(K, 3, 3, C, scale=(1.0 / (C * 9)) ** 0.5)
    y, (s, ss) = conv.conv_fwd(x, w, 1, 1, stats=True, tile=tile)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, K)
    assert torch.allclose(s.float(), yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(ss.float(), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    dy = _rand16(N, H, W, K)
    res = _rand16(N, H, W, C) if mode != 1 else None
    plain = torch.nn.grad.conv2d_input((N, C, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                       padding=1).permute(0, 2, 3, 1)
    if res is not None:
        plain = plain + res.float()
    if mode == 0:
        dx = conv.conv_dgrad(dy, w, H, W, 1, 1, residual=res, tile=tile)
        assert _rel(dx, plain) < 1e-2
        return
    y1 = _rand16(N, H, W, C)
    yf1 = y1.float().view(-1, C)
    m1, i1 = yf1.mean(0), torch.rsqrt(yf1.var(0, unbiased=False) + 1e-5)
    coef1 = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3, m1, i1]).contiguous()
    y2 = _rand16(N, H, W, C) if mode == 3 else None
    coef2 = coef1 if mode == 3 else None
    out = torch.relu(_rand16(N, H, W, C)) if mode > 1 else None
    om = conv.pack_relu_mask(out) if mode > 1 else None
    K_ = 4 if mode == 3 else 2
    slots = torch.zeros(native.C.stat_slots() * C * K_, dtype=torch.float64, device=DEV)
    dz = conv.conv_dgrad(dy, w, H, W, 1, 1, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots), tile=tile)
    mask = ((y1.float() * coef1[:C] + coef1[C:2 * C]) > 0) if mode == 1 else (out.float() > 0)
    assert _rel(dz, plain * mask) < 1e-2
    sums = slots.view(-1, C, K_).sum(0)
    dzf = dz.float().view(-1, C).double()
    x1 = ((y1.float() - m1) * i1).view(-1, C).double()
    assert torch.allclose(sums[:, 0], dzf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sums[:, 1], (dzf * x1).sum(0), rtol=1e-3, atol=1e-2)
    if mode == 3:
        x2 = ((y2.float() - m1) * i1).view(-1, C).double()
        assert torch.allclose(sums[:, 3], (dzf * x2).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("case", [(6, 14, 14, 256, 256, 3, 1, 1), (4, 15, 13, 256, 512, 3, 2, 1),
                                  (5, 14, 14, 512, 256, 1, 2, 0)])
@pytest.mark.parametrize("target", [64, 1024])
def test_conv_wgrad_pp_256(case, target):
    """256x256 ping-pong weight-gradient kernel (C, Kout multiples of 256) over several splits vs torch."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(31)
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    assert native.C.conv_wgrad_plan(K, R, R, C, N * P * Q, target, False)[2] == 256
    x = _rand16(N, H, W, C)
    dy = _rand16(N, P, Q, K)
    dw = conv.conv_wgrad(x, dy, R, R, st, pad, target_blocks=target)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, R), dy.float().permute(0, 3, 1, 2),
                                      stride=st, padding=pad).permute(0, 2, 3, 1)
    assert _rel(dw, ref) < 2e-3


@pytest.mark.parametrize("case", [(2, 14, 14, 64, 128), (3, 28, 28, 128, 256), (2, 7, 7, 256, 512)])
@pytest.mark.parametrize("tile", [None, (256, 256, 64), (128, 128, 64), (256, 64, 64)])
def test_conv_dgrad_compact_phase_residual(case, tile):
    """3x3/2 dgrad + a 1x1/2 downsample's dgrad given COMPACT (phase (0,0) only, res_phase=0) vs torch fp32."""
    from pytorch_distributed_template_amd.ops import conv
    N, H, W, C, K = case
    if tile is not None and C % tile[1]:
        pytest.skip("tile N does not divide Cin")
    torch.manual_seed(12)
    P, Q = conv.out_hw(H, W, 3, 3, 2, 1)
    dy = _rand16(N, P, Q, K)
    dyd = _rand16(N, P, Q, K)
    w = _rand16(K, 3, 3, C, scale=(1.0 / (K * 9)) ** 0.5)
    wd = _rand16(K, 1, 1, C, scale=(1.0 / K) ** 0.5)
    # the downsample's data gradient on the compact P x Q grid: a stride-1 1x1 dgrad
    rc = conv.conv_dgrad(dyd, wd, P, Q, 1, 0)
    dx = conv.conv_dgrad(dy, w, H, W, 2, 1, residual=rc, res_phase=0, tile=tile)
    ref = (torch.nn.grad.conv2d_input((N, C, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=1)
           + torch.nn.grad.conv2d_input((N, C, H, W), wd.float().permute(0, 3, 1, 2),
                                        dyd.float().permute(0, 3, 1, 2), stride=2, padding=0)).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 1e-2


@pytest.mark.parametrize("B,ld,ncols", [(1200, 1024, 1000), (37, 1024, 1000), (5, 130, 130), (64, 136, 128)])
def test_colsum_matches_torch(B, ld, ncols):
    """fc bias gradient: column sums of the 16-bit logit gradient (vectorised kernel and scalar fallback)."""
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(13)
    d = _rand16(B, ld)
    out = torch.full((ncols,), float("nan"), device=DEV)
    native.C.colsum(d, B, ld, ncols, out, 0.5)
    ref = d[:, :ncols].float().sum(0) * 0.5
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fused_producer_bn_relu_layer1(dtype):
    """the layer1 conv forward and weight gradient applying the producer BN + ReLU to their staged
    input tiles must equal the unfused chain (bn_apply -> conv / wgrad) BIT FOR BIT, including the zero padding
    of image borders (BN(0) != 0: a transformed pad would show up on every border pixel)."""
    from pytorch_distributed_template_amd.ops import conv, native
    C = native.C
    torch.manual_seed(21)
    N, H, W = 3, 12, 56
    z = _rand16(N, H, W, 64, dtype=dtype)
    w = _rand16(64, 3, 3, 64, dtype=dtype, scale=1.0 / 24)
    coef = torch.cat([torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.5,
                      torch.zeros(128, device=DEV)]).contiguous()
    a = torch.empty_like(z)
    C.bn_apply(z, coef, None, None, a, 64, 0, True, None)
    ref_a = torch.relu(z.float() * coef[:64] + coef[64:128]).to(dtype)
    assert _rel(a, ref_a) < 1e-2  # (bn_apply rounds one fma; torch rounds the product and the sum)
    # forward with statistics: unfused (conv over a) vs fused (conv over z with pre_coef)
    st_u = torch.zeros(C.stat_slots() * 64 * 2, dtype=torch.float64, device=DEV)
    st_f = torch.zeros_like(st_u)
    y_u, y_f = torch.empty_like(z), torch.empty_like(z)
    C.conv_fwd(a, w, y_u, None, st_u, N, H, W, 64, 64, 3, 3, H, W, 1, 1, -1, -1, 1, 1, H, W, 1, 1, 0, 0, 256, 64, 64, 0)
    assert C.conv_fwd_pre_supported(N, H, W)
    C.conv_fwd_pre(z, w, y_f, st_f, coef, N, H, W)
    assert torch.equal(y_u, y_f)
    assert torch.equal(st_u, st_f)
    ref = F.conv2d(ref_a.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y_f, ref) < 2e-2
    # weight gradient: unfused over a vs fused over z
    dy = _rand16(N, H, W, 64, dtype=dtype)
    blocks = C.wgrad_blocks_3x3c64()
    ws_u = torch.empty(blocks * 64 * 576, device=DEV)
    ws_f = torch.empty_like(ws_u)
    pu = C.conv_wgrad_3x3c64(a, dy, ws_u, N, H, W)
    pf = C.conv_wgrad_3x3c64(z, dy, ws_f, N, H, W, coef)
    if pu == pf:
        assert torch.equal(ws_u[:pu * 64 * 576], ws_f[:pf * 64 * 576])
    else:  # PDT_WGRAD_L1_W8=1: the unfused call ran the 8-wave form (2 partials per block), the fused one 4 waves
        g_u, g_f = torch.empty(64 * 576, device=DEV), torch.empty(64 * 576, device=DEV)
        C.wgrad_reduce(ws_u, pu, 64, 576, 576, 64 * 576, g_u, 576, 1.0, False)
        C.wgrad_reduce(ws_f, pf, 64, 576, 576, 64 * 576, g_f, 576, 1.0, False)
        assert _rel(g_u, g_f) < 1e-5
    # not eligible: H % 4 != 0 (partial row tiles go to the generic kernel, which has no fused producer BN)
    assert not C.conv_fwd_pre_supported(N, 10, W)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [12544 + 37, 70000 + 5])
def test_fused_producer_bn_relu_1x1_c64(dtype, M):
    """ResNet-50 layer1's conv3: the persistent 1x1 64 -> 256 forward and the 128-pair weight-gradient tile applying
    bn2 + ReLU to their input fragments equal the unfused chain (bn_apply -> conv / wgrad) BIT FOR BIT: outputs,
    statistics and the weight-gradient partials (M tails: zero-filled rows transform to relu(shift) but meet zero
    dY rows)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    if not C.conv1x1_c64_supported(64, 256):
        pytest.skip("PDT_CONV1X1=0")
    torch.manual_seed(23)
    z = _rand16(M, 64, dtype=dtype)
    w = _rand16(256, 64, dtype=dtype, scale=0.125)
    coef = torch.cat([torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.5,
                      torch.zeros(128, device=DEV)]).contiguous()
    a = torch.empty_like(z)
    C.bn_apply(z, coef, None, None, a, 64, 0, True, None)
    st_u = torch.zeros(C.stat_slots() * 256 * 2, dtype=torch.float64, device=DEV)
    st_f = torch.zeros_like(st_u)
    y_u = torch.empty(M, 256, dtype=dtype, device=DEV)
    y_f = torch.full_like(y_u, float("nan"))
    C.reset_dispatch_counts()
    C.conv1x1_c64(a, w, y_u, st_u, M)
    C.conv1x1_c64(z, w, y_f, st_f, M, pre=coef)
    torch.cuda.synchronize()
    assert C.dispatch_counts().get("conv1x1_c64_fused_bn_relu", 0) == 1
    assert torch.equal(y_u.view(torch.int16), y_f.view(torch.int16))
    assert torch.equal(st_u, st_f)
    ref = torch.relu(z.float() * coef[:64] + coef[64:128]) @ w.float().t()
    assert _rel(y_f, ref) < 2e-2
    # weight gradient dW[256][64] = dY^T a over the M pixels
    dy = _rand16(M, 256, dtype=dtype)
    splits, pps = tuple(C.conv_wgrad_plan(256, 1, 1, 64, M, 512, False))[:2]
    outs = []
    for x_, pre in ((a, None), (z, coef)):
        ws = torch.full((splits * 256 * 64,), float("nan"), device=DEV)
        C.conv_wgrad(x_, dy, ws, 1, 1, M, 64, 256, 1, 1, 1, M, 1, 1, 0, 0, 1, 1, 64, splits, pps, 0, False, pre=pre)
        outs.append(ws)
    torch.cuda.synchronize()
    assert C.dispatch_counts().get("conv_wgrad_128_pair_fused_bn_relu", 0) == 1
    assert torch.equal(outs[0], outs[1])
    dw = outs[1].view(splits, 256, 64).sum(0)
    assert _rel(dw, dy.float().t() @ a.float()) < 1e-2


@pytest.mark.parametrize("N,H", [(3, 12), (5, 56), (1, 4)])
@pytest.mark.parametrize("variant", ["fwd", "fwd_stats", "fwd_pre", "dgrad_res", "dgrad_bn", "dgrad_bn_out"])
def test_conv_l1_pingpong_matches_4wave(variant, N, H):
    """The 8-wave ping-pong layer1 kernel (two wave groups on alternate tiles, column-swizzled halo, counted
    waits) must write BIT-IDENTICAL outputs to the 4-wave kernel (same MFMA order per accumulator) and the same
    statistics up to fp32 summation order; block counts 1..many tiles (odd / even tiles per block)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    torch.manual_seed(31)
    W = 56
    x = _rand16(N, H, W, 64)
    w = _rand16(64, 3, 3, 64, scale=1.0 / 24)
    coef = torch.cat([torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.5,
                      torch.randn(64, device=DEV) * 0.1, torch.rand(64, device=DEV) + 0.5]).contiguous()
    res = _rand16(N, H, W, 64)
    y1 = _rand16(N, H, W, 64)
    from pytorch_distributed_template_amd.ops import conv
    omask = conv.pack_relu_mask(_rand16(N, H, W, 64))

    def run(pp):
        old = C.conv_l1_set_pp(pp)
        try:
            C.reset_dispatch_counts()
            y = torch.empty_like(x)
            st = torch.zeros(C.stat_slots() * 64 * 2, dtype=torch.float64, device=DEV)
            if variant == "fwd":
                C.conv_fwd(x, w, y, None, None, N, H, W, 64, 64, 3, 3, H, W, 1, 1, -1, -1, 1, 1, H, W, 1, 1, 0, 0,
                           256, 64, 64, 0)
            elif variant == "fwd_stats":
                C.conv_fwd(x, w, y, None, st, N, H, W, 64, 64, 3, 3, H, W, 1, 1, -1, -1, 1, 1, H, W, 1, 1, 0, 0,
                           256, 64, 64, 0)
            elif variant == "fwd_pre":
                C.conv_fwd_pre(x, w, y, st, coef, N, H, W)
            elif variant == "dgrad_res":
                y = conv.conv_dgrad(x, w, H, W, 1, 1, residual=res)
            elif variant == "dgrad_bn_out":
                # block-output BN-backward reduce (residual + ReLU bitmask + BN input): EPI 3, epilogue in two halves
                y = conv.conv_dgrad(x, w, H, W, 1, 1, residual=res, bnb=(2, y1, coef, None, None, omask, st))
            else:
                y = conv.conv_dgrad(x, w, H, W, 1, 1, bnb=(1, y1, coef, None, None, None, st))
            torch.cuda.synchronize()
            return y, st, dict(C.dispatch_counts())
        finally:
            C.conv_l1_set_pp(old)

    y4, s4, d4 = run(0)
    y8, s8, d8 = run(1)
    assert d8.get("conv_l1_pp", 0) >= 1 and d4.get("conv_l1_pp", 0) == 0
    assert torch.equal(y4, y8)
    # (fp32 partial sums in another grouping: equal to summation-order rounding)
    assert torch.allclose(s4.view(-1, 128).sum(0), s8.view(-1, 128).sum(0), rtol=1e-5, atol=1e-3)
    ref = None
    if variant.startswith("fwd") and variant != "fwd_pre":
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
        assert _rel(y8, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [12544, 12544 + 37, 70000 + 5])
def test_conv1x1_c64_matches_implicit_gemm(dtype, M):
    """Persistent 1x1 64->256 conv (conv1x1.hip) vs the implicit-GEMM conv_fwd on the same operands: outputs
    bit-identical (same MFMA K order), BN statistics equal to fp64 sums of the stored outputs; M tails and the
    multi-tile-per-block path (M = 70005: 547 tiles > 2 blocks per CU)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    if not C.conv1x1_c64_supported(64, 256):
        pytest.skip("PDT_CONV1X1=0")
    torch.manual_seed(21)
    x = _rand16(M, 64, dtype=dtype)
    w = _rand16(256, 64, dtype=dtype, scale=0.125)
    y_ref = torch.empty(M, 256, dtype=dtype, device=DEV)
    C.conv_fwd(x, w, y_ref, None, None, 1, 1, M, 64, 256, 1, 1, 1, M, 1, 1, 0, 0, 1, 1, 1, M, 1, 1, 0, 0,
               128, 128, 64, 0)
    for stats in (False, True):
        y = torch.full((M, 256), float("nan"), dtype=dtype, device=DEV)
        st = torch.zeros(C.stat_slots() * 256 * 2, dtype=torch.float64, device=DEV) if stats else None
        C.conv1x1_c64(x, w, y, st, M)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
        if stats:
            s = st.view(-1, 256, 2).sum(0)
            yf = y.double()
            assert torch.allclose(s[:, 0], yf.sum(0), rtol=1e-6, atol=1e-3)
            assert torch.allclose(s[:, 1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)
    ref = x.float() @ w.float().t()
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("bm,bn", [(256, 64), (128, 128)])
def test_conv_dgrad_fused_bn_bk32_ring_bit_identical(mode, bm, bn):
    """The fused BN-backward dgrad epilogue on the 3-stage BK=32 ring (the dgrad of convs whose Kout is not a
    multiple of 64) is bit-identical to the
    2-stage BK=64 kernel (same MFMA K order, same epilogue): dz and the statistics slots, stride-2 phases with a
    compact residual on phase 0."""
    from pytorch_distributed_template_amd.ops import conv, native
    N, H, W, C, K, R, st, pad = 3, 28, 28, bn if bn == 128 else 64, 128, 3, 2, 1
    torch.manual_seed(17)
    P, Q = conv.out_hw(H, W, R, R, st, pad)
    dy = _rand16(N, P, Q, K)
    w = _rand16(K, R, R, C, scale=(1.0 / (K * R * R)) ** 0.5)
    res = _rand16(N, P, Q, C) if mode > 1 else None
    y1 = _rand16(N, H, W, C)
    coef1 = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3,
                       y1.float().view(-1, C).mean(0), torch.rand(C, device=DEV) + 0.5]).contiguous()
    y2 = _rand16(N, H, W, C) if mode == 3 else None
    coef2 = coef1.flip(0).contiguous() if mode == 3 else None
    om = conv.pack_relu_mask(torch.relu(_rand16(N, H, W, C))) if mode > 1 else None
    K_ = 4 if mode == 3 else 2
    outs = []
    for bk in (64, 32):
        slots = torch.zeros(native.C.stat_slots() * C * K_, dtype=torch.float64, device=DEV)
        dz = conv.conv_dgrad(dy, w, H, W, st, pad, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots),
                             tile=(bm, bn, bk), res_phase=0 if res is not None else -1)
        outs.append((dz, slots))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0].view(torch.int16), outs[1][0].view(torch.int16))
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("NHW", [(4, 56, 56), (3, 13, 11)])
@pytest.mark.parametrize("mode,cin", [(2, 64), (3, 64), (2, 128)])
def test_conv1x1_c64_dgrad_bnb_matches_generic(dtype, NHW, mode, cin):
    """Backward-data of a 1x1 256 -> 64 conv with the fused block-output BN-backward epilogue (residual, ReLU bit of
    the block output, sum dz, sum dz * xhat; mode 3: a second BN branch, sum dz * xhat2) on the persistent 1x1
    kernel (conv1x1.hip) vs the generic implicit-GEMM epilogue: dz bit-identical, statistics equal up to summation
    order; M tails (3 * 13 * 11 = 429 pixels); cin = 128: ResNet-50 layer2.0's 256 -> 128 conv1 (two reduction
    halves, weights staged through the input-ring area)."""
    from pytorch_distributed_template_amd.ops import conv, native
    C = native.C
    N, H, W = NHW
    torch.manual_seed(29)
    dy = _rand16(N, H, W, cin, dtype=dtype)
    w = _rand16(cin, 1, 1, 256, dtype=dtype, scale=0.125)
    res = _rand16(N, H, W, 256, dtype=dtype)

    def branch():
        yb = _rand16(N, H, W, 256, dtype=dtype)
        cb = torch.cat([torch.rand(256, device=DEV) + 0.5, torch.randn(256, device=DEV) * 0.3,
                        yb.float().view(-1, 256).mean(0), torch.rand(256, device=DEV) + 0.5]).contiguous()
        return yb, cb
    y1, coef1 = branch()
    y2, coef2 = branch() if mode == 3 else (None, None)
    K_ = 4 if mode == 3 else 2
    om = conv.pack_relu_mask(torch.relu(_rand16(N, H, W, 256)))
    outs = []
    prev, prev_x = C.conv1x1_c64_mode(0), C.conv1x1x_mode(0)  # off: the generic implicit-GEMM epilogue
    try:
        for on in (0, 1):
            C.conv1x1_c64_mode(on)
            slots = torch.zeros(C.stat_slots() * 256 * K_, dtype=torch.float64, device=DEV)
            dz = conv.conv_dgrad(dy, w, H, W, 1, 0, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots))
            outs.append((dz, slots.view(-1, 256, K_).sum(0)))
        torch.cuda.synchronize()
    finally:
        C.conv1x1_c64_mode(prev)
        C.conv1x1x_mode(prev_x)
    (dz0, s0), (dz1, s1) = outs
    assert torch.equal(dz0.view(torch.int16), dz1.view(torch.int16))
    assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)
    # and against fp64 sums of the stored dz
    d = dz1.double().view(-1, 256)
    for k, (yb, cb) in ((1, (y1, coef1)), (3, (y2, coef2))):
        if yb is None:
            continue
        xh = ((yb.float() - cb[512:768]) * cb[768:]).double().view(-1, 256)
        assert torch.allclose(s1[:, k - 1], d.sum(0), rtol=1e-4, atol=1e-2)
        assert torch.allclose(s1[:, k], (d * xh).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin", [128, 256, 512])
@pytest.mark.parametrize("M", [3000 + 37, 40000 + 5])
def test_conv1x1x_matches_implicit_gemm(dtype, cin, M):
    """Persistent sliced 1x1 cin -> 4 cin conv (conv1x1x.hip: ResNet-50 layers 2-4 conv3) vs the implicit-GEMM conv_fwd
    on the same operands: outputs bit-identical (same MFMA K order), BN statistics equal to fp64 sums of the stored
    outputs; M tails and walkers with several tiles (M = 40005)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    N = 4 * cin
    if not C.conv1x1x_supported(cin, N):
        pytest.skip("PDT_CONV1X1X=0")
    torch.manual_seed(23)
    x = _rand16(M, cin, dtype=dtype)
    w = _rand16(N, cin, dtype=dtype, scale=(1.0 / cin) ** 0.5)
    y_ref = torch.empty(M, N, dtype=dtype, device=DEV)
    C.conv_fwd(x, w, y_ref, None, None, 1, 1, M, cin, N, 1, 1, 1, M, 1, 1, 0, 0, 1, 1, 1, M, 1, 1, 0, 0,
               128, 128, 64, 0)
    cnt0 = dict(C.dispatch_counts()).get("conv1x1x", 0)
    for stats in (False, True):
        y = torch.full((M, N), float("nan"), dtype=dtype, device=DEV)
        st = torch.zeros(C.stat_slots() * N * 2, dtype=torch.float64, device=DEV) if stats else None
        C.conv1x1x(x, w, y, st, M, cin, N, 1, 0, 0, 0)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
        if stats:
            s = st.view(-1, N, 2).sum(0)
            yf = y.double()
            assert torch.allclose(s[:, 0], yf.sum(0), rtol=1e-6, atol=1e-3)
            assert torch.allclose(s[:, 1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)
    assert dict(C.dispatch_counts()).get("conv1x1x", 0) == cnt0 + 2
    ref = x.float() @ w.float().t()
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cin,NHW", [(256, (2, 56, 56)), (512, (3, 28, 28)), (256, (3, 13, 11)), (128, (2, 9, 10))])
def test_conv1x1x_strided_matches_implicit_gemm(dtype, cin, NHW):
    """The downsample conv geometry (1x1, stride 2, cin -> 2 cin) on the sliced persistent kernel's strided-input
    path vs the implicit-GEMM conv_fwd: outputs bit-identical, statistics equal to fp64 sums (odd H / W: the last
    input row / column is read, P = ceil(H / 2))."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    Nimg, H, W = NHW
    Co = 2 * cin
    if not C.conv1x1x_supported(cin, Co):
        pytest.skip("PDT_CONV1X1X=0")
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    M = Nimg * P * Q
    torch.manual_seed(27)
    x = _rand16(Nimg, H, W, cin, dtype=dtype)
    w = _rand16(Co, cin, dtype=dtype, scale=(1.0 / cin) ** 0.5)
    y_ref = torch.empty(M, Co, dtype=dtype, device=DEV)
    C.conv_fwd(x, w, y_ref, None, None, Nimg, H, W, cin, Co, 1, 1, P, Q, 2, 2, 0, 0, 1, 1, P, Q, 1, 1, 0, 0,
               128, 128, 64, 0)
    y = torch.full((M, Co), float("nan"), dtype=dtype, device=DEV)
    st = torch.zeros(C.stat_slots() * Co * 2, dtype=torch.float64, device=DEV)
    cnt0 = dict(C.dispatch_counts()).get("conv1x1x_strided", 0)
    C.conv1x1x(x, w, y, st, M, cin, Co, 2, Nimg, H, W)
    torch.cuda.synchronize()
    assert dict(C.dispatch_counts()).get("conv1x1x_strided", 0) == cnt0 + 1
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
    s = st.view(-1, Co, 2).sum(0)
    yf = y.double()
    assert torch.allclose(s[:, 0], yf.sum(0), rtol=1e-6, atol=1e-3)
    assert torch.allclose(s[:, 1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)
    ref = x[:, ::2, ::2].reshape(M, cin).float() @ w.float().t()
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("NHW", [(2, 28, 28), (3, 13, 11)])
@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("cin", [128, 256, 512])
def test_conv1x1x_dgrad_bnb_matches_generic(dtype, NHW, mode, cin):
    """Backward-data of a 1x1 4c -> c conv (ResNet-50 layers 2-4 conv1) with the fused block-output BN-backward
    epilogue (residual, ReLU bit of the block output, sum dz, sum dz * xhat; mode 3: a second BN branch) on the
    persistent sliced kernel (conv1x1x.hip) vs the generic implicit-GEMM epilogue: dz bit-identical, statistics
    equal up to summation order (and to fp64 sums of the stored dz); M tails (3 * 13 * 11 = 429 pixels)."""
    from pytorch_distributed_template_amd.ops import conv, native
    C = native.C
    N, H, W = NHW
    Co = 4 * cin
    torch.manual_seed(31)
    dy = _rand16(N, H, W, cin, dtype=dtype)
    w = _rand16(cin, 1, 1, Co, dtype=dtype, scale=(1.0 / cin) ** 0.5)
    res = _rand16(N, H, W, Co, dtype=dtype)

    def branch():
        yb = _rand16(N, H, W, Co, dtype=dtype)
        cb = torch.cat([torch.rand(Co, device=DEV) + 0.5, torch.randn(Co, device=DEV) * 0.3,
                        yb.float().view(-1, Co).mean(0), torch.rand(Co, device=DEV) + 0.5]).contiguous()
        return yb, cb
    y1, coef1 = branch()
    y2, coef2 = branch() if mode == 3 else (None, None)
    K_ = 4 if mode == 3 else 2
    om = conv.pack_relu_mask(torch.relu(_rand16(N, H, W, Co)))
    outs = []
    prev = C.conv1x1x_mode(0)
    try:
        for on in (0, 1):
            C.conv1x1x_mode(on)
            cnt0 = dict(C.dispatch_counts()).get("conv1x1x_bnb", 0)
            slots = torch.zeros(C.stat_slots() * Co * K_, dtype=torch.float64, device=DEV)
            dz = conv.conv_dgrad(dy, w, H, W, 1, 0, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots))
            outs.append((dz, slots.view(-1, Co, K_).sum(0)))
            assert dict(C.dispatch_counts()).get("conv1x1x_bnb", 0) == cnt0 + on
        torch.cuda.synchronize()
    finally:
        C.conv1x1x_mode(prev)
    (dz0, s0), (dz1, s1) = outs
    assert torch.equal(dz0.view(torch.int16), dz1.view(torch.int16))
    assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)
    d = dz1.double().view(-1, Co)
    for k, (yb, cb) in ((1, (y1, coef1)), (3, (y2, coef2))):
        if yb is None:
            continue
        xh = ((yb.float() - cb[2 * Co:3 * Co]) * cb[3 * Co:]).double().view(-1, Co)
        assert torch.allclose(s1[:, k - 1], d.sum(0), rtol=1e-4, atol=1e-2)
        assert torch.allclose(s1[:, k], (d * xh).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("mode,cin", [(2, 64), (3, 64), (2, 128)])
@pytest.mark.parametrize("NHW", [(2, 56, 56), (3, 13, 11)])
def test_conv1x1x_bnb_layer1_matches_c64(mode, cin, NHW):
    """ResNet-50 layer1's 1x1 256 -> 64 | 128 backward-data with the block-output BN epilogue on the generic sliced
    kernel (conv1x1x_l1_mode 1, the C = 64 configurations) vs the dedicated conv1x1_c64_bnb kernel: dz bit-identical,
    statistics equal up to summation order."""
    from pytorch_distributed_template_amd.ops import conv, native
    C = native.C
    N, H, W = NHW
    torch.manual_seed(37)
    dy = _rand16(N, H, W, cin)
    w = _rand16(cin, 1, 1, 256, scale=0.125)
    res = _rand16(N, H, W, 256)

    def branch():
        yb = _rand16(N, H, W, 256)
        cb = torch.cat([torch.rand(256, device=DEV) + 0.5, torch.randn(256, device=DEV) * 0.3,
                        yb.float().view(-1, 256).mean(0), torch.rand(256, device=DEV) + 0.5]).contiguous()
        return yb, cb
    y1, coef1 = branch()
    y2, coef2 = branch() if mode == 3 else (None, None)
    K_ = 4 if mode == 3 else 2
    om = conv.pack_relu_mask(torch.relu(_rand16(N, H, W, 256)))
    outs = []
    prev = C.conv1x1x_l1_mode(0)
    try:
        for on in (0, 1):
            C.conv1x1x_l1_mode(on)
            cnt0 = dict(C.dispatch_counts()).get("conv1x1x_bnb", 0)
            slots = torch.zeros(C.stat_slots() * 256 * K_, dtype=torch.float64, device=DEV)
            dz = conv.conv_dgrad(dy, w, H, W, 1, 0, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots))
            outs.append((dz, slots.view(-1, 256, K_).sum(0)))
            assert dict(C.dispatch_counts()).get("conv1x1x_bnb", 0) == cnt0 + on
        torch.cuda.synchronize()
    finally:
        C.conv1x1x_l1_mode(prev)
    (dz0, s0), (dz1, s1) = outs
    assert torch.equal(dz0.view(torch.int16), dz1.view(torch.int16))
    assert torch.allclose(s0, s1, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("width,groups,stride,H", [(128, 32, 1, 14), (256, 32, 2, 14), (128, 2, 1, 9),
                                                   (256, 64, 2, 8), (128, 32, 1, 56)])
def test_grouped_conv_slices_match_torch(width, groups, stride, H):
    """ResNeXt grouped 3x3 conv on the channel-slice kernels (gconv_fwd / gconv_dgrad / gconv_wgrad: 64-channel
    slices with block-diagonal weights, strided operands) vs fp32 torch F.conv2d(groups=...): forward with the BN
    statistics of the slices in one buffer, backward data (stride-2: sub-pixel phases) with and without the fused
    inner-BN reduce, and the weight gradient's diagonal blocks.  At 56 x 56, stride 1 (ResNeXt stage 1) the forward
    and backward data run on the layer1 halo kernel with strided operands (conv_l1pp_kernel SL)."""
    from pytorch_distributed_template_amd.ops import conv, native
    C_ = native.C
    torch.manual_seed(3)
    C_.reset_dispatch_counts()
    N, W, R, pad, S = 2, H, 3, 1, 64
    cg = width // groups
    P, Q = conv.out_hw(H, W, R, R, stride, pad)
    x = _rand16(N, H, W, width)
    wg = _rand16(width, R, R, cg, scale=(1.0 / (cg * 9)) ** 0.5)  # grouped KRSC weight
    # dense block-diagonal slice weights [nslice][64][R][R][64]
    nsl = width // S
    dense = torch.zeros(nsl, S, R, R, S, dtype=wg.dtype, device=DEV)
    for j in range(nsl):
        for k in range(S):
            g0 = (k // cg) * cg
            dense[j, k, :, :, g0:g0 + cg] = wg[j * S + k]
    # forward + statistics
    y = torch.full((N, P, Q, width), float("nan"), dtype=x.dtype, device=DEV)
    st = torch.zeros(C_.stat_slots() * width * 2, dtype=torch.float64, device=DEV)
    for j in range(nsl):
        C_.gconv_fwd(x, dense[j].reshape(-1), y, st, N, H, W, width, R, stride, pad, P, Q, j, 256, 64)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wg.float().permute(0, 3, 1, 2), stride=stride, padding=pad,
                   groups=groups).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
    s = st.view(-1, width, 2).sum(0)
    yf = y.double().reshape(-1, width)
    assert torch.allclose(s[:, 0], yf.sum(0), rtol=1e-6, atol=1e-3)
    assert torch.allclose(s[:, 1], (yf * yf).sum(0), rtol=1e-6, atol=1e-3)
    # backward data: per slice the phase weights of the dense slice weight
    dy = _rand16(N, P, Q, width)
    derived, phases_of = [], []
    off = 0
    for j in range(nsl):
        pl = []
        flat_j = dense[j].reshape(-1)
        for ph, pw, rs, ss, ioff_h, ioff_w in conv.dgrad_phases(R, R, stride, pad):
            m = conv.dgrad_weight_index(S, S, R, R, rs, ss)
            if m.numel() == 0 or H - ph <= 0 or W - pw <= 0:
                continue
            derived.append(flat_j[m.to(DEV)])
            pl.append([ph, pw, len(rs), len(ss), ioff_h, ioff_w, off])
            off += m.numel()
        phases_of.append(pl)
    derived = torch.cat(derived)
    dx = torch.full((N, H, W, width), float("nan"), dtype=x.dtype, device=DEV)
    for j in range(nsl):
        C_.gconv_dgrad(dy, derived, dx, N, P, Q, width, H, W, stride, phases_of[j], j, 256, 64)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = wg.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, wr, stride=stride, padding=pad, groups=groups).backward(dy.float().permute(0, 3, 1, 2))
    torch.cuda.synchronize()
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    # fused inner-BN reduce (mode 1): dz = dx * relu'(y1 * scale + shift), sums of dz and dz * xhat
    y1 = _rand16(N, H, W, width)
    coef = torch.cat([torch.rand(width, device=DEV) + 0.5, torch.randn(width, device=DEV) * 0.3,
                      y1.float().view(-1, width).mean(0), torch.rand(width, device=DEV) + 0.5]).contiguous()
    slots = torch.zeros(C_.stat_slots() * width * 2, dtype=torch.float64, device=DEV)
    dz = torch.full_like(dx, float("nan"))
    for j in range(nsl):
        C_.gconv_dgrad(dy, derived, dz, N, P, Q, width, H, W, stride, phases_of[j], j, 256, 64, bn_y1=y1,
                       bn_coef1=coef, bn_slots=slots)
    torch.cuda.synchronize()
    mask = (y1.float() * coef[:width] + coef[width:2 * width]) > 0
    dz_ref = torch.where(mask, dx.float(), torch.zeros_like(dx.float()))
    assert torch.equal(dz, dz_ref.to(dz.dtype))
    sums = slots.view(-1, width, 2).sum(0)
    xhat = (y1.float() - coef[2 * width:3 * width]) * coef[3 * width:]
    assert torch.allclose(sums[:, 0].float(), dz.float().view(-1, width).sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sums[:, 1].float(), (dz.float() * xhat).view(-1, width).sum(0), rtol=1e-3, atol=1e-2)
    # weight gradient: dense slice partials, diagonal blocks == the grouped weight gradient
    splits, pps, _ = C_.conv_wgrad_plan(S, R, R, S, N * P * Q, 256, False)
    ldw = R * R * S
    ws = torch.full((splits * S * ldw,), float("nan"), device=DEV)
    dwd = torch.empty(nsl, S, ldw, device=DEV)
    for j in range(nsl):
        C_.gconv_wgrad(x, dy, ws, N, H, W, width, R, P, Q, stride, pad, j, ldw, splits, pps)
        C_.wgrad_reduce(ws, splits, S, ldw, ldw, S * ldw, dwd[j].view(-1), ldw, 1.0, False)
    torch.cuda.synchronize()
    dwd = dwd.view(nsl, S, R, R, S)
    got = torch.stack([dwd[j, k, :, :, (k // cg) * cg:(k // cg) * cg + cg] for j in range(nsl) for k in range(S)])
    assert _rel(got, wr.grad.permute(0, 2, 3, 1)) < 1e-2
    # every slice in ONE launch (j = -1, blockIdx.z = slice): bit-identical outputs, statistics and partial sums
    y2 = torch.full_like(y, float("nan"))
    st2 = torch.zeros_like(st)
    C_.gconv_fwd(x, dense.reshape(-1), y2, st2, N, H, W, width, R, stride, pad, P, Q, -1, 256, 64)
    dx2 = torch.full_like(dx, float("nan"))
    C_.gconv_dgrad(dy, derived, dx2, N, P, Q, width, H, W, stride, phases_of[0], -1, 256, 64)
    dz2 = torch.full_like(dx, float("nan"))
    slots2 = torch.zeros_like(slots)
    C_.gconv_dgrad(dy, derived, dz2, N, P, Q, width, H, W, stride, phases_of[0], -1, 256, 64, bn_y1=y1,
                   bn_coef1=coef, bn_slots=slots2)
    ws2 = torch.full((splits * nsl * S * ldw,), float("nan"), device=DEV)
    C_.gconv_wgrad(x, dy, ws2, N, H, W, width, R, P, Q, stride, pad, -1, ldw, splits, pps)
    dwd2 = torch.empty(nsl * S * ldw, device=DEV)
    C_.wgrad_reduce(ws2, splits, nsl * S, ldw, ldw, nsl * S * ldw, dwd2, ldw, 1.0, False)
    torch.cuda.synchronize()
    assert torch.equal(y2, y) and torch.equal(st2, st)
    assert torch.equal(dx2, dx) and torch.equal(dz2, dz) and torch.equal(slots2, slots)
    assert torch.equal(dwd2.view(nsl, S, R, R, S), dwd)
    if H == 56 and stride == 1:  # forward, backward data, backward data with the BN reduce; per slice and all slices
        assert C_.dispatch_counts().get("conv_l1_sliced", 0) == 6 * nsl, C_.dispatch_counts()
        # the weight gradient of every slice on the layer1 halo kernel: partials [parts][nslice][64][576]
        parts = C_.wgrad_blocks_3x3c64()
        ws4 = torch.full((parts * nsl * S * ldw,), float("nan"), device=DEV)
        p = C_.gconv_wgrad_l1(x, dy, ws4, N, H, W, width)
        dwd4 = torch.empty(nsl * S * ldw, device=DEV)
        C_.wgrad_reduce(ws4, p, nsl * S, ldw, ldw, nsl * S * ldw, dwd4, ldw, 1.0, False)
        torch.cuda.synchronize()
        dwd4 = dwd4.view(nsl, S, R, R, S)
        got4 = torch.stack([dwd4[j, k, :, :, (k // cg) * cg:(k // cg) * cg + cg] for j in range(nsl) for k in range(S)])
        assert _rel(got4, got) < 1e-5  # (the same products, another fp32 summation order)
        assert _rel(got4, wr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("tile", [(256, 64, 64), (128, 128, 64), (256, 128, 64), (256, 256, 64)])
def test_phased_dgrad_one_launch_equals_per_phase_launches(tile):
    """Strided backward-data runs all its sub-pixel phases in ONE launch (grid.y = phase, the grid sized for the largest
    phase, surplus blocks only zeroing their statistics rows).  dX must be bit-identical to launching every phase on its
    own, for every tile family, including partial M tiles."""
    from pytorch_distributed_template_amd.ops import conv, native
    bm, bn, bk = tile
    N, H, W, K = 3, 19, 17, 128
    C = bn if bn >= 128 else 64
    torch.manual_seed(31)
    w = _rand16(K, 3, 3, C, scale=(1.0 / (C * 9)) ** 0.5)
    P, Q = conv.out_hw(H, W, 3, 3, 2, 1)
    dy = _rand16(N, P, Q, K)
    dx = conv.conv_dgrad(dy, w, H, W, 2, 1, tile=tile)
    wflat = w.reshape(-1)
    ref = torch.full_like(dx, float("nan"))
    for ph, pw, rs, ss, ioff_h, ioff_w in conv.dgrad_phases(3, 3, 2, 1):
        idx = conv.dgrad_weight_index(K, C, 3, 3, rs, ss).to(w.device)
        wt = wflat[idx].contiguous()
        native.C.conv_dgrad(dy, wt, ref, None, N, P, Q, K, C, H, W, 2, [[ph, pw, len(rs), len(ss), ioff_h, ioff_w, 0]],
                            bm, bn, bk)
    assert torch.equal(dx, ref)
