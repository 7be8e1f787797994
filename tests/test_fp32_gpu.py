"""The native fp32 path (reference precision: `distributed.py` / `dataparallel.py` train without autocast):
fp32 MFMA conv forward / multi-phase backward-data / weight gradient vs PyTorch fp32 autograd, the fp32 executor's
training step vs an fp32 torch model, and the entry script on --precision fp32 (MI355X)."""
import copy
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _no_tf32():
    old = (torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    yield
    torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32 = old


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


SHAPES = [  # N, H, Cin, Cout, k, stride
    (2, 56, 64, 64, 3, 1), (3, 30, 64, 128, 3, 1),  # layer1 geometry (the halo weight-gradient kernel) and a ragged W
    (4, 14, 64, 128, 3, 1), (4, 14, 64, 64, 3, 2), (4, 14, 128, 256, 1, 2), (3, 9, 192, 128, 3, 1),
    (2, 7, 256, 512, 3, 2), (5, 10, 64, 256, 1, 1),
]


def _tiles(n):
    """every (BM, BN) tile the fp32 conv kernel has for a GEMM-N of n: the 4-wave 128-row and 8-wave 256-row ones"""
    out = [(128, 128 if n % 128 == 0 else 64)]
    if n == 64:
        out += [(256, 64), (512, 64)]
    if n % 256 == 0:
        out.append((256, 256))
    if n % 128 == 0:
        out.append((256, 128))
    return out


@pytest.mark.parametrize("shape", SHAPES)
def test_conv32_fwd_dgrad_wgrad_match_torch(shape):
    from pytorch_distributed_template_amd.ops import native
    from pytorch_distributed_template_amd.ops.conv import dgrad_phases, dgrad_weight_index
    C = native.C
    N, H, cin, cout, k, st = shape
    pad = k // 2
    torch.manual_seed(0)
    x = torch.randn(N, cin, H, H, device=DEV, requires_grad=True)
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).requires_grad_()
    res_nchw = torch.randn(N, cout, (H + 2 * pad - k) // st + 1, (H + 2 * pad - k) // st + 1, device=DEV)
    y = F.conv2d(x, w, stride=st, padding=pad)
    gy = torch.randn_like(y)
    y.backward(gy)
    P = y.shape[2]
    xh = x.detach().permute(0, 2, 3, 1).contiguous()
    wk = w.detach().permute(0, 2, 3, 1).contiguous()  # KRSC
    # forward + BN statistics + residual, every tile configuration
    resh = res_nchw.permute(0, 2, 3, 1).contiguous()
    ref = (y.detach() + res_nchw).permute(0, 2, 3, 1)
    for bm, bn in _tiles(cout):
        out = torch.empty(N, P, P, cout, device=DEV)
        sp = torch.empty(C.stat_slots() * cout * 2, dtype=torch.float64, device=DEV)
        C.conv32_fwd(xh, wk.reshape(-1), out, resh, sp, N, H, H, cin, cout, k, k, P, P, st, pad, bm, bn)
        assert _rel(out, ref) < 1e-5, (bm, bn)
        s = sp.view(C.stat_slots(), cout, 2).sum(0)
        assert _rel(s[:, 0], ref.reshape(-1, cout).double().sum(0)) < 1e-6
        assert _rel(s[:, 1], (ref.reshape(-1, cout).double() ** 2).sum(0)) < 1e-6
    # backward-data: every sub-pixel phase in one launch
    wflat = wk.reshape(-1)
    pieces, phases, off = [], [], 0
    for ph, pw, rs, ss, ioff_h, ioff_w in dgrad_phases(k, k, st, pad):
        idx = dgrad_weight_index(cout, cin, k, k, rs, ss).to(DEV)
        if idx.numel():
            pieces.append(wflat[idx])
        phases.append([ph, pw, len(rs), len(ss), ioff_h, ioff_w, off])
        off += idx.numel()
    wt = torch.cat(pieces)
    gyh = gy.permute(0, 2, 3, 1).contiguous()
    for bm, bn in _tiles(cin):
        dx = torch.empty(N, H, H, cin, device=DEV)
        C.conv32_dgrad(gyh, wt, dx, None, N, P, P, cout, cin, H, H, st, phases, bm, bn)
        assert _rel(dx, x.grad.permute(0, 2, 3, 1)) < 1e-5, (bm, bn)
    # weight gradient (split-K over pixels + fixed-order split reduction)
    ldw = k * k * cin
    npix = N * P * P
    pps = ((npix + 2) // 3 + 63) // 64 * 64
    splits = (npix + pps - 1) // pps
    tiles = [64] + ([128] if cin % 128 == 0 and cout % 128 == 0 else []) + (
        [3] if k == 3 and st == 1 and cin % 64 == 0 and cout % 64 == 0 and H <= 62 else [])
    for tile in tiles:
        sp, pp = (splits, pps) if tile != 3 else (3, (N * P + 2) // 3)  # halo kernel: splits over output rows
        ws = torch.empty(sp * cout * ldw, device=DEV)
        C.wgrad32(xh, gyh, ws, N, H, H, cin, cout, k, k, P, P, st, pad, ldw, sp, pp, tile)
        dw = torch.empty(cout * ldw, device=DEV)
        C.wgrad_reduce(ws, sp, cout, ldw, ldw, cout * ldw, dw, ldw, 1.0, False)
        assert _rel(dw.view(cout, k, k, cin), w.grad.permute(0, 2, 3, 1)) < 1e-5, tile


def _setup(arch, N, HW, seed=0):
    from pytorch_distributed_template_amd.models import resnet
    from pytorch_distributed_template_amd.models.executor32 import ResNetExecutor32
    from pytorch_distributed_template_amd.optim.flat import FlatBuffers, FlatParams
    torch.manual_seed(seed)
    model = getattr(resnet, arch)()
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(model).to(DEV).train()
    flat = FlatParams(model, DEV, None)
    FlatBuffers(model, DEV)
    ex = ResNetExecutor32(model, flat, DEV)
    x = torch.randn(N, 3, HW, HW, device=DEV)
    t = torch.randint(0, 1000, (N,), device=DEV)
    return model, ref, flat, ex, x, t


@pytest.mark.parametrize("arch,N,HW,chunk", [("resnet18", 8, 64, None), ("resnet50", 4, 128, None),
                                             ("resnet50", 4, 64, None), ("resnet18", 6, 224, 4),
                                             ("resnet34", 4, 128, None), ("resnet101", 2, 128, None),
                                             ("resnet152", 2, 128, None), ("wide_resnet50_2", 2, 128, None),
                                             ("wide_resnet101_2", 2, 128, None), ("resnext50_32x4d", 2, 128, None),
                                             ("resnext101_64x4d", 2, 96, None)])
def test_executor32_train_step_matches_torch_fp32(arch, N, HW, chunk):
    """The whole fp32 step vs an fp64 PyTorch oracle, judged against PyTorch's own fp32 autograd: logits, loss,
    every gradient and the running statistics must be no worse than torch fp32 (+ a small absolute floor) --
    random-init ResNets amplify rounding differences through the backward chain, so a fixed fp32 tolerance
    would be meaningless.  (ResNet-50 at 64 px, i.e. BatchNorm over 4 x 2 x 2 = 16 values per channel in
    layer4, is ill-conditioned enough that a single ReLU-mask flip of a near-zero pre-activation in the last
    block moves that block's gradients by ~1 % (round-4 fp64 comparison).  128 px keeps the comparison meaningful.)
    (chunk: the im2col stem processed in several image chunks.)  ResNeXts: grouped convs as gathered 64-channel
    slices on the dense fp32 kernels."""
    model, ref, flat, ex, x, t = _setup(arch, N, HW)
    if chunk:
        ex._stem_chunk = lambda n: chunk
    ref64 = copy.deepcopy(ref).double()
    ref64b = copy.deepcopy(ref).double()
    logits, met = ex.train_step(x, t)
    torch.cuda.synchronize()
    out = ref(x)
    loss = F.cross_entropy(out, t)
    loss.backward()
    out64 = ref64(x.double())
    F.cross_entropy(out64, t).backward()
    # sensitivity floor: the fp64 gradients themselves under a 1e-4 relative input nudge -- the size of fp32's
    # own forward rounding at ResNet-50 depth (torch fp32 and ours both reach ~7e-5 vs fp64 at the last block,
    # the round-4 fp64 comparison); ReLU-mask flips of near-zero pre-activations move whole blocks' gradients by ~1 %
    # (an additive random nudge: BatchNorm normalises a uniform input scaling away)
    g = torch.Generator(device=DEV).manual_seed(5)
    F.cross_entropy(ref64b(x.double() + 1e-4 * torch.randn(x.shape, device=DEV, generator=g).double()), t).backward()
    assert _rel(logits, out64.detach()) <= 3 * _rel(out.detach(), out64.detach()) + 1e-5
    assert abs(met[0].item() - loss.item()) < 1e-3 * max(1.0, loss.item())
    bad = []
    for (n, p), (_, p2), (_, p3), (_, p4) in zip(model.named_parameters(), ref.named_parameters(),
                                                 ref64.named_parameters(), ref64b.named_parameters()):
        ours, theirs, floor = _rel(p.grad, p3.grad), _rel(p2.grad, p3.grad), _rel(p4.grad, p3.grad)
        if ours > 3 * max(theirs, floor) + 1e-4:
            bad.append((n, ours, theirs, floor))
    assert not bad, bad[:6]
    for (n, b), (_, b2), (_, b3) in zip(model.named_buffers(), ref.named_buffers(), ref64.named_buffers()):
        if "running" in n:
            assert _rel(b, b3) <= 3 * _rel(b2, b3) + 1e-6, n


def test_native_trainer_fp32_learns_and_evaluates_in_fp32():
    """NativeTrainer at fp32 (no shadow) reduces the loss; a bf16 trainer's --eval-precision fp32 path evaluates
    on the fp32 kernels over the fp32 master (equal to an fp32 trainer's eval of the same weights)."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(0)
    tr = NativeTrainer(registry.create("resnet18"), DEV, dtype=torch.float32, lr=0.05)
    assert tr.flat.shadow is None
    x = torch.randn(16, 3, 64, 64, device=DEV)
    t = torch.randint(0, 1000, (16,), device=DEV)
    losses = [tr.train_step(x, t)[1][0].item() for _ in range(10)]
    assert losses[-1] < 0.6 * losses[0], losses
    torch.manual_seed(1)
    tb = NativeTrainer(registry.create("resnet18"), DEV, dtype=torch.bfloat16, eval_fp32=True)
    tb.train_step(x, t)
    l16, _ = tb.eval_step(x, t)
    torch.manual_seed(2)
    t32 = NativeTrainer(registry.create("resnet18"), DEV, dtype=torch.float32)
    t32.model.load_state_dict(tb.model.state_dict())
    t32.on_state_loaded()
    l32, _ = t32.eval_step(x, t)
    torch.cuda.synchronize()
    assert torch.equal(l16, l32)


def test_entry_script_fp32_native(tmp_path):
    out = str(tmp_path / "out")
    r = subprocess.run([sys.executable, "distributed.py", "--outpath", out, "--synthetic", "--synthetic-train-size", "256",
                        "--synthetic-val-size", "64", "--image-size", "64", "-j", "0", "--epochs", "1", "-b", "64",
                        "--exist-policy", "delete", "--precision", "fp32"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, PYTHONUNBUFFERED="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    log = open(os.path.join(out + "_resnet18", "experiment.log")).read()
    assert "=> engine: native | compute dtype: float32" in log


def test_fp32_syncbn_native_comm_world1_equals_plain_bn():
    """--precision fp32 with --sync_batchnorm on the native communicator (forced at world 1, identity all-reduces):
    the fp32 executor's SyncBN path runs (it used to raise AttributeError on _sync_sum_fwd) and matches plain BN."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    x = torch.randn(8, 3, 64, 64, device=DEV)
    t = torch.randint(0, 1000, (8,), device=DEV)
    out = []
    for sync in (True, False):
        torch.manual_seed(0)
        tr = NativeTrainer(registry.create("resnet18"), DEV, dtype=torch.float32, comm="native", force_comm=True,
                           sync_bn=sync)
        for _ in range(2):
            tr.train_step(x, t)
        torch.cuda.synchronize()
        out.append(tr.flat.data.clone())
    assert _rel(out[0], out[1]) < 1e-5


@pytest.mark.parametrize("tile", [(128, 64), (256, 64)])
def test_conv32_stem_window_mode_matches_torch(tile):
    """fp32 stem in window mode (conv32 over the zero-padded NHWC4 image: K = 7 kernel rows x (8 pixels x 4 channels),
    no im2col buffer) vs torch's fp32 conv2d, with the BN statistics epilogue."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    torch.manual_seed(3)
    N, H, W = 3, 64, 48
    x = torch.randn(N, 3, H, W, device=DEV)
    w = torch.randn(64, 3, 7, 7, device=DEV) / 147 ** 0.5
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = max(H + 6, (P - 1) * 2 + 7), max(W + 6, (Q - 1) * 2 + 8)
    xp = torch.empty(N * Hp * Wp * 4, device=DEV)
    C.stem_pack32(x, xp, N, 3, H, W, 3, Hp, Wp)
    ww = torch.zeros(64, 7, 8, 4, device=DEV)
    ww[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    y = torch.empty(N * P * Q * 64, device=DEV)
    st = torch.zeros(C.stat_slots() * 64 * 2, dtype=torch.float64, device=DEV)
    C.conv32_stem_fwd(xp, ww.reshape(-1).contiguous(), y, st, N, Hp, Wp, 7, P, Q, 2, 64, *tile)
    ref = F.conv2d(x, w, stride=2, padding=3).permute(0, 2, 3, 1)
    assert _rel(y.view(N, P, Q, 64), ref) < 1e-5
    s = st.view(-1, 64, 2).sum(0)
    yf = y.view(-1, 64).double()
    assert torch.allclose(s[:, 0], yf.sum(0), rtol=1e-5, atol=1e-3)
    assert torch.allclose(s[:, 1], (yf * yf).sum(0), rtol=1e-5, atol=1e-3)


def test_fp32_executor_window_stem_matches_im2col_stem(monkeypatch):
    """PDT_FP32_STEM_WIN=1 (window-mode stem forward) trains like the im2col stem: same loss / gradients to fp32
    rounding of a different summation order."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(0)
    model = registry.create("resnet18")
    x = torch.randn(4, 3, 64, 64, device=DEV)
    t = torch.randint(0, 1000, (4,), device=DEV)
    outs = []
    for win in ("0", "1"):
        monkeypatch.setenv("PDT_FP32_STEM_WIN", win)
        tr = NativeTrainer(copy.deepcopy(model), torch.device(DEV), dtype=torch.float32, lr=0.0)
        assert tr.executor.stem_win == (win == "1")
        logits, met = tr.train_step(x, t)
        torch.cuda.synchronize()
        ex = tr.executor
        outs.append((logits.float().clone(), ex._g(ex.fc_slot).clone(), tr.flat.grad.clone(),
                     ex._g(ex.stem.slot).clone()))
    assert _rel(outs[1][0], outs[0][0]) < 1e-5
    # the fc gradient sees the forward only through features and logits; the whole-network gradient also goes
    # through max-pool argmaxes and ReLU masks that a last-bit difference of the stem output can flip (random init,
    # batch 4): bounded, not bitwise
    assert _rel(outs[1][1], outs[0][1]) < 1e-4
    assert _rel(outs[1][3], outs[0][3]) < 5e-2, (outs[1][3][:8], outs[0][3][:8])
    assert _rel(outs[1][2], outs[0][2]) < 5e-2


@pytest.mark.parametrize("all_pairs", [0, 1])
def test_wgrad32_stem_window_pair_matches_torch(all_pairs):
    """fp32 stem weight gradient in window-pair mode (tap = kernel-row pair over the padded NHWC4 image) vs
    torch.nn.grad.conv2d_weight in fp32: one block per pair (wgrad32_kernel) and all 4 pairs per block
    (wgrad32_stem4_kernel)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    torch.manual_seed(4)
    N, H, W = 3, 40, 36
    x = torch.randn(N, 3, H, W, device=DEV)
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    Hp, Wp = max(H + 6, (P - 1) * 2 + 8), max(W + 6, (Q - 1) * 2 + 8)
    xp = torch.empty(N * Hp * Wp * 4, device=DEV)
    C.stem_pack32(x, xp, N, 3, H, W, 3, Hp, Wp)
    dy = torch.randn(N, P, Q, 64, device=DEV)
    npix = N * P * Q
    splits, pps = 7, ((npix + 6) // 7 + 63) // 64 * 64
    splits = (npix + pps - 1) // pps
    ws = torch.empty(splits * 64 * 256, device=DEV)
    C.reset_dispatch_counts()
    C.wgrad32_stem(xp, dy.contiguous(), ws, N, Hp, Wp, 4, 64, P, Q, 2, splits, pps, all_pairs)
    assert dict(C.dispatch_counts()).get("wgrad32_stem4", 0) == all_pairs
    dw = ws.view(splits, 64, 4, 2, 8, 4).sum(0)  # [k][pair][row in pair][pixel s][channel]
    dw = dw.reshape(64, 8, 8, 4)[:, :7, :7, :3].permute(0, 3, 1, 2)  # rows 0..7 -> 7 kernel rows
    ref = torch.nn.grad.conv2d_weight(x, (64, 3, 7, 7), dy.permute(0, 3, 1, 2), stride=2, padding=3)
    assert _rel(dw, ref) < 1e-5


def test_fp32_fused_bn_backward_reduce_matches_separate_pass(monkeypatch):
    """The inner BatchNorms' backward reduce fused into the fp32 backward-data epilogue (conv32 EPI 2) gives the
    gradients of the separate bn_bwd_reduce32 pass to fp32 summation-order rounding, and really runs."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.models.executor32 import ResNetExecutor32
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(1)
    model = registry.create("resnet18")
    x = torch.randn(4, 3, 64, 64, device=DEV)
    t = torch.randint(0, 1000, (4,), device=DEV)
    outs = []
    for fuse in (False, True):
        monkeypatch.setattr(ResNetExecutor32, "_FUSE_BN", fuse)
        tr = NativeTrainer(copy.deepcopy(model), torch.device(DEV), dtype=torch.float32, lr=0.0)
        native.C.reset_dispatch_counts()
        logits, met = tr.train_step(x, t)
        torch.cuda.synchronize()
        n_fused = dict(native.C.dispatch_counts()).get("conv32_dgrad_bn_reduce_epilogue", 0)
        assert (n_fused > 0) == fuse
        outs.append((logits.float().clone(), tr.flat.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])  # the forward is untouched
    assert _rel(outs[1][1], outs[0][1]) < 1e-3


@pytest.mark.parametrize("N,H,W,cin,cout", [(2, 56, 56, 64, 64), (5, 10, 10, 64, 64), (3, 7, 9, 128, 128)])
def test_conv32_halo_kernel_matches_restaging_kernel_and_torch(N, H, W, cin, cout):
    """The fp32 3x3/s1 halo kernel (all 9 taps off one staged halo per 32-channel chunk; tiles spanning several
    images, ragged widths, 2 output-channel tiles) vs torch fp32 and vs the per-tap restaging conv32_kernel:
    forward + residual + BN statistics, and stride-1 backward-data."""
    from pytorch_distributed_template_amd.ops import native
    from pytorch_distributed_template_amd.ops.conv import dgrad_phases, dgrad_weight_index
    C = native.C
    torch.manual_seed(3)
    x = torch.randn(N, cin, H, W, device=DEV, requires_grad=True)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (cin * 9) ** 0.5).requires_grad_()
    res = torch.randn(N, cout, H, W, device=DEV)
    y = F.conv2d(x, w, padding=1)
    gy = torch.randn_like(y)
    y.backward(gy)
    xh, wk = x.detach().permute(0, 2, 3, 1).contiguous(), w.detach().permute(0, 2, 3, 1).contiguous()
    resh, gyh = res.permute(0, 2, 3, 1).contiguous(), gy.permute(0, 2, 3, 1).contiguous()
    ref = (y.detach() + res).permute(0, 2, 3, 1)
    wflat = wk.reshape(-1)
    pieces, phases, off = [], [], 0
    for ph, pw, rs, ss, ioff_h, ioff_w in dgrad_phases(3, 3, 1, 1):
        idx = dgrad_weight_index(cout, cin, 3, 3, rs, ss).to(DEV)
        pieces.append(wflat[idx])
        phases.append([ph, pw, len(rs), len(ss), ioff_h, ioff_w, off])
        off += idx.numel()
    wt = torch.cat(pieces)
    got = {}
    prev = C.conv32_set_halo(1)
    try:
        for halo in (1, 0):
            C.conv32_set_halo(halo)
            C.reset_dispatch_counts()
            out = torch.empty(N, H, W, cout, device=DEV)
            sp = torch.zeros(C.stat_slots() * cout * 2, dtype=torch.float64, device=DEV)
            C.conv32_fwd(xh, wflat, out, resh, sp, N, H, W, cin, cout, 3, 3, H, W, 1, 1, 128, 64)
            dx = torch.empty(N, H, W, cin, device=DEV)
            C.conv32_dgrad(gyh, wt, dx, None, N, H, W, cout, cin, H, W, 1, phases, 128, 64)
            torch.cuda.synchronize()
            n = dict(C.dispatch_counts()).get("conv32_halo", 0)
            assert n == (2 if halo else 0), n
            assert _rel(out, ref) < 1e-5, halo
            s = sp.view(C.stat_slots(), cout, 2).sum(0)
            assert _rel(s[:, 0], ref.reshape(-1, cout).double().sum(0)) < 1e-6
            assert _rel(s[:, 1], (ref.reshape(-1, cout).double() ** 2).sum(0)) < 1e-6
            assert _rel(dx, x.grad.permute(0, 2, 3, 1)) < 1e-5, halo
            got[halo] = (out, dx)
    finally:
        C.conv32_set_halo(prev)
    assert _rel(got[1][0], got[0][0]) < 1e-6 and _rel(got[1][1], got[0][1]) < 1e-6


def test_fp32_fused_stem_tail_matches_the_separate_passes(monkeypatch):
    """The stem's backward tail with dz recomputed inside the BN-backward reduce and apply (no stored dz) gives the
    gradients of maxpool_bwd_relu32 + bn_bwd_reduce32 + bn_bwd_apply32 to fp32 rounding (the same operations; the
    compiler's fma contraction may differ between the kernels), and really runs."""
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry
    from pytorch_distributed_template_amd.models.executor32 import ResNetExecutor32
    from pytorch_distributed_template_amd.ops import native
    torch.manual_seed(2)
    model = registry.create("resnet18")
    x = torch.randn(3, 3, 80, 72, device=DEV)
    t = torch.randint(0, 1000, (3,), device=DEV)
    outs = []
    for fuse in (False, True):
        monkeypatch.setattr(ResNetExecutor32, "_FUSE_STEM", fuse)
        tr = NativeTrainer(copy.deepcopy(model), torch.device(DEV), dtype=torch.float32, lr=0.0)
        native.C.reset_dispatch_counts()
        logits, met = tr.train_step(x, t)
        torch.cuda.synchronize()
        cnt = dict(native.C.dispatch_counts())
        assert (cnt.get("stem_pool_bwd_fused32", 0) + cnt.get("stem_pool_bwd_reduce_out32", 0) > 0) == fuse
        outs.append(tr.flat.grad.clone())
    assert _rel(outs[1], outs[0]) < 1e-5


def test_wgrad32_stem_fused_dy_matches_apply_then_wgrad():
    """The 4-pair fp32 stem weight gradient with dY computed in the kernel (max-pool backward from the pooled gradient
    and argmax, ReLU mask, BN-backward apply) equals stem_pool_bwd_apply32 followed by the plain 4-pair kernel: same
    float operations in the same order -- random argmax codes included (border windows whose code points outside the
    image select nothing in both), an odd pooled width, and a split whose last chunk is partial."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    torch.manual_seed(6)
    N, H, W = 2, 42, 38
    x = torch.randn(N, 3, H, W, device=DEV)
    P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    OH, OW = (P - 1) // 2 + 1, (Q - 1) // 2 + 1
    Hp, Wp = max(H + 6, (P - 1) * 2 + 8), max(W + 6, (Q - 1) * 2 + 8)
    xp = torch.empty(N * Hp * Wp * 4, device=DEV)
    C.stem_pack32(x, xp, N, 3, H, W, 3, Hp, Wp)
    y0 = torch.randn(N * P * Q * 64, device=DEV)
    dp = torch.randn(N * OH * OW * 64, device=DEV)
    idx = torch.randint(0, 9, (N * OH * OW * 64,), device=DEV, dtype=torch.uint8)
    coef = torch.cat([torch.rand(64, device=DEV) + 0.5, torch.randn(64, device=DEV) * 0.3,  # scale | shift
                      torch.randn(64, device=DEV), torch.rand(64, device=DEV) + 0.5])  # mean | invstd
    bcoef = torch.randn(192, device=DEV)
    npix = N * P * Q
    pps = ((npix + 4) // 5 + 63) // 64 * 64
    splits = (npix + pps - 1) // pps
    assert npix % 32 != 0 or splits * pps > npix
    dy = torch.empty(npix * 64, device=DEV)
    C.stem_pool_bwd_apply32(dp, idx, y0, coef, bcoef, dy, N, P, Q, 64)
    ws_ref = torch.zeros(splits * 64 * 256, device=DEV)
    C.wgrad32_stem(xp, dy, ws_ref, N, Hp, Wp, 4, 64, P, Q, 2, splits, pps, 1)
    ws = torch.zeros(splits * 64 * 256, device=DEV)
    C.reset_dispatch_counts()
    C.wgrad32_stem_fused(xp, dp, idx, y0, coef, bcoef, ws, N, Hp, Wp, P, Q, 2, splits, pps)
    torch.cuda.synchronize()
    assert dict(C.dispatch_counts()).get("wgrad32_stem4_fused", 0) == 1
    assert _rel(ws, ws_ref) < 1e-6, _rel(ws, ws_ref)
    print("bit-identical:", torch.equal(ws, ws_ref))


def test_stem_pool_bwd_reduce_out32_matches_window_gather():
    """The stem's BN-backward sums over the POOLED output (mask out > 0, BN input recovered as (out - shift) / scale)
    equal the window-gather reduce over the 112x112 conv output to fp32 rounding -- negative and zero BN scales
    included (a zero scale contributes xhat = 0 in both)."""
    from pytorch_distributed_template_amd.ops import native
    C = native.C
    torch.manual_seed(8)
    N, H, W, ch = 3, 23, 18, 64
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y0 = torch.randn(N * H * W * ch, device=DEV)
    sc = torch.rand(ch, device=DEV) + 0.2
    sc[:8] = -sc[:8]
    sc[8] = 0.0
    coef = torch.cat([sc, torch.randn(ch, device=DEV) * 0.5, torch.randn(ch, device=DEV) * 0.1,
                      torch.rand(ch, device=DEV) + 0.5])
    out = torch.empty(N * OH * OW * ch, device=DEV)
    idx = torch.empty(N * OH * OW * ch, device=DEV, dtype=torch.uint8)
    C.bn_relu_maxpool32(y0, coef, out, idx, N, H, W, ch)
    dp = torch.randn(N * OH * OW * ch, device=DEV)
    ref = torch.zeros(64 * ch * 2, device=DEV, dtype=torch.float64)
    got = torch.zeros_like(ref)
    C.stem_pool_bwd_reduce32(dp, idx, y0, coef, ref, 7, N, H, W, ch)
    C.stem_pool_bwd_reduce_out32(dp, out, coef, got, 5, ch)
    r, g = ref.view(64, ch, 2).sum(0), got.view(64, ch, 2).sum(0)
    scale = dp.abs().view(-1, ch).sum(0).double()  # sum |dz| bounds both sums' rounding
    assert ((r - g).abs() <= 1e-5 * scale[:, None] + 1e-9).all(), ((r - g).abs() / scale[:, None]).max()
