"""End-to-end numerics of the native ResNet executor vs the plain PyTorch fp32 model (MI355X)."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(arch="resnet18", N=8, HW=64, dtype=torch.bfloat16, seed=0):
    from pytorch_distributed_template_amd.models import resnet
    from pytorch_distributed_template_amd.models.executor import ResNetExecutor
    from pytorch_distributed_template_amd.optim.flat import FlatBuffers, FlatParams
    torch.manual_seed(seed)
    model = getattr(resnet, arch)()
    # make BN affine params non-trivial so their gradients are exercised
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(model).to(DEV).train()
    flat = FlatParams(model, DEV, dtype)
    FlatBuffers(model, DEV)
    ex = ResNetExecutor(model, flat, DEV, dtype)
    # the reference computes in fp32 on the same 16-bit-rounded weights
    with torch.no_grad():
        for (n, p), (n2, p2) in zip(model.named_parameters(), ref.named_parameters()):
            p2.copy_(p.detach().to(dtype).float())
    x = torch.randn(N, 3, HW, HW, device=DEV)
    t = torch.randint(0, 1000, (N,), device=DEV)
    return model, ref, flat, ex, x, t


def ref_scale(b):
    return b.float().norm().clamp_min(1e-3)


def _relnorm(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("arch,dtype", [("resnet18", torch.bfloat16), ("resnet18", torch.float16),
                                        ("resnet50", torch.bfloat16), ("resnext50_32x4d", torch.bfloat16),
                                        ("resnext50_32x4d", torch.float16)])
def test_train_step_matches_reference(arch, dtype):
    """Gradients vs an fp32 reference, judged against stock PyTorch autocast at the same 16-bit dtype
    (random-init ResNets amplify 16-bit rounding through the BN backward chain; the oracle is "no
    worse than torch.autocast")."""
    model, ref, flat, ex, x, t = _setup(arch, N=8 if arch == "resnet18" else 4, dtype=dtype)
    tb = copy.deepcopy(ref)
    logits, met = ex.train_step(x, t)
    torch.cuda.synchronize()
    out = ref(x)
    loss = F.cross_entropy(out, t)
    loss.backward()
    with torch.autocast("cuda", dtype=dtype):
        ob = tb(x)
        lb = F.cross_entropy(ob, t)
    lb.backward()
    assert abs(met[0].item() - loss.item()) / loss.item() < 5e-3
    assert _relnorm(logits, out.detach()) < 1.5 * _relnorm(ob.detach(), out.detach()) + 0.02
    bad = []
    for (n, p), (_, p2), (_, p3) in zip(model.named_parameters(), ref.named_parameters(), tb.named_parameters()):
        ours, theirs = _relnorm(p.grad, p2.grad), _relnorm(p3.grad, p2.grad)
        if ours > 1.5 * theirs + 0.02:
            bad.append((n, ours, theirs))
    assert not bad, bad[:5]
    # running statistics follow the batch statistics like nn.BatchNorm2d (judged against autocast too)
    bad = []
    for (n, b), (_, b2), (_, b3) in zip(model.named_buffers(), ref.named_buffers(), tb.named_buffers()):
        if "running" in n:
            scale = b2.float().norm().clamp_min(1e-3)
            ours, theirs = ((b - b2).norm() / scale).item(), ((b3 - b2).norm() / scale).item()
            if ours > 1.5 * theirs + 0.01:
                bad.append((n, ours, theirs))
    assert not bad, bad[:5]


def test_eval_step_matches_reference():
    model, ref, flat, ex, x, t = _setup("resnet18")
    ex.train_step(x, t)   # populate running stats
    ref(x)
    ref.eval()
    logits, met = ex.eval_step(x, t)
    with torch.no_grad():
        out = ref(x)
    assert _relnorm(logits, out) < 5e-2
    assert abs(met[0].item() - F.cross_entropy(out, t).item()) < 5e-2


def test_training_reduces_loss():
    from pytorch_distributed_template_amd.optim.sgd import FusedSGD
    model, ref, flat, ex, x, t = _setup("resnet18", N=16)
    opt = FusedSGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    losses = []
    for _ in range(12):
        _, met = ex.train_step(x, t)
        opt.step()
        ex.update_derived()
        losses.append(met[0].item())
    assert losses[-1] < losses[0] * 0.5, losses


# kernel variants the 224x224 ResNet-18 step must dispatch (C.dispatch_counts(), csrc/common.h PDT_COUNT):
# the dedicated stem, layer1 halo-reuse fwd/dgrad, the 9-tap layer1 weight gradient, the fused stem
# weight gradient, the ping-pong 256x256 conv and weight-gradient kernels, phased strided dgrad with the
# compact downsample residual
R18_224_KERNELS = ("stem_fwd", "conv_l1_fwd", "conv_l1_dgrad", "wgrad3x3_c64", "wgrad_stem_fused", "conv_pp_fwd",
                   "conv_pp_dgrad", "conv_wgrad_pp", "conv_generic_dgrad_phased", "conv_dgrad_compact_residual",
                   "conv_l1_fwd_fused_bn_relu", "wgrad3x3_c64_fused_bn_relu")


# ResNet-50's specialised kernels: the persistent 1x1 64->256 forward, the fused-BN 1x1 backward-data kernel in its
# one-branch, two-branch (downsample block) and 128-reduction-channel forms, and the 512x128 ping-pong tile the shipped
# tile table picks for its 1x1 convs (csrc/kernels/conv1x1.hip, conv_fwd.hip)
R50_224_KERNELS = ("conv1x1_c64", "conv1x1_c64_bnb_1br", "conv1x1_c64_bnb_2br", "conv1x1_c64_bnb_c128",
                   "conv_pp_512x128", "stem_fwd", "conv_pp_fwd", "conv_wgrad_pp", "wgrad_stem_fused", "conv1x1x",
                   "conv1x1x_bnb", "conv1x1x_bnb_2br", "conv1x1_c64_fused_bn_relu", "conv_wgrad_128_pair_fused_bn_relu")


def test_resnet50_fused_bn2_conv3_is_bit_identical():
    """ResNet-50 layer1's bn2 + ReLU applied by conv3's forward and weight gradient (no a2 tensor) gives the same
    step as the unfused chain bit for bit: logits, loss and every gradient."""
    model, ref, flat, ex, x, t = _setup("resnet50", N=4, HW=224, dtype=torch.bfloat16)
    from pytorch_distributed_template_amd.ops import native
    outs = []
    for fuse in (False, True):
        ex.fuse_pre_1x1 = fuse
        flat.grad.zero_()
        native.C.reset_dispatch_counts()
        logits, met = ex.train_step(x, t)
        torch.cuda.synchronize()
        n = native.C.dispatch_counts().get("conv1x1_c64_fused_bn_relu", 0)
        assert n == (3 if fuse else 0), n
        outs.append((logits.clone(), met.clone(), flat.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("arch,N", [("resnet18", 16), ("resnet18", 32), ("resnet50", 8), ("resnet34", 4),
                                    ("resnet101", 3), ("resnet152", 2), ("wide_resnet50_2", 3),
                                    ("wide_resnet101_2", 2), ("resnext50_32x4d", 4), ("resnext101_32x8d", 2),
                                    ("resnext101_64x4d", 2)])
def test_train_step_matches_reference_224(arch, N, monkeypatch):
    """The bench geometry (224x224) for every arch the native engine accepts (engine/runner.py NATIVE_ARCHS):
    gradients and running stats vs fp32 torch, judged against torch autocast bf16, with the specialised kernels
    asserted to have run (ResNet-18 and ResNet-50; the shipped B = 1200 tile table re-keyed to this batch so its
    tile choices are exercised)."""
    from pytorch_distributed_template_amd.models import executor
    from pytorch_distributed_template_amd.ops import native
    if arch == "resnet50":
        monkeypatch.setattr(executor, "_TUNED", {(k[0], N) + k[2:]: v for k, v in executor._TUNED.items()})
    model, ref, flat, ex, x, t = _setup(arch, N=N, HW=224, dtype=torch.bfloat16)
    tb = copy.deepcopy(ref)
    native.C.reset_dispatch_counts()
    logits, met = ex.train_step(x, t)
    torch.cuda.synchronize()
    counts = {k: v for k, v in native.C.dispatch_counts().items() if v}
    print("dispatch", arch, N, counts)
    want = {"resnet18": R18_224_KERNELS, "resnet50": R50_224_KERNELS,
            "resnext50_32x4d": ("gconv_fwd", "gconv_dgrad", "gconv_wgrad")}.get(arch, ())
    missing = [k for k in want if not counts.get(k)]
    assert not missing, (missing, counts)
    out = ref(x)
    loss = F.cross_entropy(out, t)
    loss.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ob = tb(x)
        lb = F.cross_entropy(ob, t)
    lb.backward()
    # loss within 5e-3 (ResNet-18/50); the deeper archs at N = 2-4 carry 12-16 % bf16 logits error vs fp32 in BOTH
    # engines (tools/deep_arch_probe.py: wide_resnet101_2 logits rel 0.138 ours / 0.135 autocast, resnext101_32x8d
    # 0.137 / 0.136, 0.122 / 0.131; the loss off by up to 1.6 % ours and 1 % autocast depending on the seed), so their
    # loss is held to 2.5e-2 and the logits / gradient checks below carry the comparison with autocast
    tol = 5e-3 if arch in ("resnet18", "resnet50") else 2.5e-2
    assert abs(met[0].item() - loss.item()) / loss.item() < tol
    assert _relnorm(logits, out.detach()) < 1.5 * _relnorm(ob.detach(), out.detach()) + 0.02
    bad = []
    for (n, p), (_, p2), (_, p3) in zip(model.named_parameters(), ref.named_parameters(), tb.named_parameters()):
        ours, theirs = _relnorm(p.grad, p2.grad), _relnorm(p3.grad, p2.grad)
        if ours > 1.5 * theirs + 0.02:
            bad.append((n, round(ours, 4), round(theirs, 4)))
    assert not bad, bad[:5]
    bad = []
    for (n, b), (_, b2), (_, b3) in zip(model.named_buffers(), ref.named_buffers(), tb.named_buffers()):
        if "running" in n:
            scale = b2.float().norm().clamp_min(1e-3)
            ours, theirs = ((b - b2).norm() / scale).item(), ((b3 - b2).norm() / scale).item()
            if ours > 1.5 * theirs + 0.01:
                bad.append((n, ours, theirs))
    assert not bad, bad[:5]


def _grads_after_step(side: bool, delay_side: int = 0, delay_main: int = 0, arch="resnet18", N=16, steps=1,
                      env=None, dtype=torch.bfloat16):
    """Run ``steps`` train steps (+ SGD + derived-layout refresh) and return (grad, data, buffers) copies.
    ``delay_side`` / ``delay_main`` spin-kernel cycles are injected ahead of every side-stream weight
    gradient / after it on the compute stream, to shake out missing cross-stream dependencies.  ``env``: extra
    PDT_* settings read when the executor is built."""
    import os
    from pytorch_distributed_template_amd.optim.sgd import FusedSGD
    env = dict(env or {})
    env["PDT_WGRAD_STREAM"] = "1" if side else "0"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        model, ref, flat, ex, x, t = _setup(arch, N=N, HW=224, dtype=dtype)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    del ref
    if delay_side or delay_main:
        orig = ex._side_wgrad

        def slow(reads, fn):
            def fn2():
                if delay_side:
                    torch.cuda._sleep(delay_side)  # on the side stream: the wgrad starts late
                fn()
            orig(reads, fn2)
            if delay_main:
                torch.cuda._sleep(delay_main)  # compute stream falls behind the side stream
        ex._side_wgrad = slow
    opt = FusedSGD(flat, lr=0.1, momentum=0.9, weight_decay=1e-4)
    for _ in range(steps):
        ex.train_step(x, t)
        ex._join_side()
        opt.step()
        ex.update_derived()
    torch.cuda.synchronize()
    bufs = torch.cat([b.float().reshape(-1) for n, b in model.named_buffers() if "running" in n])
    return flat.grad.clone(), flat.data.clone(), bufs, flat.slots


@pytest.mark.parametrize("delay_side,delay_main", [(0, 0), (2_000_000, 0), (0, 2_000_000)])
def test_side_stream_bitwise_equals_single_stream(delay_side, delay_main):
    """Race detector for the two-stream backward (weight gradients on a side stream): with or without
    injected delays on either stream, gradients, the SGD update and running statistics must be BIT-identical
    to the single-stream schedule (same kernels, same arithmetic order -- any difference is a missing
    cross-stream dependency)."""
    g0, d0, b0, slots = _grads_after_step(False, steps=2)
    g1, d1, b1, _ = _grads_after_step(True, delay_side, delay_main, steps=2)
    bad = [(s.name, int((g0[s.offset:s.offset + s.numel] != g1[s.offset:s.offset + s.numel]).sum()))
           for s in slots if not torch.equal(g0[s.offset:s.offset + s.numel], g1[s.offset:s.offset + s.numel])]
    assert not bad, bad[:10]
    assert torch.equal(d0, d1)
    assert torch.equal(b0, b1)


def _poison_allocator(gib: float = 24.0):
    """Fill the caching allocator's free memory with 0xFF bytes (NaN in every float format) so a kernel that
    reads memory nobody wrote produces NaN / different bits instead of silently reading zeros."""
    big = [torch.full((int(gib * 2 ** 30) // 4,), -1, dtype=torch.int32, device=DEV)]
    small = [torch.full((128 * 1024,), -1, dtype=torch.int32, device=DEV) for _ in range(2048)]  # 512 KiB each
    torch.cuda.synchronize()
    del big, small


def test_no_reads_of_unwritten_memory():
    """Two identical 224-px training steps, the second with the allocator pre-filled with NaN bytes: results
    must be bit-identical (no kernel may read a buffer region that was never written)."""
    g0, d0, b0, slots = _grads_after_step(True, steps=2)
    torch.cuda.empty_cache()
    _poison_allocator()
    g1, d1, b1, _ = _grads_after_step(True, steps=2)
    bad = [(s.name, int((g0[s.offset:s.offset + s.numel] != g1[s.offset:s.offset + s.numel]).sum()))
           for s in slots if not torch.equal(g0[s.offset:s.offset + s.numel], g1[s.offset:s.offset + s.numel])]
    assert not bad, bad[:10]
    assert torch.equal(d0, d1)
    assert torch.equal(b0, b1)


_VALIDATE_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
from pytorch_distributed_template_amd.models import registry
from pytorch_distributed_template_amd.ops import native, validate
dev = torch.device("cuda:0")
torch.manual_seed(0)
tr = NativeTrainer(registry.create("resnet18"), dev, dtype=torch.bfloat16)
x = torch.randn(8, 3, 64, 64, device=dev)
t = torch.randint(0, 1000, (8,), device=dev)
for _ in range(2):
    tr.train_step(x, t)
torch.cuda.synchronize()
v = validate.validator()
print("CLEAN_CALLS", v.calls, "WRAPPED", hasattr(native.C.conv_fwd, "__wrapped__"))
x[0, 0, 5, 5] = float("nan")
try:
    tr.train_step(x, t)
except validate.NonFiniteError as e:
    print("CAUGHT", str(e).splitlines()[0])
"""


def test_validation_mode_localises_nonfinite(tmp_path):
    """PDT_VALIDATE=2 over the real kernels: clean steps pass with every native op launch-checked and
    scanned; a NaN pixel is attributed to the first op that spreads it (the stem input packing)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    log = tmp_path / "ops.log"
    env = dict(os.environ, PDT_VALIDATE="2", PDT_VALIDATE_LOG=str(log))
    r = subprocess.run([sys.executable, "-c", _VALIDATE_SCRIPT.format(root=root)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    clean = [ln for ln in r.stdout.splitlines() if ln.startswith("CLEAN_CALLS")][0].split()
    assert int(clean[1]) > 100 and clean[3] == "True", r.stdout
    caught = [ln for ln in r.stdout.splitlines() if ln.startswith("CAUGHT")]
    assert caught and "native op `stem_pack` wrote" in caught[0], r.stdout + r.stderr[-2000:]
    ops = log.read_text().splitlines()
    assert ops[-1].startswith("stem_pack ") and any(o.startswith("conv_fwd ") for o in ops)
