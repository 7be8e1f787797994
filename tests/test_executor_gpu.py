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
                                        ("resnet50", torch.bfloat16)])
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
                   "conv_pp_dgrad", "conv_wgrad_pp", "conv_generic_dgrad_phased", "conv_dgrad_compact_residual")


@pytest.mark.parametrize("arch,N", [("resnet18", 16), ("resnet18", 32), ("resnet50", 8)])
def test_train_step_matches_reference_224(arch, N):
    """The bench geometry (224x224): gradients and running stats vs fp32 torch, judged against torch
    autocast bf16, with the specialised kernels asserted to have run."""
    from pytorch_distributed_template_amd.ops import native
    model, ref, flat, ex, x, t = _setup(arch, N=N, HW=224, dtype=torch.bfloat16)
    tb = copy.deepcopy(ref)
    native.C.reset_dispatch_counts()
    logits, met = ex.train_step(x, t)
    torch.cuda.synchronize()
    counts = {k: v for k, v in native.C.dispatch_counts().items() if v}
    print("dispatch", arch, N, counts)
    if arch == "resnet18":
        missing = [k for k in R18_224_KERNELS if not counts.get(k)]
        assert not missing, (missing, counts)
    out = ref(x)
    loss = F.cross_entropy(out, t)
    loss.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ob = tb(x)
        lb = F.cross_entropy(ob, t)
    lb.backward()
    assert abs(met[0].item() - loss.item()) / loss.item() < 5e-3
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
