"""Diagnostic: per-parameter gradient error of the native executor vs an fp32 reference, next to
the error of stock PyTorch bf16 autocast vs the same reference (what "bf16 noise" looks like)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from pytorch_distributed_template_amd.models import resnet
from pytorch_distributed_template_amd.models.executor import ResNetExecutor
from pytorch_distributed_template_amd.optim.flat import FlatBuffers, FlatParams

DEV = "cuda"
arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
HW = int(sys.argv[3]) if len(sys.argv) > 3 else 64
torch.manual_seed(0)
model = getattr(resnet, arch)()
for m in model.modules():
    if isinstance(m, torch.nn.BatchNorm2d):
        m.weight.data.uniform_(0.5, 1.5)
        m.bias.data.uniform_(-0.2, 0.2)
ref = copy.deepcopy(model).to(DEV).train()
with torch.no_grad():
    for p in ref.parameters():
        p.copy_(p.to(torch.bfloat16).float())
tb = copy.deepcopy(ref)
flat = FlatParams(model, DEV, torch.bfloat16)
FlatBuffers(model, DEV)
ex = ResNetExecutor(model, flat, DEV, torch.bfloat16)
x = torch.randn(N, 3, HW, HW, device=DEV)
t = torch.randint(0, 1000, (N,), device=DEV)
logits, met = ex.train_step(x, t)
out = ref(x)
loss = F.cross_entropy(out, t)
loss.backward()
with torch.autocast("cuda", dtype=torch.bfloat16):
    out_b = tb(x)
    loss_b = F.cross_entropy(out_b, t)
loss_b.backward()


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-20)).item()


print(f"loss ours {met[0].item():.5f} ref {loss.item():.5f} torch-bf16 {loss_b.item():.5f}")
print(f"logits rel ours {rel(logits, out):.4f} torch-bf16 {rel(out_b, out):.4f}")
print(f"{'param':40s} {'ours':>8s} {'torchbf16':>9s}")
for (n, p), (_, p2), (_, p3) in zip(model.named_parameters(), ref.named_parameters(), tb.named_parameters()):
    print(f"{n:40s} {rel(p.grad, p2.grad):8.4f} {rel(p3.grad, p2.grad):9.4f}")
