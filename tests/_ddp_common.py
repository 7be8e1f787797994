"""Shared model / batch construction for the DDP numerics tests and their rank script."""
import torch


def make_model(seed: int = 0, arch: str = "resnet18"):
    from pytorch_distributed_template_amd.models import registry
    torch.manual_seed(seed)
    model = registry.create(arch)
    g = torch.Generator().manual_seed(seed + 7)
    for m in model.modules():  # non-trivial BN affine parameters, so their gradients matter
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.4 - 0.2)
    return model


def make_batch(n: int, hw: int, seed: int = 1234):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 3, hw, hw, generator=g), torch.randint(0, 1000, (n,), generator=g)
