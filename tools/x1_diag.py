"""One-off: conv1x1x_bnb (C = 64 configuration) vs conv1x1_c64_bnb statistics against fp64 sums of the stored dz."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from pytorch_distributed_template_amd.ops import conv, native  # noqa: E402

C = native.C
DEV = "cuda"
for (N, H, W), cin, mode in (((4, 56, 56), 64, 2), ((4, 56, 56), 64, 3), ((2, 28, 28), 128, 3),
                              ((2, 28, 28), 256, 2), ((2, 28, 28), 256, 3), ((2, 14, 14), 512, 3)):
    Co = 256 if cin <= 128 else 4 * cin
    torch.manual_seed(29)
    dy = (torch.randn(N, H, W, cin, device=DEV)).to(torch.bfloat16)
    w = (torch.randn(cin, 1, 1, Co, device=DEV) * 0.125).to(torch.bfloat16)
    res = torch.randn(N, H, W, Co, device=DEV).to(torch.bfloat16)
    y1 = torch.randn(N, H, W, Co, device=DEV).to(torch.bfloat16)
    coef1 = torch.cat([torch.rand(Co, device=DEV) + 0.5, torch.randn(Co, device=DEV) * 0.3,
                       y1.float().view(-1, Co).mean(0), torch.rand(Co, device=DEV) + 0.5]).contiguous()
    y2 = torch.randn(N, H, W, Co, device=DEV).to(torch.bfloat16) if mode == 3 else None
    coef2 = torch.cat([torch.rand(Co, device=DEV) + 0.5, torch.randn(Co, device=DEV) * 0.3,
                       y2.float().view(-1, Co).mean(0), torch.rand(Co, device=DEV) + 0.5]).contiguous() if mode == 3 else None
    K_ = 4 if mode == 3 else 2
    om = conv.pack_relu_mask(torch.relu(torch.randn(N, H, W, Co, device=DEV).to(torch.bfloat16)))
    for label, c64, l1 in (("c64", 1, 0), ("x1", 1, 1), ("generic", 0, 0)):  # noqa
        C.conv1x1_c64_mode(c64)
        C.conv1x1x_l1_mode(l1)
        pm = C.conv1x1x_mode(-1)
        if label == "generic":
            C.conv1x1x_mode(0)
        slots = torch.zeros(C.stat_slots() * Co * K_, dtype=torch.float64, device=DEV)
        dz = conv.conv_dgrad(dy, w, H, W, 1, 0, residual=res, bnb=(mode, y1, coef1, y2, coef2, om, slots))
        torch.cuda.synchronize()
        C.conv1x1x_mode(pm)
        s = slots.view(-1, Co, K_).sum(0)
        d = dz.double().view(-1, Co)
        xh = ((y1.float() - coef1[2 * Co:3 * Co]) * coef1[3 * Co:]).double().view(-1, Co)
        r0, r1 = d.sum(0), (d * xh).sum(0)
        e0 = ((s[:, 0] - r0).abs() / (r0.abs() + 1)).max().item()
        e1 = ((s[:, 1] - r1).abs() / (r1.abs() + 1)).max().item()
        e3 = 0.0
        if mode == 3:
            xh2 = ((y2.float() - coef2[2 * Co:3 * Co]) * coef2[3 * Co:]).double().view(-1, Co)
            r3 = (d * xh2).sum(0)
            e3 = ((s[:, 3] - r3).abs() / (r3.abs() + 1)).max().item()
        print(f"cin {cin} mode {mode} {label:8s} stats err sum {e0:.3e} sum*xhat {e1:.3e} sum*xhat2 {e3:.3e} "
              f"dz sum {d.abs().sum().item():.6e}", flush=True)
