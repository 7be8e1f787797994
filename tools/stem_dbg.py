import os, sys, torch
sys.path.insert(0, "/root/repo" if os.path.exists("/root/repo") else ".")
from pytorch_distributed_template_amd.ops import native
C_ = native.C
DEV = "cuda"
torch.manual_seed(9)
N, H, W = 2, 64, 64
K = C = 64
P, Q = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
Hp, Wp = max(H + 6, 2 * (P - 1) + 8), max(W + 6, 2 * (Q - 1) + 8)
x = torch.randn(N, 3, H, W, device=DEV)
xp = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device=DEV)
C_.stem_pack(x, xp, N, 3, H, W, 3, Hp, Wp)
y = (torch.randn(N, P, Q, C, device=DEV)).to(torch.bfloat16)
coef = torch.cat([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.2, torch.zeros(C, device=DEV), torch.ones(C, device=DEV)]).contiguous()
OH, OW = (P - 1) // 2 + 1, (Q - 1) // 2 + 1
out = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=DEV)
idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=DEV)
C_.bn_relu_maxpool(y, coef, out, idx, N, P, Q, C)
dp = torch.randn(N, OH, OW, C, device=DEV).to(torch.bfloat16)
bcoef = torch.cat([torch.rand(C, device=DEV), torch.randn(C, device=DEV) * 0.1, torch.randn(C, device=DEV) * 0.1]).contiguous()
pairs, ldw = 4, 256
splits, pps, _ = C_.conv_wgrad_plan(K, pairs, 1, 64, N * P * Q, 64, True)
dy = torch.empty_like(y)
C_.stem_pool_bwd_apply(dp, idx, y, coef, bcoef, dy, N, P, Q, C)
ws = torch.empty(splits * K * ldw, device=DEV)
C_.conv_wgrad(xp, dy, ws, N, Hp, Wp, 64, K, pairs, 1, P, Q, 2, 2, 0, 0, 2, 2, ldw, splits, pps, 4, True)
t1 = torch.empty(K * ldw, device=DEV)
C_.wgrad_reduce(ws, splits, K, ldw, ldw, K * ldw, t1, ldw, 1.0, False)
ws2 = torch.full_like(ws, float("nan"))
C_.conv_wgrad_stem_fused(xp, dp, idx, y, coef, bcoef, ws2, N, Hp, Wp, pairs, P, Q, 2, 2, ldw, splits, pps)
t2 = torch.empty(K * ldw, device=DEV)
C_.wgrad_reduce(ws2, splits, K, ldw, ldw, K * ldw, t2, ldw, 1.0, False)
torch.cuda.synchronize()
print("counts", {k: v for k, v in C_.dispatch_counts().items() if v and "stem" in k})
a, b = t1.view(K, 4, 2, 32), t2.view(K, 4, 2, 32)
d = (a - b).abs()
print("rel", ((a - b).norm() / a.norm()).item())
print("err by pair", [round((d[:, t].norm() / a[:, t].norm()).item(), 4) for t in range(4)])
print("err by half", [round((d[:, :, h].norm() / a[:, :, h].norm()).item(), 4) for h in range(2)])
print("err by s", [round((d[..., s*4:(s+1)*4].norm() / a[..., s*4:(s+1)*4].norm()).item(), 4) for s in range(8)])
print("err by k-block", [round((d[k*16:(k+1)*16].norm() / a[k*16:(k+1)*16].norm()).item(), 4) for k in range(4)])
