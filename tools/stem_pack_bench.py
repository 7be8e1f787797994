import torch, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pytorch_distributed_template_amd.ops import native
C = native.C
N = 1200
x = torch.randn(N, 3, 224, 224, device="cuda")
Hp, Wp = 230, 230
out = torch.empty(N * Hp * Wp * 4, dtype=torch.bfloat16, device="cuda")
C.stem_pack(x, out, N, 3, 224, 224, 3, Hp, Wp)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    C.stem_pack(x, out, N, 3, 224, 224, 3, Hp, Wp)
e1.record(); torch.cuda.synchronize()
ref = torch.nn.functional.pad(x, (3, 3, 3, 3)).permute(0, 2, 3, 1)
ref = torch.cat([ref, torch.zeros_like(ref[..., :1])], -1).to(torch.bfloat16).reshape(-1)
print(os.environ.get("PDT_NATIVE_SO", "in-tree"), "stem_pack us", e0.elapsed_time(e1) / 10 * 1000, "exact", torch.equal(out, ref))
