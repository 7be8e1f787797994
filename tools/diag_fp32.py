"""Diagnostic: per-parameter gradient error of the native fp32 executor vs an fp64 torch oracle, next to torch
fp32's own error (tests/test_fp32_gpu.py prints only the first failures)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
torch.backends.cudnn.allow_tf32 = False
torch.backends.cuda.matmul.allow_tf32 = False
from test_fp32_gpu import _rel, _setup  # noqa: E402

for arch, N, HW in [(a.split(":")[0], int(a.split(":")[1]), int(a.split(":")[2])) for a in sys.argv[1:]]:
    model, ref, flat, ex, x, t = _setup(arch, N, HW)
    ref64 = copy.deepcopy(ref).double()
    ex.train_step(x, t)
    out = ref(x)
    F.cross_entropy(out, t).backward()
    F.cross_entropy(ref64(x.double()), t).backward()
    torch.cuda.synchronize()
    print(f"== {arch} N={N} HW={HW}")
    for (n, p), (_, p2), (_, p3) in zip(model.named_parameters(), ref.named_parameters(), ref64.named_parameters()):
        ours, theirs = _rel(p.grad, p3.grad), _rel(p2.grad, p3.grad)
        flag = " <<<" if ours > 3 * theirs + 1e-4 else ""
        print(f"{n:40s} ours {ours:.2e} torch32 {theirs:.2e}{flag}")


def intermediates(arch="resnet50", N=4, HW=64):
    """Forward error progression (stem output and every block output) of the fp32 executor and of torch fp32,
    both vs an fp64 torch forward of the same weights."""
    model, ref, flat, ex, x, t = _setup(arch, N, HW)
    ref64 = copy.deepcopy(ref).double()
    box = {}
    orig = ex._backward

    def keep(saved, dlog):
        box["saved"] = saved
        return orig(saved, dlog)
    ex._backward = keep
    a64, a32 = {}, {}

    def hook(store, name):
        return lambda m, i, o: store.__setitem__(name, o.detach())
    hs = []
    for store, net in ((a64, ref64), (a32, ref)):
        hs.append(net.maxpool.register_forward_hook(hook(store, "x0")))
        hs.append(net.conv1.register_forward_hook(hook(store, "y0")))
        for li, layer in enumerate((net.layer1, net.layer2, net.layer3, net.layer4)):
            for bi, blk in enumerate(layer):
                hs.append(blk.register_forward_hook(hook(store, f"l{li + 1}.{bi}")))
    ex.train_step(x, t)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref64(x.double())
        ref(x)
    sv = box["saved"]
    nhwc = lambda a: a.permute(0, 2, 3, 1).reshape(-1)
    print(f"y0    ours {_rel(sv['y0'], nhwc(a64['y0'])):.2e}  torch32 {_rel(a32['y0'], a64['y0']):.2e}")
    print(f"x0    ours {_rel(sv['x0'], nhwc(a64['x0'])):.2e}  torch32 {_rel(a32['x0'], a64['x0']):.2e}")
    k = 0
    for li, layer in enumerate((ref64.layer1, ref64.layer2, ref64.layer3, ref64.layer4)):
        for bi in range(len(layer)):
            nm = f"l{li + 1}.{bi}"
            print(f"{nm:5s} ours {_rel(sv['blocks'][k]['out'], nhwc(a64[nm])):.2e}  torch32 {_rel(a32[nm], a64[nm]):.2e}")
            k += 1
    last = sv["blocks"][-1]["out"]
    ref_out = nhwc(a64[f"l4.{len(ref64.layer4) - 1}"])
    flips = ((last > 0) != (ref_out > 0)).nonzero().flatten()
    print(f"last block ReLU-mask disagreements vs fp64: {flips.numel()} "
          f"(values ours / fp64: {[(float(last[i]), float(ref_out[i])) for i in flips[:4]]})")
    for h in hs:
        h.remove()


if __name__ == "__main__" and len(sys.argv) == 1:
    intermediates()
