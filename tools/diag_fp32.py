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
    """Compare the fp32 executor's saved forward tensors of the last block with an fp64 torch forward."""
    model, ref, flat, ex, x, t = _setup(arch, N, HW)
    ref64 = copy.deepcopy(ref).double()
    box = {}
    orig = ex._backward

    def keep(saved, dlog):
        box["saved"] = saved
        box["dlog"] = dlog.clone()
        return orig(saved, dlog)
    ex._backward = keep
    acts = {}
    blk = ref64.layer4[-1]
    hooks = [blk.register_forward_hook(lambda m, i, o: acts.__setitem__("out", o)),
             blk.register_forward_hook(lambda m, i, o: acts.__setitem__("in", i[0])),
             blk.bn3.register_forward_hook(lambda m, i, o: acts.__setitem__("y3", i[0])),
             blk.bn2.register_forward_hook(lambda m, i, o: acts.__setitem__("y2", i[0]))]
    ex.train_step(x, t)
    torch.cuda.synchronize()
    ref64(x.double())
    rec = box["saved"]["blocks"][-1]
    nhwc = lambda a: a.permute(0, 2, 3, 1).reshape(-1)
    print("block in ", _rel(rec["x"], nhwc(acts["in"])))
    print("y2       ", _rel(rec["ys"][1], nhwc(acts["y2"])))
    print("y3       ", _rel(rec["ys"][2], nhwc(acts["y3"])))
    print("out      ", _rel(rec["out"], nhwc(acts["out"])))
    print("feat     ", _rel(box["saved"]["feat"], acts["out"].mean((2, 3)).reshape(-1)))
    for h in hooks:
        h.remove()


if __name__ == "__main__" and len(sys.argv) == 1:
    intermediates()
