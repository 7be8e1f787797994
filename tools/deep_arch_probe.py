"""Loss / logits deviation of the native bf16 executor vs fp32 torch and vs torch autocast bf16, for deep archs at
small N (diagnostic for tests/test_executor_gpu.py::test_train_step_matches_reference_224)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_executor_gpu import _relnorm, _setup  # noqa: E402

CASES = [("wide_resnet101_2", 2, 0), ("wide_resnet101_2", 2, 1), ("wide_resnet101_2", 4, 0),
         ("resnet152", 2, 0), ("wide_resnet50_2", 3, 0)]
if len(sys.argv) > 1:  # arch:N:seed ...
    CASES = [(a.split(":")[0], int(a.split(":")[1]), int(a.split(":")[2])) for a in sys.argv[1:]]
for arch, N, seed in CASES:
    model, ref, flat, ex, x, t = _setup(arch, N=N, HW=224, dtype=torch.bfloat16, seed=seed)
    tb = copy.deepcopy(ref)
    logits, met = ex.train_step(x, t)
    torch.cuda.synchronize()
    with torch.no_grad():
        out = ref(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ob = tb(x)
    loss, lb = F.cross_entropy(out, t).item(), F.cross_entropy(ob.float(), t).item()
    print(arch, N, seed, f"loss ours {met[0].item():.4f} fp32 {loss:.4f} autocast {lb:.4f}",
          f"logits rel ours {_relnorm(logits, out):.4f} autocast {_relnorm(ob, out):.4f}", flush=True)
    del model, ref, flat, ex, tb
    torch.cuda.empty_cache()
