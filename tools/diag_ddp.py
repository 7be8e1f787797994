"""Diagnostic: native DDP (2 ranks x B/2 over gloo on one GPU) vs one process averaging the two halves'
gradients -- per-slot bitwise comparison of the all-reduced gradient, repeated to expose flakiness."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
sys.path.insert(0, os.path.dirname(HERE))
import test_ddp_numerics_gpu as T  # noqa: E402
from _ddp_common import make_batch  # noqa: E402


class _P:
    def __init__(self, d):
        self.d = d

    def __truediv__(self, o):
        return os.path.join(self.d, o)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B = T.B
    X, Tg = make_batch(2 * B, T.HW)
    xa, ta, xb, tb = X[:B].cuda(), Tg[:B].cuda(), X[B:].cuda(), Tg[B:].cuda()
    box = {}

    def steps(tr):
        tr.executor.train_step(xa, ta, grad_div=float(B))
        ga = tr.flat.grad.clone()
        tr.executor.train_step(xb, tb, grad_div=float(B))
        box["ga"], box["gb"] = ga, tr.flat.grad.clone()
        tr.flat.grad.add_(ga)
        box["g"] = tr.flat.grad.clone()

    tr, before = T._single(steps)
    want = box["g"].cpu()
    os.makedirs("/tmp/diag_ddp", exist_ok=True)
    for r in range(reps):
        res = T._run_ranks(_P("/tmp/diag_ddp"), PDT_TEST_SAVE_LOCAL=1)
        r0 = torch.load("/tmp/diag_ddp/rank0.pt.r0", weights_only=True)
        r1 = torch.load("/tmp/diag_ddp/rank0.pt.r1", weights_only=True)

        def cmp(tag, got, ref):
            bad = []
            for s in tr.flat.slots:
                a, b = got[s.offset:s.offset + s.numel], ref[s.offset:s.offset + s.numel]
                if not torch.equal(a, b):
                    bad.append((s.name, int((a != b).sum()), round(((a - b).norm() / b.norm()).item(), 5)))
            print(f"rep {r} {tag}: {len(bad)} slots differ", bad, flush=True)
        cmp("allreduced", res["grad"], want)
        cmp("r0==r1", r0["grad"], r1["grad"])
        cmp("local0 vs ga", r0["local"], box["ga"].cpu())
        cmp("local1 vs gb", r1["local"], box["gb"].cpu())


if __name__ == "__main__":
    main()
