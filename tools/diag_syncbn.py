"""Diagnostic: per-tensor relative update error of native SyncBN DDP (2 ranks x B/2 over gloo on one GPU)
vs a single process on the full batch, next to non-sync DDP vs the same oracle (the BN-statistics
effect) and the 16-bit rounding floor; per dtype and step count."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
sys.path.insert(0, os.path.dirname(HERE))
import test_ddp_numerics_gpu as T  # noqa: E402
from _ddp_common import make_batch, make_model  # noqa: E402
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer  # noqa: E402


class _P:
    def __init__(self, d):
        self.d = d

    def __truediv__(self, o):
        return os.path.join(self.d, o)


def single(dtype, steps, x, t):
    tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=dtype)
    before = tr.flat.data.clone()
    for _ in range(steps):
        tr.train_step(x, t)
    torch.cuda.synchronize()
    return tr, before.cpu(), tr.flat.data.cpu()


def rel(tr, before, a, b):
    out = {}
    for s in tr.flat.slots:
        da = (a - before)[s.offset:s.offset + s.numel]
        db = (b - before)[s.offset:s.offset + s.numel]
        out[s.name] = ((da - db).norm() / db.norm().clamp_min(1e-12)).item()
    return out


def main():
    tmp = _P("/tmp")
    X, Tt = make_batch(2 * T.B, T.HW)
    x, t = X.cuda(), Tt.cuda()
    for dt_name, dtype in (("fp16", torch.float16), ("bf16", torch.bfloat16)):
        for steps in (1, 2):
            sync = T._run_ranks(tmp, PDT_TEST_SYNCBN=1, PDT_TEST_STEPS=steps, PDT_TEST_DTYPE=dt_name)["data"]
            nos = T._run_ranks(tmp, PDT_TEST_SYNCBN=0, PDT_TEST_STEPS=steps, PDT_TEST_DTYPE=dt_name)["data"]
            tr, before, full = single(dtype, steps, x, t)
            # rounding floor: the full batch with the inputs nudged by one part in 1e6
            _, _, full2 = single(dtype, steps, x * (1 + 1e-6), t)
            rs, rn, rf = rel(tr, before, sync, full), rel(tr, before, nos, full), rel(tr, before, full2, full)
            print(f"== {dt_name} steps={steps}")
            for k in list(rs)[::4] + [list(rs)[-1]]:
                print(f"  {k:28s} sync {rs[k]:.4f}  nosync {rn[k]:.4f}  floor {rf[k]:.4f}")
            print(f"  MAX sync {max(rs.values()):.4f} nosync {max(rn.values()):.4f} floor {max(rf.values()):.4f}",
                  flush=True)


if __name__ == "__main__":
    main()
