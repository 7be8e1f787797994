"""Diagnostic for the intermittent native-DDP mismatch: run the 2-rank worker (no extra synchronisation) several
times and compare each rank's initial parameters, all-reduced gradient and final parameters with a single-process
oracle (computed once) and with each other."""
import os
import sys
import tempfile

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
    comm = sys.argv[1] if len(sys.argv) > 1 else "native"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    B = T.B
    X, Tg = make_batch(2 * B, T.HW)
    box = {}

    def steps(tr):
        box["init"] = tr.flat.data.clone()
        tr.executor.train_step(X[:B].cuda(), Tg[:B].cuda(), grad_div=float(B))
        box["ga"] = tr.flat.grad.clone()
        tr.executor.train_step(X[B:].cuda(), Tg[B:].cuda(), grad_div=float(B))
        box["gb"] = tr.flat.grad.clone()
        tr.flat.grad.add_(box["ga"])
        tr.optimizer.step(grad_scale=0.5)

    tr, _ = T._single(steps)
    want = {k: v.cpu() for k, v in box.items()}
    slots = tr.flat.slots

    def diff(a, b):
        return [s.name for s in slots if not torch.equal(a[s.offset:s.offset + s.numel], b[s.offset:s.offset + s.numel])]

    for rep in range(reps):
        d = tempfile.mkdtemp()
        T._run_ranks(_P(d), PDT_TEST_SYNCBN=0, PDT_TEST_STEPS=1, PDT_TEST_COMM=comm, PDT_TEST_SAVE_RANKS=1)
        r = [torch.load(os.path.join(d, f"rank0.pt.r{i}"), weights_only=True) for i in range(2)]
        g = want["ga"] + want["gb"]
        dd = diff(r[0]['grad'], g)
        if dd:
            mx = (r[0]['grad'] - g).abs().max().item()
            print(f"   differing slots ({len(dd)}): {dd}  max |diff| {mx:.3e}", flush=True)
        print(f"rep {rep}: init r0 vs oracle {len(diff(r[0]['init'], want['init']))} slots, "
              f"r1 vs r0 {len(diff(r[1]['init'], r[0]['init']))}; grad r0 vs oracle {len(diff(r[0]['grad'], g))} "
              f"{diff(r[0]['grad'], g)[:3]}, r1 vs r0 {len(diff(r[1]['grad'], r[0]['grad']))}; "
              f"grad r0 vs 2*ga {len(diff(r[0]['grad'], 2 * want['ga']))}, vs 2*gb {len(diff(r[0]['grad'], 2 * want['gb']))}",
              flush=True)


if __name__ == "__main__":
    main()
