"""Probe the one native op the noisy replay check flagged (conv_dgrad_bn, fused block-output BN reduce, 2 branches):
intercept its calls during one ResNet-18 training step (224 px, B = 16), then replay each intercepted call --reps
times from a snapshot of its arguments while another process keeps the GPU busy, and report how often the BN
statistics (the fp64 slots) or the data gradient change.  PDT_SCRATCH_POISON=1 in the environment fills the
kernels' internal scratch with NaN first (unwritten statistics rows then show up as NaN)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from _ddp_common import make_batch, make_model  # noqa: E402
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer  # noqa: E402
from pytorch_distributed_template_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    calls = []
    mod = native.load()
    orig = mod.conv_dgrad_bn

    def spy(*args):
        r = orig(*args)
        torch.cuda.synchronize()
        calls.append(([x.clone() if isinstance(x, torch.Tensor) else x for x in args], args))
        return r
    mod.conv_dgrad_bn = spy
    X, T = make_batch(16, 224)
    tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=torch.bfloat16)
    tr.train_step(X.cuda(), T.cuda())
    torch.cuda.synchronize()
    mod.conv_dgrad_bn = orig
    print(f"intercepted {len(calls)} conv_dgrad_bn calls", flush=True)
    total_bad = 0
    for ci, (snap, live) in enumerate(calls):
        # the op's outputs after its first run are the reference; re-run from the pre-call snapshot is not
        # possible (outputs were captured after), so run twice from the post-call state of the INPUTS: every
        # argument that is an output (dx #2, slots #-2) is overwritten by each run, inputs are unchanged
        args = [x.clone() if isinstance(x, torch.Tensor) else x for x in snap]
        orig(*args)
        torch.cuda.synchronize()
        ref = [x.clone() if isinstance(x, torch.Tensor) else None for x in args]
        bad = {}
        nan = 0
        for _ in range(a.reps):
            orig(*args)
            torch.cuda.synchronize()
            for k, (x, r) in enumerate(zip(args, ref)):
                if isinstance(x, torch.Tensor) and not torch.equal(x.view(-1).view(torch.uint8), r.view(-1).view(torch.uint8)):
                    bad[k] = bad.get(k, 0) + 1
                    if k == 22 and bad[k] <= 3:  # slots [64][C][K]: which slot / channel / quantity moved
                        Kq = 4 if snap[16] == 3 else 2
                        C = x.numel() // (64 * Kq)
                        idx = (x.view(-1) != r.view(-1)).nonzero().view(-1)[:12].tolist()
                        det = [(i // (C * Kq), (i // Kq) % C, i % Kq, float(r.view(-1)[i]), float(x.view(-1)[i]))
                               for i in idx]
                        print(f"   call {ci}: slots (slot, channel, k, before, after): {det}", flush=True)
                    r.copy_(x)
            for x in args:
                if isinstance(x, torch.Tensor) and x.is_floating_point() and not bool(torch.isfinite(x).all()):
                    nan += 1
        shapes = [tuple(x.shape) if isinstance(x, torch.Tensor) else x for x in snap[:3]]
        print(f"call {ci}: mode {snap[16]} dy/derived/dx {shapes}: changed args {bad} over {a.reps} reps, "
              f"non-finite outputs {nan}", flush=True)
        total_bad += sum(bad.values()) + nan
    return 1 if total_bad else 0


if __name__ == "__main__":
    sys.exit(main())
