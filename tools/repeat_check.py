"""Bitwise repeatability probe: N identically seeded native trainers (ResNet-18, 224 px, B = 16, 3 steps each) in
one process must end with bit-identical fp32 parameters.

    python tools/repeat_check.py [--reps 6]          (PDT_WGRAD_STREAM=0: single-stream schedule)
    python tools/repeat_check.py --replay [--steps 2] (intra-kernel race detector: PDT_VALIDATE=3 re-runs every
                                                      native op from a snapshot of its arguments and reports any op
                                                      whose bits change, plus gradient guard bands; exit 1 on a finding)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--replay" in sys.argv:  # must precede the first native-op access
    os.environ.update(PDT_VALIDATE="3", PDT_VALIDATE_COLLECT="1", PDT_VALIDATE_GUARD="64")
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from _ddp_common import make_batch, make_model  # noqa: E402
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--poison", action="store_true",
                    help="before every trainer: fill the caching allocator's free memory with 0xFF bytes (NaN), "
                         "so a read of memory no kernel wrote shows up as a difference")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--replay", action="store_true", help="PDT_VALIDATE=3 replay-determinism + guard-band run")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    if a.replay:
        return replay(a)
    X, T = make_batch(16, 224)
    x, t = X.cuda(), T.cuda()
    ref, bad = None, 0
    for rep in range(a.reps):
        if a.poison and rep > 0:
            torch.cuda.empty_cache()
            big = torch.full((6 * 2 ** 30 // 4,), -1, dtype=torch.int32, device="cuda")
            small = [torch.full((128 * 1024,), -1, dtype=torch.int32, device="cuda") for _ in range(1024)]
            torch.cuda.synchronize()
            del big, small
        tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=torch.bfloat16)
        for _ in range(a.steps):
            tr.train_step(x, t)
        torch.cuda.synchronize()
        d = tr.flat.data.clone()
        del tr
        ref = d if ref is None else ref
        eq = torch.equal(d, ref)
        bad += not eq
        print("rep", rep, "equal", eq, "maxdiff", (d - ref).abs().max().item(), flush=True)
    return 1 if bad else 0


def replay(a) -> int:
    from pytorch_distributed_template_amd.ops import validate
    X, T = make_batch(a.batch, 224)
    x, t = X.cuda(), T.cuda()
    tr = NativeTrainer(make_model(seed=0), "cuda:0", dtype=torch.bfloat16)
    for s in range(a.steps):
        tr.train_step(x, t)
        torch.cuda.synchronize()
        v = validate.validator()
        print(f"step {s}: {v.replayed} op launches replayed x{v.replays}, findings {len(v.findings)}", flush=True)
    tr.eval_step(x, t)
    torch.cuda.synchronize()
    v = validate.validator()
    for f in v.findings:
        print("NONDETERMINISTIC:", f, flush=True)
    print(f"replayed {v.replayed} op launches, {len(v.findings)} nondeterministic, guard bands intact", flush=True)
    return 1 if v.findings else 0


if __name__ == "__main__":
    sys.exit(main())
