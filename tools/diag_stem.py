"""Diagnostic: stem conv timing in situ (the executor's own buffers after real training steps) vs on
fresh buffers, to separate kernel speed from memory-state effects.  GPU only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
from pytorch_distributed_template_amd.models import registry


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    tr = NativeTrainer(registry.create("resnet18"), dev, dtype=torch.bfloat16, lr=0.1, momentum=0.9,
                       weight_decay=1e-4)
    B = 1200
    x = torch.randn(B, 3, 224, 224, device=dev)
    t = torch.randint(0, 1000, (B,), device=dev)
    for _ in range(3):
        tr.train_step(x, t)
    torch.cuda.synchronize()
    ex = tr.executor
    C = ex.C
    st = ex.stem
    P0 = Q0 = 112
    Hp = Wp = 230
    xp = ex._buf("stem_in", B * Hp * Wp * 4)
    y0 = ex._buf("y0", B * P0 * Q0 * st.cout)
    wst = ex.derived[ex.stem_w_off:ex.stem_w_off + st.cout * ex.stem_pairs * 64]
    sp = ex._buf(("stats", st.cout), ex.n_slots * st.cout * 2, torch.float64)
    bm, bn = ex.stem_tile
    print("stem_w_off", ex.stem_w_off, "wst ptr % 256", wst.data_ptr() % 256, "xp ptr % 256", xp.data_ptr() % 256,
          "y0 ptr % 256", y0.data_ptr() % 256)

    def run(xp_, w_, y_, sp_):
        return lambda: C.conv_fwd(xp_, w_, y_, None, sp_, B, Hp, Wp, 64, st.cout, ex.stem_pairs, 1, P0, Q0, 2, 2, 0, 0,
                                  2, 0, P0, Q0, 1, 1, 0, 0, bm, bn, 64, 4)

    flops = 2.0 * B * P0 * Q0 * 64 * 147
    us = timeit(run(xp, wst, y0, sp))
    print(f"in-situ buffers: {us:.1f} us  {flops / us / 1e6:.1f} TF/s")
    w2 = wst.clone()
    us = timeit(run(xp, w2, y0, sp))
    print(f"cloned weights: {us:.1f} us")
    xp2 = xp.clone()
    us = timeit(run(xp2, wst, y0, sp))
    print(f"cloned input: {us:.1f} us")
    y2 = torch.empty_like(y0)
    us = timeit(run(xp, wst, y2, sp))
    print(f"fresh output: {us:.1f} us")
    us = timeit(run(xp, wst, y0, None))
    print(f"no stats: {us:.1f} us")
    xr = (torch.randn_like(xp.float()) * 0.5).to(xp.dtype)
    us = timeit(run(xr, wst, y0, sp))
    print(f"random input: {us:.1f} us")
    wr = (torch.randn_like(wst.float()) * 0.05).to(wst.dtype)
    us = timeit(run(xp, wr, y0, sp))
    print(f"random weights: {us:.1f} us")
    # whole train step, for reference
    us = timeit(lambda: tr.train_step(x, t), reps=3)
    print(f"train step: {us / 1e3:.2f} ms")
    us = timeit(run(xp, wst, y0, sp))
    print(f"in-situ again: {us:.1f} us")


if __name__ == "__main__":
    main()
