"""Backward-data epilogue cost per ResNet-18 3x3 stride-1 shape at B=1200.

    python tools/epi_bench.py [--batch 1200] [--reps 5] [--shapes 0,1]

For each shape, times (µs) the same convolution with each epilogue the executor uses:
forward + BN statistics, plain dgrad, dgrad + residual, and the fused BN-backward reduces
(mode 1: ReLU mask from the BN input; mode 2: mask from the block output bitmask + residual;
mode 3: as 2 plus a second BN branch).  The gap to the plain dgrad is the epilogue's price.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_template_amd.ops import conv, native

SHAPES = [(56, 64), (28, 128), (14, 256), (7, 512)]  # H, C (3x3/1/1, Cin == Cout)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="")
    a = ap.parse_args()
    C_ = native.C
    dev = "cuda"
    sel = [int(v) for v in a.shapes.split(",")] if a.shapes else range(len(SHAPES))
    for H, C in [SHAPES[i] for i in sel]:
        N = a.batch
        t = lambda *s: (torch.randn(*s, device=dev) * 0.5).to(torch.bfloat16)
        x, dy, res, y1, y2 = t(N, H, H, C), t(N, H, H, C), t(N, H, H, C), t(N, H, H, C), t(N, H, H, C)
        w = t(C, 3, 3, C) * 0.05
        out = torch.relu(t(N, H, H, C))
        om = conv.pack_relu_mask(out)
        coef = torch.cat([torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3,
                          torch.zeros(C, device=dev), torch.ones(C, device=dev)]).contiguous()
        slots2 = torch.zeros(C_.stat_slots() * C * 2, dtype=torch.float64, device=dev)
        slots4 = torch.zeros(C_.stat_slots() * C * 4, dtype=torch.float64, device=dev)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        bm, bn = conv.conv_tile(C, 9 * C)
        idx = conv.dgrad_weight_index(C, C, 3, 3, [0, 1, 2], [0, 1, 2]).to(dev)
        wt = w.reshape(-1)[idx].contiguous()
        phases = [[0, 0, 3, 3, 1, 1, 0]]
        row = {"shape": [H, C], "tile": [bm, bn]}
        row["fwd_stats"] = timeit(lambda: C_.conv_fwd(x, w, y, None, slots2, N, H, H, C, C, 3, 3, H, H, 1, 1, -1, -1, 1, 1,
                                                      H, H, 1, 1, 0, 0, bm, bn, 64, 0), a.reps)
        row["dgrad"] = timeit(lambda: C_.conv_dgrad(dy, wt, dx, None, N, H, H, C, C, H, H, 1, phases, bm, bn, 64), a.reps)
        row["dgrad_res"] = timeit(lambda: C_.conv_dgrad(dy, wt, dx, res, N, H, H, C, C, H, H, 1, phases, bm, bn, 64),
                                  a.reps)
        row["epi_m1"] = timeit(lambda: C_.conv_dgrad_bn(dy, wt, dx, None, N, H, H, C, C, H, H, 1, phases, bm, bn, 64,
                                                        1, y1, coef, None, None, None, slots2, -1), a.reps)
        row["epi_m2_res"] = timeit(lambda: C_.conv_dgrad_bn(dy, wt, dx, res, N, H, H, C, C, H, H, 1, phases, bm, bn, 64,
                                                            2, y1, coef, None, None, om, slots2, -1), a.reps)
        row["epi_m3_res"] = timeit(lambda: C_.conv_dgrad_bn(dy, wt, dx, res, N, H, H, C, C, H, H, 1, phases, bm, bn, 64,
                                                            3, y1, coef, y2, coef, om, slots4, -1), a.reps)
        row = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in row.items()}
        print(json.dumps(row), flush=True)
        del x, dy, res, y1, y2, out, y, dx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
