"""Cost of the fused producer BN + ReLU in the layer1 kernels at B=1200.

    python tools/pre_bench.py [--batch 1200] [--reps 5]

Times (µs): bn_apply (the pass the fusion removes), conv_l1 forward with statistics over the activation vs over
the raw producer output with the in-LDS transform, and the 9-tap weight gradient likewise.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_template_amd.ops import native


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1000.0, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1200)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    C, N, H, W = native.C, a.batch, 56, 56
    dev = "cuda"
    z = (torch.randn(N, H, W, 64, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
    coef = torch.cat([torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.3,
                      torch.zeros(128, device=dev)]).contiguous()
    act, y = torch.empty_like(z), torch.empty_like(z)
    dy = torch.randn_like(z, dtype=torch.float32).to(torch.bfloat16)
    st = torch.zeros(C.stat_slots() * 128, dtype=torch.float64, device=dev)
    blocks = C.wgrad_blocks_3x3c64()
    ws = torch.empty(blocks * 64 * 576, device=dev)
    row = {
        "bn_apply": timeit(lambda: C.bn_apply(z, coef, None, None, act, 64, 0, True, None), a.reps),
        "conv_fwd_stats": timeit(lambda: C.conv_fwd(act, w, y, None, st, N, H, W, 64, 64, 3, 3, H, W, 1, 1, -1, -1, 1, 1,
                                                    H, W, 1, 1, 0, 0, 256, 64, 64, 0), a.reps),
        "conv_fwd_pre": timeit(lambda: C.conv_fwd_pre(z, w, y, st, coef, N, H, W), a.reps),
        "wgrad": timeit(lambda: C.conv_wgrad_3x3c64(act, dy, ws, N, H, W), a.reps),
        "wgrad_pre": timeit(lambda: C.conv_wgrad_3x3c64(z, dy, ws, N, H, W, coef), a.reps),
    }
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
