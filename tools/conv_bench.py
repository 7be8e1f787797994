"""Per-layer conv kernel timing sweep (ResNet-18 shapes at B=1200) over tile configs.

    python tools/conv_bench.py [--batch 1200] [--reps 5]

Prints TFLOP/s for forward (each supported (BM, BN) tile), backward-data and weight-gradient
(several split targets) of every distinct ResNet-18 conv shape.  Used to pick the per-shape tile table.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_distributed_template_amd.ops import conv, native

SHAPES = [  # H, Cin, Cout, k, stride
    (56, 64, 64, 3, 1), (56, 64, 128, 3, 2), (28, 128, 128, 3, 1), (56, 64, 128, 1, 2),
    (28, 128, 256, 3, 2), (14, 256, 256, 3, 1), (28, 128, 256, 1, 2), (14, 256, 512, 3, 2),
    (7, 512, 512, 3, 1), (14, 256, 512, 1, 2),
]
SHAPES_R50 = [  # ResNet-50 bottleneck 1x1 convs: H, Cin, Cout, k, stride
    (56, 64, 256, 1, 1), (56, 256, 64, 1, 1), (28, 512, 128, 1, 1), (28, 128, 512, 1, 1), (14, 1024, 256, 1, 1),
    (14, 256, 1024, 1, 1), (7, 2048, 512, 1, 1), (7, 512, 2048, 1, 1),
]
FWD_TILES = [(256, 256, 64), (512, 128, 64), (128, 128, 64), (256, 256, 32), (256, 128, 64), (256, 128, 32), (256, 64, 64),
             (128, 64, 64), (64, 128, 64), (256, 64, 32), (128, 128, 32)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps


def stem_bench(C, N, reps):
    """ResNet stem (7x7/2 over the zero-padded NHWC4 image): 1-row windows (BK=32) vs row pairs (BK=64)."""
    dev = "cuda"
    H = W = 224
    P = Q = 112
    Hp = Wp = 230
    xp = (torch.randn(N * Hp * Wp * 4, device=dev) * 0.5).to(torch.bfloat16)
    y = torch.empty(N * P * Q * 64, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(C.stat_slots() * 64 * 2, device=dev, dtype=torch.float64)
    flops = 2.0 * N * P * Q * 64 * 147
    row = {"shape": "stem"}
    w1 = (torch.randn(64 * 7 * 32, device=dev) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(64 * 4 * 64, device=dev) * 0.05).to(torch.bfloat16)
    for stats in (False, True):
        sp = st if stats else None
        tag = "_stats" if stats else ""
        for (bm, bk) in ((256, 32), (128, 32)):
            def f(bm=bm, bk=bk):
                C.conv_fwd(xp, w1, y, None, sp, N, Hp, Wp, 32, 64, 7, 1, P, Q, 2, 2, 0, 0, 1, 0, P, Q, 1, 1, 0, 0,
                           bm, 64, 32, 4)
            row[f"row_{bm}x64x32{tag}"] = round(flops / timeit(f, reps) / 1e9, 1)
        for bm in (256, 128):
            def g(bm=bm):
                C.conv_fwd(xp, w2, y, None, sp, N, Hp, Wp, 64, 64, 4, 1, P, Q, 2, 2, 0, 0, 2, 0, P, Q, 1, 1, 0, 0,
                           bm, 64, 64, 4)
            row[f"pair_{bm}x64x64{tag}"] = round(flops / timeit(g, reps) / 1e9, 1)
        for bpc in (1, 2):
            def h(bpc=bpc):
                C.stem_fwd(xp, w1, y, sp, N, Hp, Wp, P, Q, bpc)
            row[f"stemk_bpc{bpc}{tag}"] = round(flops / timeit(h, reps) / 1e9, 1)
    row["note"] = "TF/s on the true 7x7x3 FLOPs"
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only-stem", action="store_true")
    ap.add_argument("--skip-stem", action="store_true")
    ap.add_argument("--shapes", default="", help="comma-separated indices into SHAPES (default: all)")
    ap.add_argument("--r50", action="store_true", help="ResNet-50 1x1 shapes (SHAPES_R50), forward with statistics")
    ap.add_argument("--stats", action="store_true", help="forward tiles with the BN statistics epilogue (as in training)")
    a = ap.parse_args()
    C = native.C
    dev = "cuda"
    res = []
    if not a.skip_stem:
        stem_bench(C, a.batch, a.reps)
    if a.only_stem:
        return
    table = SHAPES_R50 if a.r50 else SHAPES
    sel = [int(v) for v in a.shapes.split(",")] if a.shapes else range(len(table))
    for (H, ci, co, k, st) in [table[i] for i in sel]:
        pad = k // 2
        N = a.batch
        P = (H + 2 * pad - k) // st + 1
        x = torch.randn(N, H, H, ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(co, k, k, ci, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, P, P, co, device=dev).to(torch.bfloat16)
        y = torch.empty(N, P, P, co, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * N * P * P * co * ci * k * k
        row = {"shape": [H, ci, co, k, st]}
        for (bm, bn, bk) in FWD_TILES:
            if co % bn:
                continue
            sp = torch.zeros(C.stat_slots() * co * 2, dtype=torch.float64, device=dev) if (a.r50 or a.stats) else None

            def f(bm=bm, bn=bn, bk=bk, sp=sp):
                C.conv_fwd(x, w, y, None, sp, N, H, H, ci, co, k, k, P, P, st, st, -pad, -pad, 1, 1, P, P, 1, 1,
                           0, 0, bm, bn, bk, 0)
            row[f"fwd_{bm}x{bn}x{bk}"] = round(flops / timeit(f, a.reps) / 1e9, 1)
        if a.r50:  # forward-with-statistics tiles only; + the best tile's effective HBM rate (x + w + y bytes)
            best = max(v for kk, v in row.items() if kk.startswith("fwd_"))
            nbytes = 2.0 * (N * H * H * ci + co * k * k * ci + N * P * P * co)
            row["best_TBps"] = round(best * 1e12 / flops * nbytes / 1e12, 2)
            row["best_us"] = round(flops / (best * 1e12) * 1e6, 1)
            bt = max((kk for kk in row if kk.startswith("fwd_")), key=lambda kk: row[kk])
            bm, bn, bk = (int(v) for v in bt[4:].split("x"))
            row["best_nostats_us"] = round(timeit(lambda: C.conv_fwd(
                x, w, y, None, None, N, H, H, ci, co, k, k, P, P, st, st, -pad, -pad, 1, 1, P, P, 1, 1, 0, 0, bm, bn,
                bk, 0), a.reps) * 1e3, 1)
            row["copy_y_us"] = round(timeit(lambda: y.copy_(dy), a.reps) * 1e3, 1)  # read + write of y's bytes
            row["fill_y_us"] = round(timeit(lambda: y.fill_(1.0), a.reps) * 1e3, 1)  # write-only
            print(json.dumps(row), flush=True)
            continue
        dx = torch.empty(N, H, H, ci, device=dev, dtype=torch.bfloat16)
        pieces, phases, off = [], [], 0
        for ph, pw, rs, ss, ih, iw in conv.dgrad_phases(k, k, st, pad):
            idx = conv.dgrad_weight_index(co, ci, k, k, rs, ss).to(dev)
            if idx.numel():
                pieces.append(w.reshape(-1)[idx])
            phases.append([ph, pw, len(rs), len(ss), ih, iw, off])
            off += idx.numel()
        wt = torch.cat(pieces).contiguous()
        dts = [conv.conv_tile(ci) + (64,)] + [t for t in ((256, 256, 64), (512, 128, 64), (128, 128, 64),
                                                           (256, 128, 32)) if ci % t[1] == 0]
        for bm, bn, bk in dict.fromkeys(dts):
            row[f"dgrad_{bm}x{bn}x{bk}"] = round(flops / timeit(lambda: C.conv_dgrad(
                dy, wt, dx, None, N, P, P, co, ci, H, H, st, phases, bm, bn, bk), a.reps) / 1e9, 1)
        if C.wgrad_3x3c64_supported(ci, co, k, k, H, st, pad):
            blocks = C.wgrad_blocks_3x3c64()
            ws = torch.empty(blocks * 64 * 576, device=dev)
            outw = torch.empty(64 * 576, device=dev)

            def l1():
                C.conv_wgrad_3x3c64(x, dy, ws, N, H, H)
                C.wgrad_reduce(ws, blocks, 64, 576, 576, 64 * 576, outw, 576, 1.0, False)
            row["wgrad_l1"] = round(flops / timeit(l1, a.reps) / 1e9, 1)
        for tb in (256, 512, 1024, 2048, 4096, 8192):
            row[f"wgrad_{tb}"] = round(flops / timeit(lambda tb=tb: conv.conv_wgrad(x, dy, k, k, st, pad, tb), a.reps) / 1e9, 1)
        print(json.dumps(row), flush=True)
        res.append(row)
        del x, w, dy, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
