"""Bandwidth of the BatchNorm elementwise passes (bn_apply / bn_bwd_apply) at ResNet shapes, B = 1200.

    python tools/ew_bench.py [--so A.so B.so ...]   # one subprocess per build of the extension (PDT_NATIVE_SO)

(Round 5 chose 4 vectors per thread with this script: csrc/kernels/bn.hip kEwU.)

Prints one JSON line per (U, pass, shape): microseconds and TB/s of the bytes the pass must move.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import torch
    sys.path.insert(0, ROOT)
    from pytorch_distributed_template_amd.ops import native
    C_ = native.C
    dev = "cuda"
    N = 1200
    shapes = [(56, 64), (56, 256), (28, 128), (14, 256), (7, 512), (7, 2048)]
    out = []

    def timeit(fn, reps=10):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    for hw, c in shapes:
        n = N * hw * hw * c
        y = torch.randn(n, device=dev).to(torch.bfloat16)
        r = torch.randn(n, device=dev).to(torch.bfloat16)
        o = torch.empty_like(y)
        o2 = torch.empty_like(y)
        m = torch.empty(n // 8, dtype=torch.uint8, device=dev)
        coef = torch.rand(4 * c, device=dev)
        bc = torch.rand(3 * c, device=dev)
        cases = {
            "apply_relu": (lambda: C_.bn_apply(y, coef, None, None, o, c, 0, True, None), 4),
            "apply_res_relu_mask": (lambda: C_.bn_apply(y, coef, r, None, o, c, 1, True, m), 6.125),
            "apply_bnres_relu_mask": (lambda: C_.bn_apply(y, coef, r, coef, o, c, 2, True, m), 6.125),
            "bwd_apply": (lambda: C_.bn_bwd_apply(y, None, r, bc, o, None, None, None, None, c), 6),
            "bwd_apply_mask_dz": (lambda: C_.bn_bwd_apply(y, m, r, bc, o, None, None, None, o2, c), 8.125),
            "bwd_apply_2br": (lambda: C_.bn_bwd_apply(y, m, r, bc, o, r, bc, o2, None, c), 10.125),
        }
        for name, (fn, bpe) in cases.items():
            us = timeit(fn)
            out.append({"so": os.environ.get("PDT_NATIVE_SO", "in-tree"), "pass": name, "hw": hw, "C": c, "us": round(us, 1),
                        "TB_s": round(bpe * n / us / 1e6, 2)})
            print(json.dumps(out[-1]), flush=True)
        del y, r, o, o2, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", nargs="+", default=[""])
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    for so in a.so:
        env = dict(os.environ)
        if so:
            env["PDT_NATIVE_SO"] = so
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
