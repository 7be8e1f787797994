"""Streaming bandwidth of the elementwise-kernel structure variants (C.bw_probe): out = 0.5*x + y over
241M bf16 elements (ResNet-18 layer1 activation size at B = 1200), 6 B per element.

    python tools/bw_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_template_amd.ops import native  # noqa: E402

C = native.C
n = 1200 * 56 * 56 * 64
x = torch.randn(n, device="cuda").to(torch.bfloat16)
y = torch.randn(n, device="cuda").to(torch.bfloat16)
o = torch.empty_like(x)
names = {0: "U1", 1: "U2", 2: "U4", 3: "U2 nt-ld nt-st", 4: "U2 nt-st", 5: "U1 nt-st", 6: "U4 nt-st", 7: "U1 nt-ld nt-st"}
for mode in range(8):
    for blocks in (2048, 8192, 32768, 131072):
        for _ in range(2):
            C.bw_probe(mode, x, y, o, blocks)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            C.bw_probe(mode, x, y, o, blocks)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(json.dumps({"variant": names[mode], "blocks": blocks, "us": round(ms * 1e3, 1),
                          "TB_s": round(6 * n / ms / 1e9, 2)}), flush=True)
ref = (0.5 * x.float() + y.float()).to(torch.bfloat16)
C.bw_probe(0, x, y, o, 8192)
torch.cuda.synchronize()
assert torch.equal(o, ref)
print("ok")
