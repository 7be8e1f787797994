"""Stock PyTorch-ROCm (MIOpen/hipBLASLt) ResNet training-step timing: the yardstick our kernels must beat.

Not part of the framework: a measurement tool only.
"""
import argparse, time, json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn
from pytorch_distributed_template_amd.models import registry

p = argparse.ArgumentParser()
p.add_argument("--arch", default="resnet18")
p.add_argument("--bs", type=int, default=1200)
p.add_argument("--steps", type=int, default=10)
p.add_argument("--dtype", default="bf16")
p.add_argument("--benchmark", type=int, default=1, help="cudnn.benchmark (MIOpen search) as the reference sets it")
p.add_argument("--cl", type=int, default=1)
a = p.parse_args()
torch.backends.cudnn.benchmark = bool(a.benchmark)
import threading


def _heartbeat():  # MIOpen's search can stay silent for minutes: keep the run visibly alive
    while True:
        time.sleep(30)
        print("...", flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()
dev = torch.device("cuda:0")
m = registry.create(a.arch).to(dev)
if a.cl:
    m = m.to(memory_format=torch.channels_last)
opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
crit = nn.CrossEntropyLoss()
x = torch.randn(a.bs, 3, 224, 224, device=dev)
if a.cl:
    x = x.to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (a.bs,), device=dev)
dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[a.dtype]
def step():
    with torch.autocast("cuda", dtype=dt, enabled=dt is not None):
        out = m(x)
        loss = crit(out, y)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
for i in range(3):  # warm-up (MIOpen's benchmark-mode search happens here: print progress, it can be long)
    t0 = time.time()
    step()
    torch.cuda.synchronize()
    print(f"warm-up step {i}: {time.time() - t0:.1f} s", flush=True)
t = time.time()
for _ in range(a.steps):
    step()
    torch.cuda.synchronize()
    print(".", end="", flush=True)
print()
el = (time.time() - t) / a.steps
print(json.dumps({"arch": a.arch, "bs": a.bs, "dtype": a.dtype, "channels_last": a.cl, "ms_per_step": el * 1e3,
                  "img_per_s": a.bs / el, "max_mem_GB": torch.cuda.max_memory_allocated() / 1e9}))
