"""Validation cost of the reference-precision default: eval images/s of a bf16-trained ResNet-18 evaluated in bf16
(--eval-precision compute) vs in fp32 on the fp32 kernels (--eval-precision auto/fp32), batch 1200 on one GPU, and
the per-epoch cost for the 50,000 ImageNet validation images."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer  # noqa: E402
from pytorch_distributed_template_amd.models import registry  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(1200, 3, 224, 224, device=dev)
    t = torch.randint(0, 1000, (1200,), device=dev)
    out = {}
    for name, e32 in (("bf16", False), ("fp32", True)):
        torch.manual_seed(0)
        tr = NativeTrainer(registry.create("resnet18"), dev, dtype=torch.bfloat16, eval_fp32=e32)
        tr.train_step(x, t)
        for _ in range(3):
            tr.eval_step(x, t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            tr.eval_step(x, t)
        torch.cuda.synchronize()
        ips = 10 * 1200 / (time.perf_counter() - t0)
        out[name] = {"eval_img_per_s": round(ips), "val_epoch_s_50k": round(50000 / ips, 2)}
        del tr
    print(json.dumps(out))


if __name__ == "__main__":
    main()
