"""Reproduce the axes of the reference's published table (SURVEY §6 / BASELINE.md) on MI355X.

The reference reports, for ResNet-18 at node batch 1200 on 3x TITAN Xp: GPU memory, 5-epoch wall clock and
Top-1 for DataParallel, DDP, DDP+AMP and DDP+AMP+SyncBN (`README.md:11-14`).  This tool measures the same
configurations with this framework's trainers on the GPUs visible to ONE process (run it under
`python -m pytorch_distributed_template_amd.launch` for multi-rank DDP rows):

* train and eval throughput (synthetic ImageNet-shaped data generated in HBM, random init),
* peak device memory (torch caching-allocator peak, the analogue of the nvidia-smi figure),
* projected 5-epoch wall clock = 5 x (1,281,167 / train img/s + 50,000 / eval img/s) -- training and
  validation compute only (no JPEG decoding: there is no dataset on this machine).

Top-1 needs the real ImageNet and is not measured.  Output: one JSON line per configuration and a
markdown table (``--md PATH``).

    python tools/reference_table.py [--batch 1200] [--steps 10] [--md profiles/reference_table_1gpu.md]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
from pytorch_distributed_template_amd.models import registry
from pytorch_distributed_template_amd.parallel.dp import NativeDataParallelTrainer

TRAIN_IMAGES, VAL_IMAGES = 1281167, 50000
PUBLISHED = {  # README.md:11-14 (3x TITAN Xp, node batch 1200): memory MB, 5-epoch seconds
    "dp": (11329, 7633), "ddp": (11329, 4612), "ddp_amp": (8679, 4680), "ddp_amp_syncbn": (8679, 8173)}


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    return (time.perf_counter() - t0) / steps


def run(mode, batch, steps, warmup, arch):
    world = dist.get_world_size() if dist.is_initialized() else 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    torch.cuda.init()
    torch.manual_seed(0)
    model = registry.create(arch)
    amp = mode.startswith("ddp_amp")
    dtype = torch.float16 if amp else torch.bfloat16
    torch.cuda.reset_peak_memory_stats(dev)
    if mode == "dp":
        ids = list(range(torch.cuda.device_count()))
        tr = NativeDataParallelTrainer(model, ids, dtype=dtype)
        per_rank = batch  # DataParallel scatters the node batch itself
    else:
        tr = NativeTrainer(model, dev, dtype=dtype, use_amp=amp, sync_bn=mode.endswith("syncbn"))
        per_rank = batch // world  # reference semantics: -b is the node total
    g = torch.Generator(device=dev)
    g.manual_seed(1 + local)
    x = torch.randn(per_rank, 3, 224, 224, device=dev, generator=g)
    t = torch.randint(0, 1000, (per_rank,), device=dev, generator=g)
    st = timed(lambda: tr.train_step(x, t), steps, warmup)
    se = timed(lambda: tr.eval_step(x, t), steps, warmup)
    node_train = batch / st
    node_eval = batch / se
    mem = torch.cuda.max_memory_allocated(dev) / 2 ** 20
    res = {"mode": mode, "arch": arch, "world": world, "node_batch": batch, "dtype": str(dtype).split(".")[-1],
           "train_ms_per_step": round(st * 1e3, 2), "train_img_s": round(node_train, 1),
           "eval_img_s": round(node_eval, 1), "peak_mem_mb": round(mem, 1),
           "proj_5epoch_s": round(5 * (TRAIN_IMAGES / node_train + VAL_IMAGES / node_eval), 1),
           "published_mem_mb": PUBLISHED[mode][0], "published_5epoch_s": PUBLISHED[mode][1]}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1200, help="node-total batch (reference -b)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--modes", default="dp,ddp,ddp_amp,ddp_amp_syncbn")
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        torch.cuda.set_device(int(os.environ["LOCAL_RANK"]))
        dist.init_process_group("nccl", device_id=torch.device("cuda", int(os.environ["LOCAL_RANK"])))
    rows = []
    for mode in a.modes.split(","):
        if mode == "dp" and dist.is_initialized():
            continue
        r = run(mode, a.batch, a.steps, a.warmup, a.arch)
        rows.append(r)
        if not dist.is_initialized() or dist.get_rank() == 0:
            print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()
    if a.md and (not dist.is_initialized() or dist.get_rank() == 0):
        with open(a.md, "w") as f:
            f.write(f"# Reference table axes on MI355X ({rows[0]['world'] if rows else 1} rank(s), "
                    f"{torch.cuda.device_count()} visible GPU(s), {a.arch}, node batch {a.batch})\n\n")
            f.write("Synthetic data, random init; projected 5-epoch time = training + validation compute only. "
                    "Published column: 3x TITAN Xp (`README.md:11-14`).\n\n")
            f.write("| method | dtype | train img/s | eval img/s | peak mem (MB) | proj. 5-epoch (s) | "
                    "published mem (MB) | published 5-epoch (s) |\n|---|---|---:|---:|---:|---:|---:|---:|\n")
            for r in rows:
                f.write(f"| {r['mode']} | {r['dtype']} | {r['train_img_s']} | {r['eval_img_s']} | {r['peak_mem_mb']} | "
                        f"{r['proj_5epoch_s']} | {r['published_mem_mb']} | {r['published_5epoch_s']} |\n")
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
