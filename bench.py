#!/usr/bin/env python
"""Headline benchmark: ResNet-18 DDP training throughput (images/s, whole node) on MI355X.

BASELINE.json metric: "images/sec (node) ResNet-18 DDP bs=1200/GPU at 1/2/4/8 MI355X".
Each rank trains torchvision-layout ResNet-18 (random init) on a synthetic ImageNet-shaped batch
(1200 x 3 x 224 x 224 fp32 + int64 labels per GPU, generated on device) with the full reference
training step: BN buffer broadcast, forward, cross-entropy, top-1 accuracy, metric all-reduce,
backward with bucketed RCCL gradient all-reduce overlapped with backward, SGD(momentum 0.9, wd 1e-4)
step.  Compute dtype bf16 (fp32 master weights / gradients / BN statistics).

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
                 --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.  ``vs_baseline`` divides by the reference's best published node
throughput (DDP, 3x TITAN Xp: 5 x 1,281,167 images / 4612 s = 1389 img/s).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REF_IMG_PER_S = 5 * 1281167 / 4612.0  # BASELINE.md, DDP row (derived from README.md:12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch-per-gpu", type=int, default=1200)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--sync-bn", action="store_true")
    ap.add_argument("--bucket-cap-mb", type=float, default=25.0)
    ap.add_argument("--last-bucket-mb", type=float, default=1.0,
                    help="last-produced gradient bucket (the only all-reduce not overlapped with backward); <= 0: "
                         "DDP's first-bucket policy")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--graph", action="store_true", help="replay the training step as a captured HIP graph")
    ap.add_argument("--autotune", action="store_true", help="time every conv tile candidate once per shape")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the benchmark) or gloo (multi-rank rehearsal on fewer GPUs than ranks)")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":  # rehearsal: ranks may share a GPU
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    torch.manual_seed(0)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    model = registry.create(args.arch)
    tr = NativeTrainer(model, dev, dtype=dtype, lr=0.1, momentum=0.9, weight_decay=1e-4,
                       use_amp=(args.dtype == "fp16"), sync_bn=args.sync_bn, bucket_cap_mb=args.bucket_cap_mb,
                       graph=args.graph, autotune=args.autotune,
                       last_bucket_mb=args.last_bucket_mb if args.last_bucket_mb > 0 else None)
    B = args.batch_per_gpu
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    batches = [(torch.randn(B, 3, args.image_size, args.image_size, device=dev, generator=g),
                torch.randint(0, 1000, (B,), device=dev, generator=g)) for _ in range(2)]

    def step(i):
        x, t = batches[i % len(batches)]
        return tr.train_step(x, t)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if args.autotune and rank == 0:
        for k, v in tr.executor._tiles.items():
            print("tile", k, v, file=sys.stderr)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    met = None
    for i in range(args.steps):
        _, met = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (node) ResNet-18 DDP bs=1200/GPU at 1/2/4/8 MI355X" if args.arch == "resnet18"
            else f"images/sec (node) {args.arch} DDP bs={B}/GPU",
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / REF_IMG_PER_S, 3), "dtype": args.dtype, "data": "synthetic",
            "config": {"model": args.arch, "global_batch": B * world, "seq_len": None,
                       "image": [3, args.image_size, args.image_size], "parallelism": f"dp{world}",
                       "per_gpu_batch": B, "sync_bn": args.sync_bn, "engine": "native-hip",
                       "last_loss": round(float(met[0].item()), 4) if met is not None else None}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
