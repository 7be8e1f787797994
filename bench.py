#!/usr/bin/env python
"""Headline benchmark: ResNet-18 DDP training throughput (images/s, whole node) on MI355X.

BASELINE.json metric: "images/sec (node) ResNet-18 DDP bs=1200/GPU at 1/2/4/8 MI355X".
Each rank trains torchvision-layout ResNet-18 (random init) on a synthetic ImageNet-shaped batch
(1200 x 3 x 224 x 224 fp32 + int64 labels per GPU, generated on device) with the full reference
training step: BN buffer broadcast, forward, cross-entropy, top-1 accuracy, metric all-reduce,
backward with bucketed RCCL gradient all-reduce overlapped with backward, SGD(momentum 0.9, wd 1e-4)
step.  Compute dtype bf16 (fp32 master weights / gradients / BN statistics).

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python bench.py --gpus N ...       (spawns N ranks itself through our launcher), or
             python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
                 --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.  ``vs_baseline`` divides by the reference's best published node
throughput (DDP, 3x TITAN Xp: 5 x 1,281,167 images / 4612 s = 1389 img/s).

Collectives (``--comm``): ``native`` (default) = this framework's own RCCL communicator and C++
gradient bucketer on its own HIP stream (csrc/comm.cpp) for EVERY GPU collective of the step, with
torch.distributed (gloo) used only as the rendezvous store; ``torch`` = RCCL through c10d
ProcessGroupNCCL.  After the timed steps the ranks compare fp64 checksums of their parameters
(``params_equal_across_ranks``: DDP replicas must stay bit-identical) and the JSON records the RCCL
communicator size, the gradient bucket layout and the exposed (not overlapped) gradient all-reduce
time per step, measured with HIP events around the bucketer's final wait.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REF_IMG_PER_S = 5 * 1281167 / 4612.0  # BASELINE.md, DDP row (derived from README.md:12)
ROOT = os.path.dirname(os.path.abspath(__file__))


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher environment bench.py spawns them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch-per-gpu", type=int, default=1200)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="compute dtype (fp32: the reference's distributed.py precision, native fp32 MFMA kernels)")
    ap.add_argument("--sync-bn", action="store_true")
    ap.add_argument("--bucket-cap-mb", type=float, default=25.0)
    ap.add_argument("--last-bucket-mb", type=float, default=1.0,
                    help="last-produced gradient bucket (the only all-reduce not overlapped with backward); <= 0: "
                         "DDP's first-bucket policy")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--graph", action="store_true", help="replay the training step as a captured HIP graph")
    ap.add_argument("--autotune", action="store_true", help="time every conv tile candidate once per shape")
    ap.add_argument("--comm", default="native", choices=["native", "torch"],
                    help="native: own RCCL communicator + C++ bucketer; torch: RCCL through c10d")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the native communicator (world of 1) even on a single GPU")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the benchmark) or gloo (multi-rank rehearsal on fewer GPUs than ranks)")
    ap.add_argument("--comm-timeout", type=float, default=900.0, help="native comm watchdog timeout (s)")
    ap.add_argument("--comm-transport", default="auto", choices=["auto", "rccl", "host"],
                    help="native comm transport: rccl (one rank per GPU), host (shared memory; ranks sharing a GPU)")
    ap.add_argument("--grad-compress", default="none", choices=["none", "bf16"],
                    help="native comm: bf16 gradient all-reduce (default none: fp32, the reference's precision)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(args) -> int:
    """``--gpus N`` without a launcher environment: start N ranks through our launcher (before this
    process touches the GPU: device_count() does not initialise it) and exit with their status."""
    import torch
    n_dev = torch.cuda.device_count()
    if args.gpus > n_dev and args.dist_backend != "gloo":
        sys.stderr.write(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {n_dev} "
                         f"(use --dist-backend gloo to rehearse several ranks on fewer GPUs)\n")
        return 2
    cmd = [sys.executable, "-m", "pytorch_distributed_template_amd.launch", f"--nproc_per_node={args.gpus}",
           "--master_addr=127.0.0.1", f"--master_port={_free_port()}", "--no_local_rank",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    # ROCm IPC: hosts whose amdgpu driver only supports dmabuf-based IPC need the non-legacy mode, otherwise RCCL's
    # intra-node transport (and CUDA-tensor sharing between processes) fails with `hipIpcGetMemHandle: invalid
    # argument`.  setdefault: an explicit user setting wins.
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, cwd=ROOT, env=env)


def main() -> int:
    args = _parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            return _spawn(args)
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks\n")
            return 2

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer
    from pytorch_distributed_template_amd.models import registry

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    shared_gpus = args.dist_backend == "gloo" and world > torch.cuda.device_count()
    if shared_gpus:
        # rehearsal: ranks share GPUs, so RCCL (which refuses duplicate GPUs) is out; --comm native then runs the
        # SAME C++ communicator + bucketer over the host shared-memory transport (csrc/shm_group.h)
        local_rank %= torch.cuda.device_count()
    comm = args.comm
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if comm == "native" or args.dist_backend == "gloo":
            # rendezvous store (+ CPU collectives); every GPU collective goes through the native comm
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(0)
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    model = registry.create(args.arch)
    tr = NativeTrainer(model, dev, dtype=dtype, lr=0.1, momentum=0.9, weight_decay=1e-4,
                       use_amp=(args.dtype == "fp16"), sync_bn=args.sync_bn, bucket_cap_mb=args.bucket_cap_mb,
                       graph=args.graph, autotune=args.autotune, comm=comm, force_comm=args.force_comm,
                       comm_timeout_s=args.comm_timeout, time_comm=True, comm_transport=args.comm_transport,
                       grad_compress=args.grad_compress if comm == "native" else "none",
                       last_bucket_mb=args.last_bucket_mb if args.last_bucket_mb > 0 else None)
    nc = tr.ncomm

    def barrier():
        if nc is not None:
            nc.barrier()
        elif world > 1:
            dist.barrier()

    def all_reduce(t, op):
        if nc is not None:
            nc.all_reduce(t, op)
        elif world > 1:
            dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM}[op])

    # communicator self-test: a rank-dependent all-reduce must give the closed-form sum on every rank
    probe = torch.full((1024,), float(rank + 1), dtype=torch.float32, device=dev)
    all_reduce(probe, "sum")
    comm_ok = bool(torch.all(probe == world * (world + 1) / 2).item())
    if not comm_ok:
        sys.stderr.write(f"bench.py: rank {rank}: communicator self-test FAILED\n")
        return 3

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
    tr.exposed_comm_ms()  # drop the warm-up samples
    if args.autotune and rank == 0:
        for k, v in tr.executor._tiles.items():
            print("tile", k, v, file=sys.stderr)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    met = None
    for i in range(args.steps):
        _, met = step(i)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    all_reduce(el_t, "max")
    el = float(el_t.item())
    exposed = tr.exposed_comm_ms()
    exp_t = torch.tensor([exposed or 0.0], dtype=torch.float64, device=dev)
    all_reduce(exp_t, "max")
    # DDP invariant: replicas stay bit-identical -- compare every rank's checksum with rank 0's
    ck = tr.param_checksum()
    ref = ck.clone()
    if nc is not None and world > 1:
        nc.broadcast(ref, 0)
    elif world > 1:
        dist.broadcast(ref, 0)
    mism = torch.tensor([0.0 if torch.equal(ck, ref) else 1.0], dtype=torch.float64, device=dev)
    all_reduce(mism, "sum")
    params_equal = bool(mism.item() == 0)
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (node) ResNet-18 DDP bs=1200/GPU at 1/2/4/8 MI355X" if args.arch == "resnet18"
            else f"images/sec (node) {args.arch} DDP bs={B}/GPU",
            "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / REF_IMG_PER_S, 3), "dtype": args.dtype,
            "data": "synthetic (on-device random 3x224x224 images + labels, random-init weights)",
            "config": {"model": args.arch, "global_batch": B * world, "seq_len": None,
                       "image": [3, args.image_size, args.image_size], "parallelism": f"dp{world}",
                       "per_gpu_batch": B, "sync_bn": args.sync_bn, "engine": "native-hip",
                       "comm": (comm if world > 1 or nc is not None else "none"),
                       "dist_backend": args.dist_backend if world > 1 else None,
                       "rccl_world": (nc.count() if nc is not None and nc.transport == "rccl" else
                                      (world if world > 1 and nc is None and not shared_gpus else None)),
                       "comm_transport": nc.transport if nc is not None else None,
                       "comm_selftest": comm_ok,
                       "params_equal_across_ranks": params_equal,
                       "bucket_sizes_mb": [round(x, 3) for x in tr.bucketer.bucket_sizes_mb()] if world > 1 else [],
                       "grad_compress": args.grad_compress if comm == "native" else "none",
                       "exposed_comm_ms_per_step": round(float(exp_t.item()), 3) if world > 1 or nc is not None
                       else None,
                       "last_loss": round(float(met[0].item()), 4) if met is not None else None}}), flush=True)
    if world > 1:
        barrier()
    if nc is not None:
        tr.close()
    if world > 1:
        dist.destroy_process_group()
    return 0 if params_equal else 4


if __name__ == "__main__":
    sys.exit(main())
