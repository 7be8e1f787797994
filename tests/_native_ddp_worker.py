"""Rank script for tests/test_ddp_numerics_gpu.py: native-executor DDP (optionally SyncBN) over gloo with
every rank on cuda:0 (RCCL refuses two ranks on one GPU).  Rank 0 saves parameters, buffers and metrics
after the configured number of steps to $PDT_TEST_OUT.  Not collected by pytest (leading underscore)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from _ddp_common import make_batch, make_model  # noqa: E402
from pytorch_distributed_template_amd.engine.native_trainer import NativeTrainer  # noqa: E402


def main():
    backend = os.environ.get("PDT_TEST_BACKEND", "gloo")
    comm = os.environ.get("PDT_TEST_COMM", "torch")
    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    B = int(os.environ["PDT_TEST_B"])
    hw = int(os.environ.get("PDT_TEST_HW", "224"))
    steps = int(os.environ.get("PDT_TEST_STEPS", "1"))
    sync_bn = os.environ.get("PDT_TEST_SYNCBN", "0") == "1"
    # ranks start from different weights: the constructor broadcast must equalise them
    model = make_model(seed=0 if rank == 0 else rank + 100)
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[os.environ.get("PDT_TEST_DTYPE", "bf16")]
    tr = NativeTrainer(model, dev, dtype=dtype, sync_bn=sync_bn, bucket_cap_mb=4, comm=comm,
                       comm_timeout_s=300.0)
    local = None
    init = tr.flat.data.clone()
    if os.environ.get("PDT_TEST_SAVE_LOCAL") == "1":  # diagnostics: each bucket's local gradient before its all-reduce
        local = torch.zeros_like(tr.flat.grad)
        bk = tr.bucketer
        orig = bk.grad_ready
        pending = {b["id"]: len(b["params"]) for b in bk.buckets}

        def grad_ready(pid):
            b = bk.buckets[bk.bucket_of[pid]]
            pending[b["id"]] -= 1
            if pending[b["id"]] == 0:
                torch.cuda.synchronize()
                local[b["lo"]:b["hi"]].copy_(tr.flat.grad[b["lo"]:b["hi"]])
                torch.cuda.synchronize()
                pending[b["id"]] = len(b["params"])
            orig(pid)
        bk.grad_ready = grad_ready
        tr.executor._user_grad_ready = grad_ready
    X, T = make_batch(B * world, hw)
    x = X[rank * B:(rank + 1) * B].to(dev)
    t = T[rank * B:(rank + 1) * B].to(dev)
    mets = []
    for _ in range(steps):
        _, met = tr.train_step(x, t)
        mets.append(met.clone())
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    if local is not None or os.environ.get("PDT_TEST_SAVE_RANKS") == "1":
        torch.save({"local": local.cpu() if local is not None else None, "grad": tr.flat.grad.cpu(),
                    "init": init.cpu(), "data": tr.flat.data.cpu(), "fbuf": tr.buffers.fdata.cpu()},
                   os.environ["PDT_TEST_OUT"] + f".r{rank}")
    if rank == 0:
        torch.save({"data": tr.flat.data.cpu(), "fbuf": tr.buffers.fdata.cpu(), "ibuf": tr.buffers.idata.cpu(),
                    "met": torch.stack(mets).cpu(), "buckets": len(tr.bucketer.buckets),
                    "grad": tr.flat.grad.cpu(), "bucketer": type(tr.bucketer).__name__,
                    "transport": tr.ncomm.transport if tr.ncomm is not None else None},
                   os.environ["PDT_TEST_OUT"])
    from pytorch_distributed_template_amd.ops import validate
    v = validate.validator()
    if v is not None:  # PDT_VALIDATE runs (bench.py / pytest under PDT_VALIDATE=1): report replay-determinism findings of this rank
        print(f"[rank {rank}] validator: {v.replayed} launches replayed, {len(v.findings)} findings", flush=True)
        for f in v.findings:
            print(f"[rank {rank}] NONDETERMINISTIC: {f}", flush=True)
    dist.barrier()
    if tr.ncomm is not None:
        tr.ncomm.barrier()
        tr.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
