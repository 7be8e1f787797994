"""Experiment driver: CLI -> distributed setup -> model/trainer -> epoch loop.

Reference: ``main``/``main_worker``/``train``/``validate`` of `dataparallel.py:76-281`,
`distributed.py:85-334` and `distributed_syncBN_amp.py:88-349`.  One implementation serves the three
entry scripts (``mode`` = ``dp`` | ``ddp`` | ``ddp_amp``); log lines, TensorBoard tags, output files
and checkpoint schema are the reference's.

Per-iteration cross-rank metrics: the reference does ``barrier`` + two scalar all-reduces + ``.item()``
every iteration (`distributed.py:253-257`).  Here the trainer returns ``[loss, acc]`` already averaged
over ranks by ONE all-reduce, accumulated on device, and read on the host only at print iterations
(``--strict-sync`` restores the per-iteration barrier and host read for timing parity).
The printed running averages are identical either way.
"""
from __future__ import annotations

import datetime
import functools
import os
import random
import sys
import time
import warnings
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import cli
from ..data.loader import build_loaders
from ..models import registry
from ..models.inception import AUX_LOSS_WEIGHT
from ..optim.lr import build_scheduler
from ..utils.io import load_checkpoint, make_checkpoint_state, output_process, save_checkpoint, write_settings
from ..utils.logging import close_logger, ddp_print, get_logger
from ..utils.meters import AverageMeter, get_learning_rate
from ..utils.profiling import roctx_range
from ..utils.tensorboard import SummaryWriter

_VGG_ARCHS = ("vgg11", "vgg11_bn", "vgg13", "vgg13_bn", "vgg16", "vgg16_bn", "vgg19", "vgg19_bn", "alexnet")
NATIVE_ARCHS = ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "wide_resnet50_2", "wide_resnet101_2",
                "resnext50_32x4d", "resnext101_32x8d", "resnext101_64x4d") + _VGG_ARCHS
# 16-bit executors only (VGG and AlexNet: models/executor_vgg.py); fp32 runs them on the torch engine.  (Grouped convs
# run in both precisions: models/executor.py and models/executor32.py channel slices.)
NATIVE_ARCHS_16BIT_ONLY = _VGG_ARCHS


def seed_everything(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def resolve_precision(args, device: torch.device) -> torch.dtype:
    p = args.precision
    if p == "auto":
        if device.type != "cuda":
            p = "fp32"
        elif getattr(args, "use_amp", False):
            p = "fp16"
        else:
            p = "bf16"
    return {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[p]


def resolve_engine(args, device: torch.device, dtype: torch.dtype) -> str:
    e = args.engine
    native_ok = device.type == "cuda" and args.arch in NATIVE_ARCHS and dtype in (torch.bfloat16, torch.float16,
                                                                                  torch.float32)
    if args.arch in NATIVE_ARCHS_16BIT_ONLY and dtype == torch.float32:
        native_ok = False
    if e == "auto":
        return "native" if native_ok else "torch"
    if e == "native" and not native_ok:
        raise ValueError(f"--engine native needs a GPU and a supported arch ({', '.join(NATIVE_ARCHS)}) "
                         f"(got device={device.type}, arch={args.arch}, dtype={dtype})")
    return e


class _DeviceMeter:
    """Batch-size weighted running mean of the device-side [loss, acc] pair without host syncs."""

    def __init__(self, device):
        self.sum = torch.zeros(2, dtype=torch.float64, device=device)
        self.count = 0

    def update(self, met: torch.Tensor, n: int) -> None:
        self.sum += met.double() * n
        self.count += n

    def avg(self):
        if self.count == 0:
            return 0.0, 0.0
        a = (self.sum / self.count).tolist()
        return a[0], a[1]


@functools.lru_cache(maxsize=None)
def _fault_spec():
    """``PDT_FAULT_INJECT=rank:iteration[:exit|hang[:epoch]]`` -- the fault-injection hook of SURVEY §5 ("kill rank k
    at step s"): global rank ``rank`` dies (``exit``: status 13 without any teardown, like a crashed process) or
    stops making progress forever (``hang``: the other ranks block in the next collective until ``--dist-timeout``
    / the comm watchdog fires) when it reaches training iteration ``iteration`` of epoch ``epoch`` (default 0).
    Used by tests/test_distributed_cpu.py to check that the group is torn down instead of hanging."""
    spec = os.environ.get("PDT_FAULT_INJECT")
    if not spec:
        return None
    f = spec.split(":")
    return int(f[0]), int(f[1]), (f[2] if len(f) > 2 else "exit"), (int(f[3]) if len(f) > 3 else 0)


def _maybe_inject_fault(rank: int, epoch: int, it: int) -> None:
    spec = _fault_spec()
    if spec is None or (rank, it, epoch) != (spec[0], spec[1], spec[3]):
        return
    sys.stderr.write(f"[fault injection] rank {rank}: {spec[2]} at epoch {epoch} iteration {it}\n")
    sys.stderr.flush()
    if spec[2] == "hang":
        while True:
            time.sleep(3600)
    os._exit(13)


def train_epoch(loader, trainer, epoch: int, args, logger, writer, rank: int, device):
    batch_times = AverageMeter("Time", ":6.3f")
    data_times = AverageMeter("Data", ":6.3f")
    meter = _DeviceMeter(device)
    n_iter = len(loader)
    if args.iters_per_epoch:
        n_iter = min(n_iter, args.iters_per_epoch)
    lr = get_learning_rate(trainer.optimizer)
    end = t_start = time.time()
    seen = 0
    for i, (images, target) in enumerate(loader):
        if i >= n_iter:
            break
        data_times.update(time.time() - end)
        _maybe_inject_fault(rank, epoch, i)
        if not getattr(trainer, "host_batches", False):  # native DP: ShardedBatch, shard i already on GPU i
            images = images.to(device, non_blocking=True)
            target = target.to(device, non_blocking=True)
        with roctx_range("train_step", args.profile):
            _, met = trainer.train_step(images, target)
        meter.update(met, images.size(0))
        seen += images.size(0)
        if args.strict_sync:
            if dist.is_initialized():
                dist.barrier()
            met.tolist()
        batch_times.update(time.time() - end)
        end = time.time()
        if i % args.print_freq == 0:
            loss_avg, acc_avg = meter.avg()
            ddp_print("Train epoch: [{:d}/{:d}][{:d}/{:d}]\tlr={:.6f}\tce_loss={:.4f}\ttop1_acc={:.4f}\tdata_time={:6.3f}s"
                      "\tbatch_time={:6.3f}s".format(epoch, args.epochs, i, n_iter, lr, loss_avg, acc_avg,
                                                     data_times.avg, batch_times.avg), logger, rank)
    loss_avg, acc_avg = meter.avg()
    ddp_print("||==> Train epoch: [{:d}/{:d}]\tlr={:.6f}\tce_loss={:.4f}\ttop1_acc={:.4f}\tbatch_time={:6.3f}s"
              .format(epoch, args.epochs, lr, loss_avg, acc_avg, batch_times.avg), logger, rank)
    if args.profile:
        world = dist.get_world_size() if dist.is_initialized() else 1
        ddp_print("||==> Train throughput: {:.1f} img/s (node, {} ranks)".format(
            seen * world / max(time.time() - t_start, 1e-9), world), logger, rank)
    if rank == 0 and writer is not None:
        writer.add_scalar("lr", lr, epoch)
        writer.add_scalar("Train_ce_loss", loss_avg, epoch)
        writer.add_scalar("Train_top1_accuracy", acc_avg, epoch)
    return loss_avg, acc_avg


def validate(loader, trainer, epoch: int, args, logger, writer, rank: int, device) -> float:
    batch_times = AverageMeter("Time", ":6.3f")
    meter = _DeviceMeter(device)
    n_iter = len(loader)
    if args.val_iters:
        n_iter = min(n_iter, args.val_iters)
    end = time.time()
    with torch.no_grad():
        for i, (images, target) in enumerate(loader):
            if i >= n_iter:
                break
            if not getattr(trainer, "host_batches", False):
                images = images.to(device, non_blocking=True)
                target = target.to(device, non_blocking=True)
            with roctx_range("eval_step", args.profile):
                _, met = trainer.eval_step(images, target)
            meter.update(met, images.size(0))
            if args.strict_sync:
                if dist.is_initialized():
                    dist.barrier()
                met.tolist()
            batch_times.update(time.time() - end)
            end = time.time()
            if i % args.print_freq == 0:
                loss_avg, acc_avg = meter.avg()
                ddp_print("Val epoch: [{:d}/{:d}][{:d}/{:d}]\tce_loss={:.4f}\ttop1_acc={:.4f}\tbatch_time={:6.3f}s"
                          .format(epoch, args.epochs, i, n_iter, loss_avg, acc_avg, batch_times.avg), logger, rank)
    loss_avg, acc_avg = meter.avg()
    ddp_print("||==> Val epoch: [{:d}/{:d}]\tce_loss={:.4f}\ttop1_acc={:.4f}\tbatch_time={:6.3f}s"
              .format(epoch, args.epochs, loss_avg, acc_avg, batch_times.avg), logger, rank)
    if rank == 0 and writer is not None:
        writer.add_scalar("Val_ce_loss", loss_avg, epoch)
        writer.add_scalar("Val_top1_accuracy", acc_avg, epoch)
    return acc_avg


def _peak_memory(device, devices=None):
    """(peak allocated, peak reserved) GiB since the last reset, max over ``devices`` (the DP replicas) --
    the memory column of the reference's results table (`README.md:9-14`)."""
    if device.type != "cuda":
        return None
    ids = devices or [device.index if device.index is not None else torch.cuda.current_device()]
    alloc = max(torch.cuda.max_memory_allocated(d) for d in ids) / 2 ** 30
    res = max(torch.cuda.max_memory_reserved(d) for d in ids) / 2 ** 30
    for d in ids:
        torch.cuda.reset_peak_memory_stats(d)
    return alloc, res


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    return world, rank


def build_trainer(mode: str, model, args, device, dtype, engine: str, world: int):
    use_amp = bool(getattr(args, "use_amp", False)) and dtype == torch.float16
    sync_bn = bool(getattr(args, "sync_batchnorm", False))
    common = dict(lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    torch_kw = dict(aux_loss_weight=AUX_LOSS_WEIGHT.get(args.arch, 0.3))
    if mode == "dp":
        if engine == "native":
            from ..parallel.dp import NativeDataParallelTrainer
            ids = list(range(torch.cuda.device_count()))
            if os.environ.get("PDT_DP_DEVICES"):  # rehearsal: e.g. "0,0" = two replicas sharing GPU 0
                ids = [int(v) for v in os.environ["PDT_DP_DEVICES"].split(",")]
            return NativeDataParallelTrainer(model, ids, dtype=dtype, use_amp=use_amp,
                                             eval_fp32=getattr(args, "eval_precision", "auto") in ("fp32", "auto"),
                                             **common)
        from .torch_trainer import TorchTrainer
        # nn.DataParallel semantics on the torch engine too: the node-total batch is scattered over every
        # visible GPU (`dataparallel.py:119`), not run on cuda:0 alone
        ids = list(range(torch.cuda.device_count())) if device.type == "cuda" else []
        return TorchTrainer(model, device, dtype=dtype, use_amp=use_amp, dp_device_ids=ids if len(ids) > 1 else None,
                            **common, **torch_kw)
    kw = dict(common, use_amp=use_amp, sync_bn=sync_bn, bucket_cap_mb=args.bucket_cap_mb,
              first_bucket_mb=args.first_bucket_mb)
    if engine == "native":
        from .native_trainer import NativeTrainer
        lb = float(getattr(args, "last_bucket_mb", 1.0))
        return NativeTrainer(model, device, dtype=dtype, autotune=bool(getattr(args, "autotune", False)),
                             comm=getattr(args, "comm", "native"), graph=bool(getattr(args, "graph", False)),
                             last_bucket_mb=lb if lb > 0 else None,
                             comm_timeout_s=float(getattr(args, "dist_timeout", 0.0)),
                             grad_compress=getattr(args, "grad_compress", "none"),
                             comm_transport=getattr(args, "comm_transport", "auto"),
                             eval_fp32=getattr(args, "eval_precision", "auto") in ("fp32", "auto"), **kw)
    from .torch_trainer import TorchTrainer
    # CPU ranks: --comm native routes buckets / buffer broadcasts / metrics through the C++ communicator and bucketer
    # over the host shared-memory transport (on GPUs the torch engine keeps c10d, whose RCCL it already set up)
    # (single node only: the host transport is one shared-memory segment; multi-node CPU runs keep c10d / gloo)
    from ..parallel.comm import single_node
    tcomm = getattr(args, "comm", "native") if device.type == "cpu" and single_node(world) else "torch"
    return TorchTrainer(model, device, dtype=dtype, comm=tcomm, comm_timeout_s=float(getattr(args, "dist_timeout", 0.0)),
                        **kw, **torch_kw)


def main(mode: str, argv: Optional[list] = None) -> int:
    args = cli.parse_args(mode, argv)
    if args.use_gpus_flag and "HIP_VISIBLE_DEVICES" not in os.environ:
        os.environ["HIP_VISIBLE_DEVICES"] = args.gpus
    if args.seed is not None:
        seed_everything(args.seed)
        # Native engine: every kernel (BN statistics included: per-block partial rows reduced in a fixed order)
        # is deterministic, so a seeded run repeats bit for bit (tests/test_ddp_numerics_gpu.py) -- unless
        # --autotune picks conv tiles by timing.  The stock-PyTorch engine keeps cuDNN/MIOpen's caveat.
        warnings.warn("You have chosen to seed training. The native engine is deterministic (bitwise repeatable "
                      "unless --autotune picks tiles by timing); the torch engine may still pick "
                      "nondeterministic MIOpen algorithms, which can slow down training.")
    args.outpath = args.outpath + "_" + args.arch
    world, rank = (1, 0) if mode == "dp" else _dist_env()
    local_rank = getattr(args, "local_rank", 0) if mode != "dp" else 0
    if mode != "dp":
        local_rank = int(os.environ.get("LOCAL_RANK", local_rank))
        args.local_rank = local_rank
    logger = writer = None
    if rank == 0:
        output_process(args.outpath, args.exist_policy)
        logger = get_logger(args.outpath, cli.ENTRY_DEFAULTS[mode]["logger"])
        if args.tensorboard:
            writer = SummaryWriter(args.outpath)

    on_gpu = torch.cuda.is_available()
    distributed = mode != "dp" and world > 1
    if on_gpu:
        torch.cuda.set_device(local_rank if mode != "dp" else 0)
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    dtype = resolve_precision(args, device)
    engine = resolve_engine(args, device, dtype)
    if distributed:
        # native engine + native communicator: every GPU collective goes through our RCCL communicator, so the
        # process group is only the rendezvous store (+ CPU barriers): gloo, not a second RCCL communicator
        native_comm = engine == "native" and getattr(args, "comm", "native") == "native"
        backend = args.dist_backend if args.dist_backend != "auto" else (
            "nccl" if on_gpu and not native_comm else "gloo")
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device, timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
    args.nprocs = world if mode != "dp" else max(1, torch.cuda.device_count() if on_gpu else 1)

    if rank == 0:
        write_settings(args)
        logger.info(args)

    if args.pretrained:
        ddp_print("=> using pre-trained model: {}".format(args.arch), logger, rank)
    else:
        ddp_print("=> creating model: {}".format(args.arch), logger, rank)
    model = registry.create(args.arch, pretrained=args.pretrained, pretrained_path=args.pretrained_path,
                            num_classes=args.num_classes,
                            **registry.resolution_kwargs(args.arch, getattr(args, "image_size", None) or 224))
    if mode == "ddp_amp":
        if distributed and args.sync_batchnorm:
            ddp_print("=> using sync BN", logger, rank)
        else:
            ddp_print("=> not use sync BN", logger, rank)
    if mode != "dp":
        args.batch_size = int(args.batch_size / args.nprocs)

    ddp_print("=> engine: {} | compute dtype: {} | device: {} | world: {}".format(engine, str(dtype).split(".")[-1],
                                                                                device, world), logger, rank)
    trainer = build_trainer(mode, model, args, device, dtype, engine, world)
    optimizer = trainer.optimizer
    gn = getattr(args, "gpu_normalize", "off")
    if device.type != "cuda" or gn == "off" or (gn == "auto" and engine != "native"):
        args.gpu_normalize_mode = "off"
    else:
        args.gpu_normalize_mode = "native" if engine == "native" else "torch"
    lr_scheduler = build_scheduler(args.lr_scheduler, optimizer, args.step, args.gamma)
    ddp_print("lr_scheduler: SGD MultiStepLR !!!", logger, rank)

    shard_devices = [f"cuda:{i}" for i in trainer.device_ids] if getattr(trainer, "host_batches", False) else None
    train_loader, val_loader, train_sampler, val_sampler = build_loaders(args, world, rank, device, distributed,
                                                                         args.batch_size, shard_devices=shard_devices)
    best_acc1, best_acc1_index = 0.0, 0
    start_epoch = args.start_epoch
    if args.resume:
        ck = load_checkpoint(args.resume)
        trainer.model.load_state_dict(ck["state_dict"])
        trainer.on_state_loaded()  # 16-bit shadows + derived kernel weight layouts of every replica
        if "optimizer" in ck:
            optimizer.load_state_dict(ck["optimizer"])
        if "scaler" in ck:
            trainer.scaler.load_state_dict(ck["scaler"])
        start_epoch = int(ck["epoch"])
        best_acc1 = float(ck.get("best_acc1", 0.0))
        best_acc1_index = int(ck.get("best_acc1_index", 0))
        ddp_print("=> resumed from {} (epoch {})".format(args.resume, start_epoch), logger, rank)

    try:
        rc = _run_epochs(args, trainer, optimizer, lr_scheduler, train_loader, val_loader, train_sampler, val_sampler,
                         start_epoch, best_acc1, best_acc1_index, mode, logger, writer, rank, device)
    except BaseException:
        # no collective teardown is possible once a rank left the epoch loop abnormally: abort the native
        # communicators (pending RCCL work is cancelled, the watchdog stops) so this rank exits instead of hanging in
        # a collective its peers will never join; the launcher then ends the group
        abort = getattr(trainer, "abort", None)
        if abort is not None:
            abort()
        raise
    _finish(writer, logger, distributed, trainer)
    return rc


def _run_epochs(args, trainer, optimizer, lr_scheduler, train_loader, val_loader, train_sampler, val_sampler,
                start_epoch, best_acc1, best_acc1_index, mode, logger, writer, rank, device) -> int:
    if args.evaluate:
        validate(val_loader, trainer, -1, args, logger, writer, rank, device)
        return 0

    total_start = time.time()
    mem_devices = list(range(torch.cuda.device_count())) if mode == "dp" and device.type == "cuda" else None
    _peak_memory(device, mem_devices)  # reset: report per-epoch peaks
    for epoch in range(start_epoch, args.epochs):
        if train_sampler is not None:
            train_sampler.set_epoch(epoch)
        if val_sampler is not None:
            val_sampler.set_epoch(epoch)
        epoch_start = time.time()
        lr_scheduler.step(epoch)
        train_epoch(train_loader, trainer, epoch, args, logger, writer, rank, device)
        acc1 = validate(val_loader, trainer, epoch, args, logger, writer, rank, device)
        is_best = acc1 > best_acc1
        if is_best:
            best_acc1_index = epoch
            best_acc1 = acc1
        epoch_end = time.time()
        ddp_print("||==> Epoch=[{:d}/{:d}]\tbest_acc1={:.4f}\tbest_acc1_index={}\ttime_cost={:.4f}s"
                  .format(epoch, args.epochs, best_acc1, best_acc1_index, epoch_end - epoch_start), logger, rank)
        mem = _peak_memory(device, mem_devices)
        if mem is not None:
            ddp_print("||==> Peak GPU memory: {:.2f} GiB allocated, {:.2f} GiB reserved (per GPU)".format(*mem),
                      logger, rank)
            if rank == 0 and writer is not None:
                writer.add_scalar("Peak_memory_GiB", mem[0], epoch)
        if rank == 0:
            save_checkpoint(make_checkpoint_state(epoch + 1, args.arch, trainer.model, best_acc1, optimizer,
                                                  trainer.scaler, lr_scheduler,
                                                  extra={"best_acc1_index": best_acc1_index}),
                            is_best, args.outpath)
    total_end = time.time()
    ddp_print("||==> total_time_cost={:.4f}s".format(total_end - total_start), logger, rank)
    return 0


def _finish(writer, logger, distributed: bool, trainer=None) -> None:
    """Reference teardown (`distributed_syncBN_amp.py:236-237`: writer close) + collective teardown: every rank passes
    the barrier, then destroys its native communicators (ncclCommDestroy, watchdog stopped) at the same point, then
    the process group."""
    if writer is not None:
        writer.close()
    close_logger(logger)
    if distributed and dist.is_initialized():
        dist.barrier()
    close = getattr(trainer, "close", None)
    if close is not None:
        trace = os.environ.get("PDT_COMM_TRACE") == "1"
        if trace:  # (only the RCCL transport runs a watchdog thread; the host transport times out inside its waits)
            from ..parallel.comm import live_watchdogs
            before = live_watchdogs() if getattr(trainer, "ncomm", None) is not None else 0
        close()
        if trace and getattr(trainer, "ncomm", 1) is None:
            sys.stderr.write(f"[pdt comm] rank {dist.get_rank() if dist.is_initialized() else 0}: trainer closed, "
                             f"live watchdogs {before} -> {live_watchdogs()}\n")
            sys.stderr.flush()
    if distributed and dist.is_initialized():
        dist.destroy_process_group()
