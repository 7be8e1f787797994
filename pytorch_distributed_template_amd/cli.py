"""Command-line interface shared by the three entry scripts.

Every flag of the reference parsers is accepted with the same spelling, destination and default
for its entry script:

* ``dataparallel.py``          (`dataparallel.py:40-67`)
* ``distributed.py``           (`distributed.py:43-73`)
* ``distributed_syncBN_amp.py`` (`distributed_syncBN_amp.py:42-75`)

Quirk resolutions:
* Q1  ``--seed`` seeds python/numpy/torch correctly (the reference crashes on ``np.random(seed)``).
* Q2  ``type=bool`` flags: the reference treats every non-empty string as True; we parse
      ``False/false/0/no/off/''`` as False, anything else as True, and a bare flag as True.
* Q3  ``--step`` accepts ``--step 3 4``, ``--step 3,4`` and ``--step [3,4]`` and yields ints.
* Q5  ``--local_rank``, ``--local-rank`` and env ``LOCAL_RANK`` are all accepted.
* Q12 ``--gpus`` is accepted; it only sets ``HIP_VISIBLE_DEVICES`` when ``--use-gpus-flag`` is given.

Additional (MI355X-native) flags are grouped under "native options"; all have defaults that
reproduce the reference behaviour.
"""
from __future__ import annotations

import argparse
import os
from typing import List, Optional

from .models.registry import model_names

ENTRY_DEFAULTS = {
    "dp": {"gpus": "5,6,7", "outpath": "./output", "logger": "DataParallel"},
    "ddp": {"gpus": "0,1,2", "outpath": "./output_ddp_test", "logger": "DistributedDataParallel"},
    "ddp_amp": {"gpus": "0,1,2", "outpath": "./output_ddp_amp", "logger": "DistributedDataParallel_amp"},
}

_FALSE = {"false", "0", "no", "off", "n", "f", ""}


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() not in _FALSE


def parse_steps(values) -> List[int]:
    if values is None:
        return [3, 4]
    if isinstance(values, (int,)):
        return [values]
    out: List[int] = []
    for v in values if isinstance(values, (list, tuple)) else [values]:
        if isinstance(v, int):
            out.append(v)
            continue
        s = str(v).strip().strip("[]()")
        out.extend(int(x) for x in s.replace(",", " ").split() if x)
    return out


def build_parser(mode: str) -> argparse.ArgumentParser:
    if mode not in ENTRY_DEFAULTS:
        raise ValueError(mode)
    d = ENTRY_DEFAULTS[mode]
    names = model_names()
    p = argparse.ArgumentParser(description="PyTorch ImageNet Training (MI355X-native)")
    p.add_argument("--data", metavar="DIR", default="/mnt/cephfs/mixed/dataset/imagenet/", help="path to dataset")
    p.add_argument("-a", "--arch", metavar="ARCH", default="resnet18", choices=names,
                   help="model architecture: " + " | ".join(names) + "(default: resnet18)")
    p.add_argument("-j", "--workers", default=8, type=int, metavar="N", help="number of data loading workers")
    p.add_argument("--epochs", default=5, type=int, metavar="N", help="number of total epochs to run")
    p.add_argument("--step", default=[3, 4], nargs="+", metavar="step decay", help="lr decay by step")
    p.add_argument("--start-epoch", default=0, type=int, metavar="N", help="manual epoch number ()")
    p.add_argument("-b", "--batch-size", default=1200, type=int, metavar="N",
                   help="mini-batch size, the total batch size of all GPUs on the current node "
                        "when using Data Parallel or Distributed Data Parallel")
    p.add_argument("--lr", "--learning-rate", default=0.1, type=float, metavar="LR", help="initial learning rate",
                   dest="lr")
    p.add_argument("--momentum", default=0.9, type=float, metavar="M", help="momentum")
    p.add_argument("--wd", "--weight-decay", default=1e-4, type=float, metavar="W", help="weight decay (default: 1e-4)",
                   dest="weight_decay")
    p.add_argument("-p", "--print-freq", default=10, type=int, metavar="N", help="print frequency (default: 10)")
    p.add_argument("-e", "--evaluate", dest="evaluate", default=False, type=str2bool, nargs="?", const=True,
                   help="evaluate model on validation set")
    p.add_argument("--pretrained", dest="pretrained", default=False, type=str2bool, nargs="?", const=True,
                   help="use pre-trained model (loaded from a local file, see --pretrained-path)")
    p.add_argument("--seed", default=None, type=int, help="seed for initializing training")
    p.add_argument("--gpus", default=d["gpus"], metavar="gpus_id", help="N gpus for training")
    p.add_argument("--outpath", metavar="DIR", default=d["outpath"], help="path to output")
    p.add_argument("--lr-scheduler", metavar="LR scheduler", default="steplr", help="LR scheduler", dest="lr_scheduler")
    p.add_argument("--gamma", default=0.1, type=float, metavar="gamma", help="gamma")
    if mode in ("ddp", "ddp_amp"):
        p.add_argument("--local_rank", "--local-rank", dest="local_rank", type=int,
                       default=int(os.environ.get("LOCAL_RANK", "0")), help="node rank for distributed training")
    if mode == "ddp_amp":
        p.add_argument("--use_amp", dest="use_amp", default=True, type=str2bool, nargs="?", const=True,
                       help="use automatic mixed precision (amp)")
        p.add_argument("--sync_batchnorm", dest="sync_batchnorm", default=False, type=str2bool, nargs="?", const=True,
                       help="use sync batchnorm")

    g = p.add_argument_group("native options")
    g.add_argument("--engine", default="auto", choices=["auto", "native", "torch"],
                   help="native = hand-written HIP kernels (GPU, ResNet family); torch = stock PyTorch ops "
                        "(CPU reference path, or explicitly requested on GPU); auto = native on GPU when the arch is "
                        "supported, torch otherwise")
    g.add_argument("--precision", default="auto", choices=["auto", "bf16", "fp16", "fp32"],
                   help="compute dtype; auto = fp16 with --use_amp, bf16 otherwise on GPU, fp32 on CPU")
    g.add_argument("--eval-precision", default="auto", choices=["auto", "compute", "fp32"],
                   help="validation dtype: fp32 on the native fp32 kernels over the fp32 master weights (the reference "
                        "validates without autocast, `distributed_syncBN_amp.py:309-317`, and in fp32 everywhere), or "
                        "the training compute dtype; auto = fp32 (every entry script, native DataParallel included: "
                        "`dataparallel.py:243-262` validates the fp32 model)")
    g.add_argument("--synthetic", default=False, type=str2bool, nargs="?", const=True,
                   help="use synthetic ImageNet-shaped data instead of --data")
    g.add_argument("--synthetic-train-size", type=int, default=1281167)
    g.add_argument("--synthetic-val-size", type=int, default=50000)
    g.add_argument("--image-size", type=int, default=None,
                   help="crop size (default 224; 299 for inception_v3, whose aux head needs it)")
    g.add_argument("--num-classes", type=int, default=1000)
    g.add_argument("--iters-per-epoch", type=int, default=0, help="cap on train iterations per epoch (0 = full)")
    g.add_argument("--val-iters", type=int, default=0, help="cap on val iterations per epoch (0 = full)")
    g.add_argument("--bucket-cap-mb", type=float, default=25.0, help="DDP gradient bucket size (MiB)")
    g.add_argument("--first-bucket-mb", type=float, default=1.0, help="first-produced bucket (DDP policy, torch engine)")
    g.add_argument("--last-bucket-mb", type=float, default=1.0,
                   help="last-produced (stem-side) bucket of the native engine; <= 0: DDP's first-bucket policy")
    g.add_argument("--strict-sync", default=False, type=str2bool, nargs="?", const=True,
                   help="keep the reference's per-iteration barrier and host read of the metrics")
    g.add_argument("--exist-policy", default=os.environ.get("PDT_EXIST_POLICY", "prompt"),
                   choices=["prompt", "delete", "quit", "reuse"], help="what to do if the output dir exists")
    g.add_argument("--resume", default="", metavar="PATH", help="resume from a checkpoint written by this framework")
    g.add_argument("--pretrained-path", default=None, help="local torchvision-format weights for --pretrained")
    g.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    g.add_argument("--jpeg-draft", default=False, type=str2bool, nargs="?", const=True,
                   help="decode JPEGs at reduced size (libjpeg DCT scaling) ahead of the crop/resize "
                        "(throughput option; pixels differ slightly from a full decode)")
    g.add_argument("--gpu-normalize", default="auto", choices=["auto", "on", "off"],
                   help="ship uint8 images to the GPU and normalise there (fused into the native stem kernel); "
                        "auto = on for the native engine, off otherwise")
    g.add_argument("--graph", default=False, type=str2bool, nargs="?", const=True,
                   help="capture the whole native training step in a HIP graph and replay it (single process; "
                        "pays off when small batches make the step launch-bound)")
    g.add_argument("--comm", default="native", choices=["torch", "native"],
                   help="native engine collectives: this framework's own RCCL communicator and C++ gradient "
                        "bucketer (default; torch.distributed then only provides the rendezvous store) or "
                        "torch.distributed (RCCL via c10d)")
    g.add_argument("--comm-transport", default="auto", choices=["auto", "rccl", "host"],
                   help="native communicator transport: rccl (one rank per GPU) | host (shared memory: ranks sharing a "
                        "GPU, CPU ranks) | auto")
    g.add_argument("--grad-compress", default="none", choices=["none", "bf16"],
                   help="native communicator: all-reduce the gradient buckets in bf16 (half the bytes; upstream "
                        "DDP's bf16_compress_hook). Default none: fp32 like the reference")
    g.add_argument("--dist-timeout", type=float, default=1800.0,
                   help="collective timeout in seconds (a hung rank fails the job instead of hanging it)")
    g.add_argument("--profile", default=False, type=str2bool, nargs="?", const=True,
                   help="roctx ranges around train/eval steps (visible in rocprofv3 --marker-trace) and a "
                        "per-epoch throughput line")
    g.add_argument("--autotune", default=False, type=str2bool, nargs="?", const=True,
                   help="time the candidate conv tile configs once per shape and keep the fastest (the analogue of "
                        "the reference's cudnn.benchmark=True); off = the static per-shape table")
    g.add_argument("--use-gpus-flag", default=False, type=str2bool, nargs="?", const=True,
                   help="honour --gpus by setting HIP_VISIBLE_DEVICES (the reference ignores --gpus)")
    g.add_argument("--no-tensorboard", dest="tensorboard", action="store_false")
    return p


def parse_args(mode: str, argv: Optional[List[str]] = None) -> argparse.Namespace:
    args = build_parser(mode).parse_args(argv)
    args.step = parse_steps(args.step)
    if args.image_size is None:
        args.image_size = 299 if args.arch == "inception_v3" else 224
    args.mode = mode
    return args
