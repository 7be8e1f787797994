#!/usr/bin/env bash
# Launch recipe equivalent to the reference start.sh: DataParallel, DDP and DDP+AMP on 3 GPUs.
# HIP_VISIBLE_DEVICES selects GPUs (CUDA_VISIBLE_DEVICES is honoured by ROCm as well).
set -e
export HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES:-0,1,2}
NPROC=${NPROC:-3}
PORT=${MASTER_PORT:-23334}
python dataparallel.py "$@"
python -m pytorch_distributed_template_amd.launch --nproc_per_node=$NPROC --master_port=$PORT distributed.py "$@"
python -m pytorch_distributed_template_amd.launch --nproc_per_node=$NPROC --master_port=$PORT distributed_syncBN_amp.py "$@"
