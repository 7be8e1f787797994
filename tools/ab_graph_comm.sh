#!/bin/bash
# Small per-GPU batches (the reference's node batch split over 8 / 3 GPUs) with the native RCCL communicator
# (world of 1, --force-comm): eager step vs the whole step, collectives included, replayed as a HIP graph.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for bs in 150 400; do
  for mode in "" "--graph"; do
    timeout -k 10 300 python bench.py --force-comm --batch-per-gpu $bs --steps 40 --warmup 5 $mode \
      > gpurun_out/abgc_${bs}${mode:+_graph}.log 2>&1 || exit 1
  done
done
for f in gpurun_out/abgc_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"value": [0-9.]*' $f); done
