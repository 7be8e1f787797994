#!/bin/bash
# Interleaved A/B/C... of environment settings on the 1-GPU bench (same box, 2 rounds):
#   bash tools/ab_multi.sh "" "PDT_X=0" "PDT_Y=1 PDT_Z=2" ...     ("" = defaults)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
K="${AB_STEPS:-20}"
for r in 1 2; do
  i=0
  for B in "$@"; do
    i=$((i+1))
    timeout -k 10 300 env $B python bench.py --steps $K --warmup 5 ${AB_ARGS:-} > gpurun_out/ab_${r}_${i}.log 2>&1 || { echo "arm [$B] failed"; tail -5 gpurun_out/ab_${r}_${i}.log; exit 1; }
    echo "round $r [$B] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${r}_${i}.log)"
  done
done
