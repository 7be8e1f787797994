#!/bin/bash
# same-box A/B: current tree (A) vs a snapshot of an older commit copied into old_tree/ (B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/abA$i.log 2>&1 || exit 1
  timeout -k 10 300 python old_tree/bench.py --steps 20 --warmup 5 > gpurun_out/abB$i.log 2>&1 || exit 1
  echo "A(new) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abA$i.log)   B(old) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abB$i.log)"
done
