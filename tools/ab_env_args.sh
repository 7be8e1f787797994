#!/bin/bash
# A/B of environment settings on any bench configuration, interleaved on the same box:
#   bash tools/ab_env_args.sh "PDT_X=0 PDT_Y=1" [steps] [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
B="$1"; K="${2:-20}"; shift 2
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps $K --warmup 3 "$@" > gpurun_out/abA$i.log 2>&1 || exit 1
  timeout -k 10 300 env $B python bench.py --steps $K --warmup 3 "$@" > gpurun_out/abB$i.log 2>&1 || exit 1
  echo "A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abA$i.log)   B($B) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abB$i.log)"
done
