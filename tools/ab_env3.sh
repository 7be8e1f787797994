#!/bin/bash
# Interleaved same-box A/B of one env knob on the 1-GPU bench: bash tools/ab_env3.sh VAR A B [bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
V="$1"; A="$2"; B="$3"; shift 3
for i in 1 2 3; do
  env "$V=$A" timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/abe_A$i.log 2>&1 || exit 1
  env "$V=$B" timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/abe_B$i.log 2>&1 || exit 1
  echo "$V=$A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_A$i.log)   $V=$B $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abe_B$i.log)"
done
