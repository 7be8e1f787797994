#!/bin/bash
# A/B bench on one box: bash tools/ab.sh "ENV_A" "ENV_B" [rounds] [extra bench args]
# Alternates A and B runs (each its own process and time limit) and prints ms/step per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A="$1"; B="$2"; R="${3:-2}"; shift 3; EXTRA="$*"
for i in $(seq 1 "$R"); do
  for tag in A B; do
    if [ $tag = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 $EXTRA > gpurun_out/ab_$tag$i.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "run $tag$i failed rc=$rc"; tail -5 gpurun_out/ab_$tag$i.log; exit $rc; }
    echo "$tag$i [$E] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$tag$i.log)"
  done
done
