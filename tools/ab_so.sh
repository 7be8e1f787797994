#!/bin/bash
# Same-box interleaved A/B of two builds of the native extension on the 1-GPU bench:
#   bash tools/ab_so.sh build/ab/_C_base.so [steps] [extra bench args...]
# A = the in-tree _C.so, B = the given build (loaded through PDT_NATIVE_SO).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
SO="$1"; K="${2:-20}"; shift 2
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps $K --warmup 5 "$@" > gpurun_out/abA$i.log 2>&1 || exit 1
  PDT_NATIVE_SO="$SO" timeout -k 10 300 python bench.py --steps $K --warmup 5 "$@" > gpurun_out/abB$i.log 2>&1 || exit 1
  echo "A(in-tree) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abA$i.log)   B($SO) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abB$i.log)"
done
