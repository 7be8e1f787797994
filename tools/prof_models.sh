#!/bin/bash
# serial kernel traces (PDT_WGRAD_STREAM=0) of the given archs at B = 1200, fp16: bash tools/prof_models.sh ARCH...
# (run through gpurun; one rocprofv3 --kernel-trace --stats run per arch, each with its own limit)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for A in "$@"; do
  PDT_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$A" -o run -- \
    python3 "$R/bench.py" --arch "$A" --dtype fp16 --steps 3 --warmup 2 > "$R/gpurun_out/prof_$A.log" 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$R/gpurun_out/prof_$A.log"
done
