#!/bin/bash
# serial kernel traces (PDT_WGRAD_STREAM=0) of ResNet-18 bf16 at the given per-GPU batches, plus the two-stream bench
# of each: bash tools/prof_batch.sh 150 400   (run through gpurun; every step has its own time limit)
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for B in "$@"; do
  PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_b$B" -o run -- \
    python3 "$R/bench.py" --batch-per-gpu "$B" --steps 10 --warmup 3 > "$R/gpurun_out/prof_b$B.log" 2>&1 || exit 1
  timeout -k 10 300 python3 "$R/bench.py" --batch-per-gpu "$B" --steps 40 --warmup 10 > "$R/gpurun_out/bench_b$B.log" 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$R/gpurun_out/bench_b$B.log"
done
