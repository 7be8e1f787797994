#!/bin/bash
# 2-stream kernel traces of two settings (A: $PROF_A, B: $PROF_B env assignments) for timeline comparison
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  eval "cfg=\$PROF_$tag"
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_$tag" -o run -- python3 "$R/bench.py" --steps 6 --warmup 3 > "$R/gpurun_out/prof_$tag.log" 2>&1 || exit $?
  echo "$tag ($cfg): $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/prof_$tag.log)"
done
