#!/bin/bash
# The reference's own per-GPU batches (-b 1200 node-total over 8 / 3 GPUs = 150 / 400 per GPU): bench lines and a
# serial kernel trace at 150 (run through gpurun; every GPU step has its own limit, the script stops at a failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for B in 150 400; do
  timeout -k 10 300 python bench.py --batch-per-gpu $B --steps 40 --warmup 10 > gpurun_out/sb_b$B.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/sb_b$B.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_b150" -o run -- \
  python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --batch-per-gpu 150 --steps 10 --warmup 3 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_b150.log" 2>&1 || exit 1
echo prof done
