#!/bin/bash
# SyncBN forward statistics on the compute stream (default) vs through the comm stream (PDT_SYNCBN_INLINE=0),
# native communicator at a world of one, interleaved on one box; plus the no-SyncBN reference.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for i in 1 2; do
  timeout -k 10 300 python bench.py --force-comm --sync-bn --steps 20 --warmup 5 > gpurun_out/sbA$i.log 2>&1 || exit 1
  PDT_SYNCBN_INLINE=0 timeout -k 10 300 python bench.py --force-comm --sync-bn --steps 20 --warmup 5 > gpurun_out/sbB$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --force-comm --steps 20 --warmup 5 > gpurun_out/sbC$i.log 2>&1 || exit 1
  echo "inline $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sbA$i.log)  comm-stream $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sbB$i.log)  no-syncbn $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sbC$i.log)"
done
