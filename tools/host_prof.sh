#!/bin/bash
# host-side cost of the eager training step: cProfile of bench.py, and eager vs --graph on the same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --steps 20 --warmup 3 > gpurun_out/host_prof.log 2>&1 || exit 1
python -c "
import pstats; p = pstats.Stats('gpurun_out/host.prof'); p.sort_stats('tottime').print_stats(25)" > gpurun_out/host_stats.txt 2>&1
head -60 gpurun_out/host_stats.txt | tail -40
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ge_A$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/ge_B$i.log 2>&1 || exit 1
  echo "eager $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ge_A$i.log)  graph $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ge_B$i.log)"
done
