#!/bin/bash
# Tile autotune at the reference's own per-GPU batches (-b 1200 node-total on 3 GPUs = 400/GPU, on 8 = 150/GPU):
# the shapes where PDT_AUTOTUNE=1 beat the static rule go to gpurun_out/tune_<B>.jsonl; then plain vs autotuned
# vs --graph step times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for B in 400 150; do
  rm -f gpurun_out/tune_$B.jsonl
  PDT_AUTOTUNE_DUMP=gpurun_out/tune_$B.jsonl timeout -k 10 300 python bench.py --batch-per-gpu $B --steps 30 --warmup 5 --autotune > gpurun_out/tb_auto_$B.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --batch-per-gpu $B --steps 30 --warmup 5 > gpurun_out/tb_plain_$B.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --batch-per-gpu $B --steps 30 --warmup 5 --graph > gpurun_out/tb_graph_$B.log 2>&1 || exit $?
  echo "B=$B plain $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tb_plain_$B.log) autotune $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tb_auto_$B.log) graph $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tb_graph_$B.log) tuned-shapes $(wc -l < gpurun_out/tune_$B.jsonl)"
done
