#!/bin/bash
# LDS-staged conv output write-back: kernel tests, then interleaved A/B on ResNet-18 (bf16) and ResNet-50 (fp16)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
timeout -k 10 300 python -m pytest tests/test_executor_gpu.py -x -q > gpurun_out/t_e.log 2>&1 || { tail -30 gpurun_out/t_e.log; exit 1; }
tail -1 gpurun_out/t_e.log
for arch in resnet18 resnet50; do
  dt=bf16; [ $arch = resnet50 ] && dt=fp16
  for i in 1 2; do
    timeout -k 10 300 python bench.py --arch $arch --dtype $dt --steps 10 --warmup 3 > gpurun_out/so_${arch}_A$i.log 2>&1 || exit 1
    PDT_STAGE_OUT=0 timeout -k 10 300 python bench.py --arch $arch --dtype $dt --steps 10 --warmup 3 > gpurun_out/so_${arch}_B$i.log 2>&1 || exit 1
    echo "$arch staged $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/so_${arch}_A$i.log)  direct $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/so_${arch}_B$i.log)"
  done
done
