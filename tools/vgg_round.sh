#!/bin/bash
# VGG-16 on the native engine vs stock PyTorch (MIOpen) at the reference's per-GPU batches, plus a kernel table
# (run on the GPU box through gpurun; each GPU step has its own time limit, the script stops at the first failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
set -o pipefail
for B in 150 256; do
  timeout -k 10 300 python bench.py --arch vgg16 --batch-per-gpu $B --steps 10 --warmup 3 > gpurun_out/vgg16_b$B.log 2>&1 || exit 1
  grep metric gpurun_out/vgg16_b$B.log
done
timeout -k 10 300 python bench.py --arch vgg16_bn --batch-per-gpu 150 --steps 10 --warmup 3 > gpurun_out/vgg16bn_b150.log 2>&1 || exit 1
grep metric gpurun_out/vgg16bn_b150.log
timeout -k 10 400 python tools/torch_baseline.py --arch vgg16 --bs 150 --steps 5 --benchmark 0 > gpurun_out/vgg16_torch_b150.log 2>&1 || exit 1
tail -2 gpurun_out/vgg16_torch_b150.log
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_vgg" -o run -- \
  python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --arch vgg16 --batch-per-gpu 150 --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_vgg.log" 2>&1 || exit 1
echo prof done
