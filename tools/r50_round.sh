#!/bin/bash
# ResNet-50 (BASELINE config 5, fp16 AMP) stages: bench, autotune bench, serial kernel profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-/root/repo}
for stage in "$@"; do
  case "$stage" in
    bench)
      timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench_r50.log 2>&1 || exit 1
      grep metric gpurun_out/bench_r50.log ;;
    autotune)
      timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 --autotune > gpurun_out/bench_r50_at.log 2>&1 || exit 1
      grep metric gpurun_out/bench_r50_at.log ;;
    profserial)
      cd /tmp && export TMPDIR=/tmp
      PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof50s -o run -- \
        python3 $R/bench.py --arch resnet50 --dtype fp16 --steps 3 --warmup 2 > $R/gpurun_out/prof50s.log 2>&1 || exit 1
      cd $R; grep metric gpurun_out/prof50s.log ;;
  esac
done
echo "ALL DONE"
