#!/bin/bash
# staged (LDS row) epilogue of the ping-pong conv kernel: kernel tests, 1x1 sweep and step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pps.log 2>&1; rc=$?; tail -3 gpurun_out/t_pps.log; [ $rc -eq 0 ] || exit $rc
for cfg in "PDT_PP_STAGE=1" "PDT_PP_STAGE=0"; do
  env $cfg timeout -k 10 300 python tools/conv_bench.py --skip-stem --r50 --reps 5 > gpurun_out/cb_r50_pps.log 2>&1 || exit $?
  echo "== $cfg"; grep shape gpurun_out/cb_r50_pps.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'pp256', d.get('fwd_256x256x64'), 'best_us', d['best_us'], 'TBps', d['best_TBps'])"
done
REPS=2 bash tools/gpu_bench_ab.sh "PDT_PP_STAGE=1" "PDT_PP_STAGE=0"
REPS=1 BENCH_ARGS="--arch resnet50 --dtype fp16" STEPS=10 bash tools/gpu_bench_ab.sh "PDT_PP_STAGE=1" "PDT_PP_STAGE=0" "PDT_PP_STAGE=1" "PDT_PP_STAGE=0"
