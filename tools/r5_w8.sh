#!/bin/bash
# 8-wave layer1 weight gradient (PDT_WGRAD_L1_W8 = 0..3): numerics of the default, then same-box R18 A/Bs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -x -v \
  --timeout 120 --timeout-method thread -k "3x3c64 or fused_producer_bn_relu_layer1 or train_step_matches_reference_224" \
  > gpurun_out/w8_tests.log 2>&1 || { tail -30 gpurun_out/w8_tests.log; exit 1; }
tail -2 gpurun_out/w8_tests.log
bash tools/ab_env3.sh PDT_WGRAD_L1_W8 0 3 || exit 1
bash tools/ab_env3.sh PDT_WGRAD_L1_W8 2 3
