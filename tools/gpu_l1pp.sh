#!/bin/bash
# A/B of the layer1 kernels (8-wave ping-pong conv, pipelined 9-tap wgrad) + their tests + a serial profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pingpong or layer1 or fused_bn_backward or producer or 3x3c64" --timeout 120 --timeout-method thread > gpurun_out/t_l1pp.log 2>&1; rc=$?; tail -5 gpurun_out/t_l1pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -x -q -k "window" --timeout 120 --timeout-method thread > gpurun_out/t_fp32win.log 2>&1; rc=$?; tail -3 gpurun_out/t_fp32win.log; [ $rc -eq 0 ] || exit $rc
PDT_CONV_L1_PP=1 timeout -k 10 300 python tools/conv_bench.py --skip-stem --shapes 0,1,2,3 --reps 5 > gpurun_out/cb_new.log 2>&1 || exit $?
PDT_CONV_L1_PP=0 PDT_WGRAD_L1_PIPE=0 timeout -k 10 300 python tools/conv_bench.py --skip-stem --shapes 0 --reps 5 > gpurun_out/cb_old.log 2>&1 || exit $?
PDT_FWD_STAGES=3 timeout -k 10 300 python tools/conv_bench.py --skip-stem --shapes 1,2,3 --reps 5 > gpurun_out/cb_st3.log 2>&1 || exit $?
echo CB_OK
for i in 1 2; do
for cfg in "PDT_CONV_L1_PP=1 PDT_WGRAD_L1_PIPE=1" "PDT_CONV_L1_PP=0 PDT_WGRAD_L1_PIPE=0" "PDT_CONV_L1_PP=1 PDT_WGRAD_L1_PIPE=0" "PDT_CONV_L1_PP=0 PDT_WGRAD_L1_PIPE=1"; do
env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_ab.log 2>&1 || exit $?; echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_ab.log)"
done
done
for cfg in "PDT_FP32_STEM_WIN=1" "PDT_FP32_STEM_WIN=0"; do
env $cfg timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/b32.log 2>&1 || exit $?; echo "fp32 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b32.log)"
done
cd /tmp && export TMPDIR=/tmp
PDT_CONV_L1_PP=1 PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs.log" 2>&1 || exit $?
echo PROF_OK
