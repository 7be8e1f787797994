cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -x -q -k "window" --timeout 120 --timeout-method thread > gpurun_out/t_fp32win.log 2>&1; rc=$?; tail -3 gpurun_out/t_fp32win.log; [ $rc -eq 0 ] || exit $rc
for cfg in "PDT_FP32_STEM_WIN=1" "PDT_FP32_STEM_WIN=0"; do
env $cfg timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/b32.log 2>&1 || exit $?; echo "fp32 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b32.log)"
done
timeout -k 10 300 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/b50.log 2>&1 || exit $?; echo "r50 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b50.log)"
timeout -k 10 300 python tools/conv_bench.py --skip-stem --r50 --reps 5 > gpurun_out/cb_r50.log 2>&1 || exit $?
grep shape gpurun_out/cb_r50.log | cut -c1-330
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof50" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --arch resnet50 --dtype fp16 --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof50.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof32" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --dtype fp32 --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof32.log" 2>&1 || exit $?
echo DONE
