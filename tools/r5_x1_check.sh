set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "conv1x1x or conv1x1_c64" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x1.log 2>&1 || { tail -30 gpurun_out/t_x1.log; exit 1; }
tail -2 gpurun_out/t_x1.log
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py -k "resnet50" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_x1e.log 2>&1 || { tail -30 gpurun_out/t_x1e.log; exit 1; }
tail -2 gpurun_out/t_x1e.log
timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench50x.log 2>&1 || { tail -5 gpurun_out/bench50x.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench50x.log
PDT_CONV1X1X=0 timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench50x0.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench50x0.log
timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench50x_2.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench50x_2.log
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof50x" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --arch resnet50 --dtype fp16 --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof50x.log" 2>&1 || exit 1
echo ALL DONE
