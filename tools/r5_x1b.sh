# conv1x1x backward-data rework: diag, kernel tests, R50 dispatch test, 3-way bench A/B, serial profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/x1_diag.py || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "conv1x1x or conv1x1_c64" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x1.log 2>&1 || { tail -30 gpurun_out/t_x1.log; exit 1; }
tail -1 gpurun_out/t_x1.log
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py -k "resnet50" -x -q --timeout 300 --timeout-method thread > gpurun_out/t_x1e.log 2>&1 || { tail -30 gpurun_out/t_x1e.log; exit 1; }
tail -1 gpurun_out/t_x1e.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/b50_n$i.log 2>&1 || exit 1
  PDT_NATIVE_SO=build/abso/_C_prev.so timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/b50_o$i.log 2>&1 || exit 1
  PDT_X1_L1=1 timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/b50_l$i.log 2>&1 || exit 1
  echo "new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b50_n$i.log)  prev $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b50_o$i.log)  new+X1_L1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b50_l$i.log)"
done
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof50z" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --arch resnet50 --dtype fp16 --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof50z.log" 2>&1 || exit 1
echo ALL DONE
