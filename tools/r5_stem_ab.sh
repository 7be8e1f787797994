cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stem" --timeout 120 --timeout-method thread > gpurun_out/t_stem.log 2>&1; rc=$?; tail -3 gpurun_out/t_stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q -k "224 and resnet18" --timeout 200 --timeout-method thread > gpurun_out/t_e224.log 2>&1; rc=$?; tail -3 gpurun_out/t_e224.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_pair.sh PDT_STEM_ROWS 0 1 || exit $?
for i in 1 2; do
  PDT_STEM_ROWS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s0_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s1_$i.log 2>&1 || exit $?
  echo "rows0 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s0_$i.log) rows1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s1_$i.log)"
done
