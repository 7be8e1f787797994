cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stem_wgrad_fused or bn_" --timeout 120 --timeout-method thread > gpurun_out/t_stem.log 2>&1; rc=$?; tail -3 gpurun_out/t_stem.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ew_bench.py > gpurun_out/ew_bench.log 2>&1 || exit $?
for i in 1 2; do
  PDT_STEM_QUAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/q0_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/q1_$i.log 2>&1 || exit $?
  PDT_NATIVE_SO=build/abso/_C_base.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/qb_$i.log 2>&1 || exit $?
  echo "quad0 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q0_$i.log) quad1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q1_$i.log) base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qb_$i.log)"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --arch resnet50 --dtype fp16 > gpurun_out/r50_new.log 2>&1 || exit $?
PDT_NATIVE_SO=build/abso/_C_base.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --arch resnet50 --dtype fp16 > gpurun_out/r50_base.log 2>&1 || exit $?
echo "r50 new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50_new.log) base $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50_base.log)"
