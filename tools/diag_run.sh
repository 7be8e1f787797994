set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1 || { tail -20 gpurun_out/pytest_fp32.log; exit 1; }
tail -1 gpurun_out/pytest_fp32.log
for cfg in "128 0" "128 1" "256 1" "512 1" "128 0" "128 1"; do
  set -- $cfg
  PDT_FP32_BM64=$1 PDT_FP32_HALO=$2 timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/b32_$1_$2.log 2>&1 || exit 1
  echo "BM64=$1 HALO=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b32_$1_$2.log)"
done
