# same-box interleaved A/B of this tree's .so against build/abso/_C_prev.so (ResNet-18 bf16 x3, ResNet-50 fp16 x2)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/s18_n$i.log 2>&1 || exit 1
  PDT_NATIVE_SO=build/abso/_C_prev.so timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/s18_o$i.log 2>&1 || exit 1
  echo "R18 new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s18_n$i.log)  prev $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s18_o$i.log)"
done
for i in 1 2; do
  timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/s50_n$i.log 2>&1 || exit 1
  PDT_NATIVE_SO=build/abso/_C_prev.so timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/s50_o$i.log 2>&1 || exit 1
  echo "R50 new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s50_n$i.log)  prev $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s50_o$i.log)"
done
