# interleaved same-box A/B of one env knob on ResNet-50 fp16 and ResNet-18 bf16:  bash tools/r5_x1_ab.sh KNOB A B
set -o pipefail
K="$1"; A="$2"; B="$3"
mkdir -p gpurun_out
for i in 1 2; do
  env $K=$A timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/x50_a$i.log 2>&1 || exit 1
  env $K=$B timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/x50_b$i.log 2>&1 || exit 1
  echo "R50 $K=$A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x50_a$i.log)  $K=$B $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x50_b$i.log)"
done
for i in 1 2; do
  env $K=$A timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/x18_a$i.log 2>&1 || exit 1
  env $K=$B timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/x18_b$i.log 2>&1 || exit 1
  echo "R18 $K=$A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x18_a$i.log)  $K=$B $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/x18_b$i.log)"
done
