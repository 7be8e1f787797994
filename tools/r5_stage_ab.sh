# staging A/B after the 16-byte epilogues: PDT_PP_STAGE and PDT_STAGE_OUT on ResNet-18 and ResNet-50
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "PDT_PP_STAGE=1 PDT_STAGE_OUT=1" "PDT_PP_STAGE=0 PDT_STAGE_OUT=1" "PDT_PP_STAGE=0 PDT_STAGE_OUT=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/st18.log 2>&1 || exit 1
    env $cfg timeout -k 10 300 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/st50.log 2>&1 || exit 1
    echo "$cfg  R18 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/st18.log)  R50 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/st50.log)"
  done
done
