# round-5 closing benchmark records (final tree): ResNet-18 bf16 x3, ResNet-50 fp16 x2, ResNet-18 fp32, B=150 / B=400,
# ResNeXt-50 fp16, ResNet-18 SyncBN (forced comm), each line into gpurun_out/rec_*.log; R50 serial profile
set -o pipefail
mkdir -p gpurun_out
run() { local tag="$1"; shift; timeout -k 10 600 python bench.py "$@" > "gpurun_out/rec_$tag.log" 2>&1 || { tail -5 "gpurun_out/rec_$tag.log"; exit 1; }; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rec_$tag.log)"; }
run r18_1 --steps 20 --warmup 5
run r50_1 --arch resnet50 --dtype fp16 --steps 10 --warmup 3
run r18_2 --steps 20 --warmup 5
run r50_2 --arch resnet50 --dtype fp16 --steps 10 --warmup 3
run r18_3 --steps 20 --warmup 5
run r18_fp32 --dtype fp32 --steps 5 --warmup 2
run r18_b150 --steps 20 --warmup 5 --batch-per-gpu 150
run r18_b400 --steps 20 --warmup 5 --batch-per-gpu 400
run rx50 --arch resnext50_32x4d --dtype fp16 --steps 5 --warmup 2
run r18_sbn --steps 20 --warmup 5 --dtype fp16 --sync-bn --force-comm
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof50f" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --arch resnet50 --dtype fp16 --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof50f.log" 2>&1 || exit 1
echo ALL DONE
