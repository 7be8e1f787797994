#!/bin/bash
# Usage: bash tools/gpu_round.sh <stage...>   (run on the GPU box via gpurun)
# Each GPU step has its own time limit; after a crash/timeout nothing more runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for stage in "$@"; do
  case "$stage" in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      tail -30 gpurun_out/pytest_gpu.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    testk)
      timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_k.log 2>&1; rc=$?
      tail -30 gpurun_out/pytest_k.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    teste)
      timeout -k 10 600 python -m pytest tests/test_executor_gpu.py -x -q > gpurun_out/pytest_e.log 2>&1; rc=$?
      tail -30 gpurun_out/pytest_e.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?
      tail -5 gpurun_out/bench.log
      [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; } ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      tail -5 gpurun_out/prof.log
      [ $rc -eq 0 ] || { echo "prof failed rc=$rc"; exit $rc; } ;;
    prof32)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof32" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --dtype fp32 --steps 3 --warmup 1 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof32.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      tail -2 gpurun_out/prof32.log
      [ $rc -eq 0 ] || { echo "prof32 failed rc=$rc"; exit $rc; } ;;
    profserial)
      # one stream (PDT_WGRAD_STREAM=0) so per-kernel durations are not inflated by concurrency
      cd /tmp && export TMPDIR=/tmp
      PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      tail -2 gpurun_out/profs.log
      [ $rc -eq 0 ] || { echo "prof failed rc=$rc"; exit $rc; } ;;
    convbench)
      timeout -k 10 600 python tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1; rc=$?
      cat gpurun_out/conv_bench.log | grep shape
      [ $rc -eq 0 ] || { echo "conv_bench failed rc=$rc"; exit $rc; } ;;
    stembench)
      timeout -k 10 300 python tools/conv_bench.py --only-stem > gpurun_out/stem_bench.log 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "stem bench failed rc=$rc"; exit $rc; }
      rc=0
      grep shape gpurun_out/stem_bench.log
      [ $rc -eq 0 ] || { echo "stem bench (2-stage) failed rc=$rc"; exit $rc; } ;;
    l1bench)
      timeout -k 10 300 python tools/conv_bench.py --skip-stem --shapes 0 > gpurun_out/l1_bench.log 2>&1; rc=$?
      grep shape gpurun_out/l1_bench.log
      [ $rc -eq 0 ] || { echo "l1 bench failed rc=$rc"; exit $rc; } ;;
    reftable)
      timeout -k 10 600 python tools/reference_table.py --md gpurun_out/reference_table_1gpu.md > gpurun_out/reftable.log 2>&1; rc=$?
      cat gpurun_out/reftable.log | grep mode
      [ $rc -eq 0 ] || { echo "reference table failed rc=$rc"; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -5 gpurun_out/smoke.log
      [ $rc -eq 0 ] || { echo "smoke failed rc=$rc"; exit $rc; } ;;
    autotune)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 --autotune > gpurun_out/bench_autotune.log 2>&1; rc=$?
      grep metric gpurun_out/bench_autotune.log
      [ $rc -eq 0 ] || { echo "autotune bench failed rc=$rc"; exit $rc; } ;;
    dp)
      timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1; rc=$?
      tail -15 gpurun_out/pytest_dp.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    replay)
      # intra-kernel race detector: every native op of 2 training steps re-run 3x from a snapshot (PDT_VALIDATE=3)
      timeout -k 10 600 python -u tools/repeat_check.py --replay --steps 2 > gpurun_out/replay.log 2>&1; rc=$?
      tail -8 gpurun_out/replay.log
      ok_rc $rc || { echo "replay crashed rc=$rc"; exit $rc; } ;;
    repeat)
      timeout -k 10 600 python -u tools/repeat_check.py --reps 6 > gpurun_out/repeat.log 2>&1; rc=$?
      tail -8 gpurun_out/repeat.log
      ok_rc $rc || { echo "repeat crashed rc=$rc"; exit $rc; } ;;
    rehearse4)
      # 4 DDP ranks sharing the GPU: the native C++ communicator + bucketer over the host shared-memory transport
      timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29613 bench.py --gpus 4 --steps 3 --warmup 2 --dist-backend gloo --batch-per-gpu 128 \
        > gpurun_out/rehearse4.log 2>&1; rc=$?
      grep metric gpurun_out/rehearse4.log
      [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse4.log; echo "rehearse4 failed rc=$rc"; exit $rc; } ;;
    prof50)
      cd /tmp && export TMPDIR=/tmp
      PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof50" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --arch resnet50 --dtype fp16 --steps 4 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof50.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      [ $rc -eq 0 ] || { echo "prof50 failed rc=$rc"; exit $rc; } ;;
    r50sweep)
      timeout -k 10 600 python tools/conv_bench.py --skip-stem --r50 --reps 5 > gpurun_out/cb_r50.log 2>&1; rc=$?
      grep shape gpurun_out/cb_r50.log | cut -c1-200
      [ $rc -eq 0 ] || { echo "r50 sweep failed rc=$rc"; exit $rc; } ;;
    fp32win)
      timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -x -q -k "window" --timeout 120 --timeout-method thread > gpurun_out/t_fp32win.log 2>&1; rc=$?
      tail -3 gpurun_out/t_fp32win.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    bench50)
      timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench50.log 2>&1; rc=$?
      grep metric gpurun_out/bench50.log
      [ $rc -eq 0 ] || { echo "bench50 failed rc=$rc"; exit $rc; } ;;
    fp32)
      timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1; rc=$?
      tail -5 gpurun_out/pytest_fp32.log
      ok_rc $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
      timeout -k 10 600 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/bench32.log 2>&1; rc=$?
      grep metric gpurun_out/bench32.log
      [ $rc -eq 0 ] || { echo "bench32 failed rc=$rc"; exit $rc; } ;;
    table)
      # BASELINE.md's 1-GPU cells: ResNet-18 bf16, ResNet-18 fp16 AMP + SyncBN (native comm forced at world 1:
      # the whole SyncBN path with identity all-reduces), ResNet-50 fp16 AMP
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/t_r18.log 2>&1 || exit $?
      grep metric gpurun_out/t_r18.log
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 --dtype fp16 --sync-bn --force-comm > gpurun_out/t_r18sbn.log 2>&1 || exit $?
      grep metric gpurun_out/t_r18sbn.log
      timeout -k 10 600 python bench.py --steps 10 --warmup 3 --arch resnet50 --dtype fp16 > gpurun_out/t_r50.log 2>&1 || exit $?
      grep metric gpurun_out/t_r50.log ;;
    bench32)
      timeout -k 10 600 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/bench32.log 2>&1; rc=$?
      grep metric gpurun_out/bench32.log
      [ $rc -eq 0 ] || { echo "bench32 failed rc=$rc"; exit $rc; } ;;
    rehearse2)
      # 2 DDP ranks sharing the one GPU over gloo: exercises the world>1 native-trainer path
      # (bucketer, buffer broadcast, metric all-reduce, side-stream ordering) without a second GPU
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --batch-per-gpu 256 \
        > gpurun_out/rehearse2.log 2>&1; rc=$?
      grep metric gpurun_out/rehearse2.log
      [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse2.log; echo "rehearse2 failed rc=$rc"; exit $rc; } ;;
    rehearse2sbn)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --batch-per-gpu 256 \
        --sync-bn --dtype fp16 > gpurun_out/rehearse2sbn.log 2>&1; rc=$?
      grep metric gpurun_out/rehearse2sbn.log
      [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse2sbn.log; echo "rehearse2sbn failed rc=$rc"; exit $rc; } ;;
  esac
done
echo "ALL DONE"
