#!/bin/bash
# Usage (on the GPU box via gpurun): bash tools/gpu_check.sh <stage...>
# Stages: tests (full GPU suite, no -x), diag (DDP bitwise diagnostic), bench (1-GPU headline bench).
# Every GPU step has its own time limit; a crash / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for stage in "$@"; do
  case "$stage" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_all.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_all.log | tail -25
      [ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    diag)
      timeout -k 10 500 python -u tools/diag_ddp.py 6 > gpurun_out/diag_ddp.log 2>&1; rc=$?
      grep "allreduced\|local" gpurun_out/diag_ddp.log | cut -c1-200
      [ $rc -eq 0 ] || { tail -20 gpurun_out/diag_ddp.log; echo "diag failed rc=$rc"; exit $rc; } ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?
      grep metric gpurun_out/bench.log
      [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.log; echo "bench failed rc=$rc"; exit $rc; } ;;
    bench50)
      timeout -k 10 600 python bench.py --arch resnet50 --dtype fp16 --steps 10 --warmup 3 > gpurun_out/bench50.log 2>&1; rc=$?
      grep metric gpurun_out/bench50.log
      [ $rc -eq 0 ] || { tail -20 gpurun_out/bench50.log; echo "bench50 failed rc=$rc"; exit $rc; } ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      grep metric gpurun_out/prof.log
      [ $rc -eq 0 ] || { tail -5 gpurun_out/prof.log; echo "prof failed rc=$rc"; exit $rc; } ;;
    profs)
      cd /tmp && export TMPDIR=/tmp
      PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      [ $rc -eq 0 ] || { tail -5 gpurun_out/profs.log; echo "profs failed rc=$rc"; exit $rc; } ;;
    prof50)
      cd /tmp && export TMPDIR=/tmp
      PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof50s" -o run -- \
        python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --arch resnet50 --dtype fp16 --steps 3 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof50s.log" 2>&1; rc=$?
      cd "${GRAFT_REPO_ROOT:-/root/repo}"
      [ $rc -eq 0 ] || { tail -5 gpurun_out/prof50s.log; echo "prof50 failed rc=$rc"; exit $rc; } ;;
    pmcbytes)
      bash tools/pmc_bytes.sh || exit 1 ;;
    pmcbytes50)
      BENCH_ARGS="--arch resnet50 --dtype fp16" bash tools/pmc_bytes.sh || exit 1
      mv gpurun_out/pmc_bytes gpurun_out/pmc_bytes50 ;;
    pmcsq)
      bash tools/pmc_step.sh || exit 1 ;;
    testk)
      timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_ddp_numerics_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_k.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_k.log | tail -15
      [ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    convbench)
      timeout -k 10 600 python -u tools/conv_bench.py --skip-stem > gpurun_out/conv_bench.log 2>&1; rc=$?
      grep shape gpurun_out/conv_bench.log | cut -c1-400
      [ $rc -eq 0 ] || { tail -5 gpurun_out/conv_bench.log; echo "conv_bench failed rc=$rc"; exit $rc; } ;;
    testt)
      timeout -k 10 900 python -u -m pytest tests/test_training_gpu.py tests/test_comm_gpu.py tests/test_ddp_numerics_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_t.log 2>&1; rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_t.log | tail -15
      [ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit $rc; } ;;
    syncbn1)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/sb_plain.log 2>&1 && \
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 --force-comm > gpurun_out/sb_comm.log 2>&1 && \
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 --force-comm --sync-bn > gpurun_out/sb_sync.log 2>&1 && \
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 --force-comm --sync-bn --dtype fp16 > gpurun_out/sb_sync16.log 2>&1; rc=$?
      for f in sb_plain sb_comm sb_sync sb_sync16; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
      [ $rc -eq 0 ] || { tail -20 gpurun_out/sb_sync.log; exit $rc; } ;;
    test32)
      timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_32.log 2>&1; rc=$?
      grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_32.log | tail -30
      [ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; tail -30 gpurun_out/pytest_32.log; exit $rc; } ;;
    bench32)
      timeout -k 10 900 python bench.py --dtype fp32 --steps 5 --warmup 2 > gpurun_out/bench32.log 2>&1; rc=$?
      grep metric gpurun_out/bench32.log
      [ $rc -eq 0 ] || { tail -20 gpurun_out/bench32.log; echo "bench32 failed rc=$rc"; exit $rc; } ;;
    torch50)
      timeout -k 10 900 python -u tools/torch_baseline.py --arch resnet50 --dtype fp16 > gpurun_out/torch50.log 2>&1 || { tail gpurun_out/torch50.log; exit 1; }
      tail -2 gpurun_out/torch50.log ;;
    torch18fp32)
      timeout -k 10 900 python -u tools/torch_baseline.py --arch resnet18 --dtype fp32 --steps 5 > gpurun_out/torch18fp32.log 2>&1 || { tail gpurun_out/torch18fp32.log; exit 1; }
      tail -2 gpurun_out/torch18fp32.log ;;
  esac
done
echo "ALL DONE"
