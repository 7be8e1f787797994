cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "compact or dgrad" > gpurun_out/t_compact.log 2>&1 || { tail -30 gpurun_out/t_compact.log; exit 1; }
tail -2 gpurun_out/t_compact.log
timeout -k 10 600 python -m pytest tests/test_executor_gpu.py tests/test_training_gpu.py -x -q > gpurun_out/t_exec.log 2>&1 || { tail -30 gpurun_out/t_exec.log; exit 1; }
tail -2 gpurun_out/t_exec.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_A1.log 2>&1 || exit 1
PDT_COMPACT_DS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_B1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_A2.log 2>&1 || exit 1
PDT_COMPACT_DS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_B2.log 2>&1 || exit 1
for f in A1 B1 A2 B2; do echo $f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$f.log); done
