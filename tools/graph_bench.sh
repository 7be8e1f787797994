cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for bs in 32 128; do
  timeout -k 10 300 python bench.py --batch-per-gpu $bs --steps 50 --warmup 5 > gpurun_out/g_e$bs.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --batch-per-gpu $bs --steps 50 --warmup 5 --graph > gpurun_out/g_g$bs.log 2>&1 || exit 1
done
grep -h metric gpurun_out/g_*.log | cut -c1-200
