cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/abg_e$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph > gpurun_out/abg_g$r.log 2>&1 || exit 1
done
for f in gpurun_out/abg_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
