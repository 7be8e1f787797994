cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for i in 1 2; do
  PDT_TUNED_TILES=0 timeout -k 10 300 python bench.py --batch-per-gpu 150 --steps 40 --warmup 5 > gpurun_out/c150a_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --batch-per-gpu 150 --steps 40 --warmup 5 > gpurun_out/c150b_$i.log 2>&1 || exit $?
  echo "B150 static $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c150a_$i.log) tuned $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c150b_$i.log)"
done
timeout -k 10 300 python bench.py --batch-per-gpu 400 --steps 30 --warmup 5 > gpurun_out/c400.log 2>&1 || exit $?
echo "B400 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c400.log)"
