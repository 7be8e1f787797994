set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/eval_cost.py > gpurun_out/eval_cost.log 2>&1 || { tail -5 gpurun_out/eval_cost.log; exit 1; }
tail -1 gpurun_out/eval_cost.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp16 --steps 20 --warmup 5 > gpurun_out/sb_off$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --dtype fp16 --steps 20 --warmup 5 --sync-bn --force-comm > gpurun_out/sb_on$i.log 2>&1 || exit 1
  echo "fp16 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sb_off$i.log)  fp16+SyncBN(forced comm) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sb_on$i.log)"
done
PDT_SYNCBN_COMM=shared timeout -k 10 300 python bench.py --dtype fp16 --steps 20 --warmup 5 --sync-bn --force-comm > gpurun_out/sb_shared.log 2>&1 || exit 1
echo "fp16+SyncBN shared comm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sb_shared.log)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; exit $rc
