# round-5 closing GPU pass: full GPU test suite, smoke, R18 bench x2, R50 bench, R18 serial profile
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_round.sh test || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/b18_$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/b18_$i.log
done
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --arch resnet50 --dtype fp16 > gpurun_out/b50_final.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b50_final.log
cd /tmp && export TMPDIR=/tmp
PDT_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof18" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof18.log" 2>&1 || exit 1
echo ALL DONE
