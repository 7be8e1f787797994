cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/conv_bench.py --skip-stem --shapes 1,2,3 --stats --reps 5 > gpurun_out/cb_stats.log 2>&1 || exit $?
grep shape gpurun_out/cb_stats.log | cut -c1-400
REPS=2 bash tools/gpu_bench_ab.sh "PDT_WGRAD_STREAM=0 PDT_WGRAD_L1_PIPE=1" "PDT_WGRAD_STREAM=0 PDT_WGRAD_L1_PIPE=0" "PDT_WGRAD_L1_PIPE=1" "PDT_WGRAD_L1_PIPE=0"
