cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_l1on.log 2>&1 || exit 1
PDT_CONV_L1=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_l1off.log 2>&1 || exit 1
bash tools/gpu_round.sh prof
