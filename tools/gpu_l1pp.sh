cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "pingpong or layer1 or fused_bn_backward or producer" --timeout 120 --timeout-method thread > gpurun_out/t_l1pp.log 2>&1; rc=$?; tail -5 gpurun_out/t_l1pp.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
PDT_CONV_L1_PP=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_pp_$i.log 2>&1 || exit $?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_pp_$i.log
PDT_CONV_L1_PP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_old_$i.log 2>&1 || exit $?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_old_$i.log
done
cd /tmp && export TMPDIR=/tmp
PDT_CONV_L1_PP=1 PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 5 --warmup 2 > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/profs.log" 2>&1 || exit $?
echo PROF_OK
