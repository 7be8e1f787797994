set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py "tests/test_fp32_gpu.py::test_fp32_syncbn_native_comm_world1_equals_plain_bn" -x -v --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/repeat_check.py --replay --steps 2 > gpurun_out/replay.log 2>&1
rc=$?; echo "replay rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/repeat_check.py --reps 6 > gpurun_out/rep.log 2>&1
echo "rep rc=$?"
