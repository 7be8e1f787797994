set -u
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 400 python -u -m pytest "$@" -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bis_$name.log 2>&1; rc=$?; echo "$name rc=$rc $(tail -1 gpurun_out/bis_$name.log)"; [ $rc -le 1 ] || exit $rc; }
run A tests/test_ddp_numerics_gpu.py -k "averaged or seeded"
run B tests/test_comm_gpu.py tests/test_ddp_numerics_gpu.py -k "averaged or seeded or graphed or watchdog or bucketer or rccl or device_group or tcp_store"
run C tests/test_comm_gpu.py tests/test_ddp_numerics_gpu.py -k "graphed or averaged or seeded"
run D tests/test_comm_gpu.py tests/test_ddp_numerics_gpu.py -k "watchdog or averaged or seeded"
