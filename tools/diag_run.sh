set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 9000 --warmup 1 --batch-per-gpu 256 > gpurun_out/noise.log 2>&1 &
NOISE=$!
sleep 15
timeout -k 10 200 python -u tools/dgrad_bn_probe.py --reps 60 > gpurun_out/probe_fix.log 2>&1
echo "probe rc=$?"; grep -E "call (1|5|9):|slots" gpurun_out/probe_fix.log | head -8
kill $NOISE 2>/dev/null; wait $NOISE 2>/dev/null
timeout -k 10 400 python -u -m pytest tests/test_ddp_numerics_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ddpnum_fix.log 2>&1
echo "ddp numerics rc=$?"; tail -3 gpurun_out/ddpnum_fix.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_fix.log 2>&1
echo "bench rc=$?"; grep metric gpurun_out/bench_fix.log | cut -c1-200
echo done
