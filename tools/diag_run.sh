# Replay-determinism check (every native op re-run 4x from a snapshot) while a second process keeps the GPU busy
# with full training steps, so each replayed kernel runs with other kernels competing for CUs (timing-dependent
# intra-kernel races need that); then a plain repeatability run against the same noise.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 4000 --warmup 1 --batch-per-gpu 256 > gpurun_out/noise.log 2>&1 &
NOISE=$!
sleep 20
PDT_VALIDATE_REPLAYS=4 timeout -k 10 300 python -u tools/repeat_check.py --replay --steps 2 > gpurun_out/replay_noise.log 2>&1
echo "replay rc=$?"; tail -6 gpurun_out/replay_noise.log
timeout -k 10 300 python -u tools/repeat_check.py --reps 5 > gpurun_out/repeat_noise.log 2>&1
echo "repeat rc=$?"; tail -6 gpurun_out/repeat_noise.log
kill $NOISE 2>/dev/null; wait $NOISE 2>/dev/null
echo done
