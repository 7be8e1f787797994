#!/bin/bash
# HBM traffic per kernel of a short bench run (run via gpurun): pass 1 FETCH_SIZE (3 TCC counters), pass 2
# WRITE_SIZE (2 TCC counters) -- separate passes because one pass holds at most 4 TCC counters.  Summarise with
# tools/pmc_bytes_summary.py.  BENCH_ARGS passes extra bench.py flags (e.g. "--arch resnet50 --dtype fp16").
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/${PMC_OUT:-pmc_bytes}"   # PMC_OUT: output directory name (A/B runs)
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  -d "$O/fetch" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS:-} \
  > "$O/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE GRBM_GUI_ACTIVE \
  -d "$O/write" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS:-} \
  > "$O/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "pmc bytes ok"
