#!/bin/bash
# PMC counters for the layer1 conv / wgrad kernels (run on the GPU box via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$R/gpurun_out/pmc/avail.txt" 2>&1
grep -iE "LDS|MFMA|VALU_BUSY|BUSY_CYCLES|WAIT_INST" "$R/gpurun_out/pmc/avail.txt" | head -60 > "$R/gpurun_out/pmc/avail_grep.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d "$R/gpurun_out/pmc/run1" -o run -- python3 "$R/tools/conv_bench.py" --skip-stem --shapes 0 --reps 2 > "$R/gpurun_out/pmc/run1.log" 2>&1
rc=$?
echo "rc=$rc"
exit $rc
