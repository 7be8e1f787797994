#!/bin/bash
# PMC counters for the generic conv kernels on one layer shape (run via gpurun); SHAPES selects
# tools/conv_bench.py shape indices.  One pass: 8 SQ counters + GRBM_GUI_ACTIVE.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc2"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc2/run" -o run -- python3 "$R/tools/conv_bench.py" --skip-stem --shapes ${SHAPES:-5} --reps 2 \
  > "$R/gpurun_out/pmc2/run.log" 2>&1
echo "rc=$?"
