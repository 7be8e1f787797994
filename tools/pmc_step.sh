#!/bin/bash
# PMC counters (MFMA busy, wait/issue stall split, LDS conflicts) for every kernel of a short bench run
# (run via gpurun).  One pass: 8 SQ counters + GRBM_GUI_ACTIVE.  Summarise with tools/pmc_summary.py.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out/pmc_step"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc_step/run" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS:-} \
  > "$R/gpurun_out/pmc_step/run.log" 2>&1
echo "rc=$?"
