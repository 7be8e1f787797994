#!/bin/bash
# All PMC passes of one round's "before/after" record (run via gpurun): SQ timing counters (tools/pmc_step.sh),
# HBM bytes (tools/pmc_bytes.sh) and an instruction-mix / L2-hit pass.  Each pass its own process and time limit.
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/${PMC_OUT:-pmc_round}"
mkdir -p "$O"
bash "$R/tools/pmc_step.sh" || exit 1
rm -rf "$O/sq" && mv "$R/gpurun_out/pmc_step" "$O/sq"
PMC_OUT="${PMC_OUT:-pmc_round}/bytes" bash "$R/tools/pmc_bytes.sh" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  -d "$O/mix" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$O/mix.log" 2>&1
echo "mix rc=$?"
