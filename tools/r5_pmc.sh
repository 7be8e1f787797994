#!/bin/bash
# Round-5 end PMC record (run via gpurun): SQ timing, HBM bytes and instruction-mix passes (tools/pmc_round.sh) for
# ResNet-18 bf16 and ResNet-50 fp16 at B = 1200.  Summaries: tools/pmc_summary.py, tools/pmc_bytes_summary.py.
R="${GRAFT_REPO_ROOT:-/root/repo}"
echo "resnet18 passes"
PMC_OUT=r5_pmc18 bash "$R/tools/pmc_round.sh" || exit 1
echo "resnet50 passes"
PMC_OUT=r5_pmc50 BENCH_ARGS="--arch resnet50 --dtype fp16" bash "$R/tools/pmc_round.sh" || exit 1
echo "r5 pmc ok"
