#!/bin/bash
# PMC counter passes over a short serial bench run, summarised for the kernels whose name matches a filter:
#   bash tools/pmc_kernel.sh FILTER "CTR CTR ..." ["CTR ..."]...     (one rocprofv3 process per counter set)
# -> gpurun_out/pmck/<i>/run_counter_collection.csv and a summary in gpurun_out/pmck/summary.txt
R="${GRAFT_REPO_ROOT:-/root/repo}"; F="$1"; shift
mkdir -p "$R/gpurun_out/pmck"; : > "$R/gpurun_out/pmck/summary.txt"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  PDT_WGRAD_STREAM=0 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $set \
    -d "$R/gpurun_out/pmck/$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 ${BENCH_ARGS:-} \
    > "$R/gpurun_out/pmck/$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  python3 "$R/tools/pmc_kernel_summary.py" "$R/gpurun_out/pmck/$i" "$F" >> "$R/gpurun_out/pmck/summary.txt"
done
cat "$R/gpurun_out/pmck/summary.txt"
