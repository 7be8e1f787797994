#!/bin/bash
# Same-box kernel times of the layer1 weight-gradient forms: PDT_WGRAD_L1_W8 = 1 (column split) vs 2 (tap split)
R="${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for m in 1 2 1 2; do
  PDT_WGRAD_L1_W8=$m PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/w8p_$m" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/w8p_$m.log" 2>&1 || exit 1
  python3 - "$R/gpurun_out/w8p_$m/run_kernel_stats.csv" $m <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "wgrad3x3" in r["Name"] or "wgrad_reduce" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], "%.1f us/call" % (float(r["AverageNs"]) / 1e3))
PY
done
