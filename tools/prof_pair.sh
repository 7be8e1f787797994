#!/bin/bash
# Serial (one-stream) kernel traces of the 1-GPU bench under two settings of one env knob:
#   bash tools/prof_pair.sh VAR VALUE_A VALUE_B [bench args...]   -> gpurun_out/pp_A, gpurun_out/pp_B
R="${GRAFT_REPO_ROOT:-/root/repo}"; V="$1"; A="$2"; B="$3"; shift 3
cd /tmp && export TMPDIR=/tmp
for tag in A B; do
  val=$A; [ $tag = B ] && val=$B
  env "$V=$val" PDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/pp_$tag" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 "$@" > "$R/gpurun_out/pp_$tag.log" 2>&1 || exit $?
done
echo "prof_pair done"
