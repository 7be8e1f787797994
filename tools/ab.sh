#!/bin/bash
# Same-box interleaved A/B on the 1-GPU bench (3 rounds of A then B; each run its own time limit).
#   bash tools/ab.sh env VAR A B [bench args...]   one environment knob, VAR=A vs VAR=B
#   bash tools/ab.sh so PATH [bench args...]       the in-tree _C.so vs another build (loaded via PDT_NATIVE_SO)
#   bash tools/ab.sh tree DIR [bench args...]      the in-tree bench.py vs DIR/bench.py (a whole other tree, e.g.
#                                                  `git archive` of a commit plus its built _C.so)
# Bench args default to "--steps 20 --warmup 5"; extra args are appended (e.g. --arch resnet50 --dtype fp16).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
MODE="$1"; shift
case "$MODE" in
  env) V="$1"; A="$2"; B="$3"; shift 3; EA="$V=$A"; EB="$V=$B" ;;
  so) EA="PDT_AB_ARM=in-tree"; EB="PDT_NATIVE_SO=$1"; shift ;;
  tree) EA="PDT_AB_ARM=in-tree"; EB="PDT_AB_ARM=$1"; TB="$1/bench.py"; shift ;;
  *) echo "usage: ab.sh env VAR A B [args] | ab.sh so PATH [args] | ab.sh tree DIR [args]"; exit 2 ;;
esac
TB="${TB:-bench.py}"
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | grep -o '[0-9.]*$'; }
for i in 1 2 3; do
  env "$EA" timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/ab_A$i.log 2>&1 || exit 1
  env "$EB" timeout -k 10 300 python "$TB" --steps 20 --warmup 5 "$@" > gpurun_out/ab_B$i.log 2>&1 || exit 1
  echo "A($EA) $(ms gpurun_out/ab_A$i.log)   B($EB) $(ms gpurun_out/ab_B$i.log)"
done
