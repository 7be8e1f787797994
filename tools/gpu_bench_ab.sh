#!/bin/bash
# Interleaved same-box bench A/B over settings given as arguments: "ENV=1 ENV2=0" strings, optionally followed by
# " :: <extra bench.py args>"; $REPS rounds, $STEPS timed steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for i in $(seq 1 ${REPS:-2}); do
  for cfg in "$@"; do
    envs="${cfg%%::*}"; args=""
    [[ "$cfg" == *"::"* ]] && args="${cfg#*::}"
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} $args > gpurun_out/b_ab.log 2>&1 || { tail -5 gpurun_out/b_ab.log; exit 1; }
    echo "$cfg: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_ab.log)"
  done
done
