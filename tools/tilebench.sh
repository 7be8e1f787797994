#!/bin/bash
# conv tile sweep (run via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python tools/conv_bench.py --skip-stem --shapes ${SHAPES:-1,2,4,5,7,8} > gpurun_out/tile2.log 2>&1 || exit 1
