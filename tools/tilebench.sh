#!/bin/bash
# conv tile sweep with the default ring depth and with 3-stage rings forced (run via gpurun)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/conv_bench.py --skip-stem --shapes 1,2,4,5,7,8 > gpurun_out/tile2.log 2>&1 || exit 1
PDT_FWD_STAGES=3 timeout -k 10 600 python tools/conv_bench.py --skip-stem --shapes 2,5,8 > gpurun_out/tile3.log 2>&1 || exit 1
