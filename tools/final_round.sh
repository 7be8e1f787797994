cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_round.sh bench profserial prof && bash tools/r50_round.sh bench profserial && bash tools/gpu_round.sh reftable
