set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6u
bash tools/gpu_round.sh r6u quickv:mdbg > gpurun_out/r6u/mdbg.log 2>&1 || exit 1
bash tools/gpu_round.sh r6u quick quickv:base quickv:oldtail quick quickv:base quickv:oldtail quick4 quick4v:oldtail || exit 2
