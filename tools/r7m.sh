set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7m
bash tools/gpu_round.sh r7m quick quickv:nomerge quick quickv:nomerge || exit 1
