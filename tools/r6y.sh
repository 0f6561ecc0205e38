set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6y
bash tools/gpu_round.sh r6y quickv:base quickv:prefA quickv:prefB || exit 1
mkdir -p gpurun_out/r6y/a && cp gpurun_out/r6y/quick*.json gpurun_out/r6y/a/
bash tools/gpu_round.sh r6y quickv:prefB quickv:prefA quickv:base quick4v:base quick4v:prefA quick4v:prefB || exit 2
