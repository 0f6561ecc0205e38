set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7r
bash tools/gpu_round.sh r7r quick quickv:rcap7 quickv:rcap8 || exit 1
mkdir -p gpurun_out/r7r/a && cp gpurun_out/r7r/quick*.json gpurun_out/r7r/a/
bash tools/gpu_round.sh r7r quickv:rcap8 quickv:rcap7 quick quick4 quick4v:rcap7 quick4v:rcap8 || exit 2
