set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7w
bash tools/gpu_round.sh r7w quick quickv:pprio || exit 1
mkdir -p gpurun_out/r7w/a && cp gpurun_out/r7w/quick*.json gpurun_out/r7w/a/
bash tools/gpu_round.sh r7w quickv:pprio quick quick4 quick4v:pprio || exit 2
