set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6t
bash tools/gpu_round.sh r6t quick quickv:base quickv:shfl quickv:noinl quickv:oldtail || exit 1
mkdir -p gpurun_out/r6t/a && cp gpurun_out/r6t/quick*.json gpurun_out/r6t/a/
bash tools/gpu_round.sh r6t quickv:oldtail quickv:noinl quickv:shfl quickv:base quick || exit 2
