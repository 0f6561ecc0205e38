set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7d
bash tools/gpu_round.sh r7d quick quickv:prioup || exit 1
mkdir -p gpurun_out/r7d/a && cp gpurun_out/r7d/quick*.json gpurun_out/r7d/a/
bash tools/gpu_round.sh r7d quickv:prioup quick quick4 quick4v:prioup || exit 2
