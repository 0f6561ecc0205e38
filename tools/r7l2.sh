set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7l2
bash tools/gpu_round.sh r7l2 quick quicke:scan_lanes=0 || exit 1
mkdir -p gpurun_out/r7l2/a && cp gpurun_out/r7l2/quick*.json gpurun_out/r7l2/a/
bash tools/gpu_round.sh r7l2 quicke:scan_lanes=0 quick tests || exit 2
