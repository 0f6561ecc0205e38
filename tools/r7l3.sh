# the default bench line with the scan lanes (CPU baseline + PMC), twice, and rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7l3
bash tools/gpu_round.sh r7l3 bench prof || exit 1
