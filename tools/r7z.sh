# round-6 tree, part A: GPU suite, the default bench line (CPU baseline + PMC), rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7z
bash tools/gpu_round.sh r7z tests bench prof || exit 1
