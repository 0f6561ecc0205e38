# the default bench line (no flags: cfg2, 200 steps, CPU baseline + PMC) on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r8s
bash tools/gpu_round.sh r8s bench || exit 1
