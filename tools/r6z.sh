set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6z
bash tools/gpu_round.sh r6z quick quickv:base || exit 1
mkdir -p gpurun_out/r6z/a && cp gpurun_out/r6z/quick*.json gpurun_out/r6z/a/
bash tools/gpu_round.sh r6z quickv:base quick quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy" || exit 2
