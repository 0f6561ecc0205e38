set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7j
bash tools/gpu_round.sh r7j quick quickv:base || exit 1
mkdir -p gpurun_out/r7j/a && cp gpurun_out/r7j/quick*.json gpurun_out/r7j/a/
bash tools/gpu_round.sh r7j quickv:base quick quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy" || exit 2
