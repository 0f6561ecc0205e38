set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7v
bash tools/gpu_round.sh r7v quick quickv:base || exit 1
mkdir -p gpurun_out/r7v/a && cp gpurun_out/r7v/quick*.json gpurun_out/r7v/a/
bash tools/gpu_round.sh r7v quickv:base quick quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy or scan or stream or kernel_variants" || exit 2
