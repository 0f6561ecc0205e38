set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7p
bash tools/gpu_round.sh r7p quick quickv:base quicke:host_upload=0 || exit 1
mkdir -p gpurun_out/r7p/a && cp gpurun_out/r7p/quick*.json gpurun_out/r7p/a/
bash tools/gpu_round.sh r7p quicke:host_upload=0 quickv:base quick quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy or scan or stream or kernel_variants or batch" || exit 2
