set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6r
bash tools/gpu_round.sh r6r quick quickv:base || exit 1
cp gpurun_out/r6r/quick.json gpurun_out/r6r/quick_1.json; cp gpurun_out/r6r/quick_base.json gpurun_out/r6r/quick_base_1.json
bash tools/gpu_round.sh r6r quick quickv:base quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy" || exit 2
