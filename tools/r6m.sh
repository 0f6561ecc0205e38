set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6m
bash tools/gpu_round.sh r6m quick quickv:base quicke:k5_split_merge=1 || exit 1
cp gpurun_out/r6m/quick.json gpurun_out/r6m/quick_1.json; cp gpurun_out/r6m/quick_base.json gpurun_out/r6m/quick_base_1.json; cp gpurun_out/r6m/quicke_k5_split_merge_1.json gpurun_out/r6m/split_1.json
bash tools/gpu_round.sh r6m quick quickv:base quicke:k5_split_merge=1 quick4 quick4v:base quick4e:k5_split_merge=1 "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy" || exit 2
