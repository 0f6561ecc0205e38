# round-5: K5 round-0 walk issued before the fixed terms, A/B against vlib/base (the previous commit)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6f
bash tools/gpu_round.sh r6f quick quickv:base || exit 1
cp gpurun_out/r6f/quick.json gpurun_out/r6f/quick_1.json; cp gpurun_out/r6f/quick_base.json gpurun_out/r6f/quick_base_1.json
bash tools/gpu_round.sh r6f quick quickv:base quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user" || exit 2
