# round-5: K5 run-length term items A/B (vlib/base = the previous commit), then the K5 tests
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6e
bash tools/gpu_round.sh r6e quick quickv:base || exit 1
cp gpurun_out/r6e/quick.json gpurun_out/r6e/quick_1.json; cp gpurun_out/r6e/quick_base.json gpurun_out/r6e/quick_base_1.json
bash tools/gpu_round.sh r6e quick quickv:base quick4 quick4v:base "tests:all_candidates or full_size or big or postings or variants or every_user" || exit 2
