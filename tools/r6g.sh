# round-5: K5 finer tail blocks (PF_DEBUG k5_tail=N; default 128) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6g
bash tools/gpu_round.sh r6g quick quicke:k5_tail=0 quicke:k5_tail=256 quicke:k5_tail=64 || exit 1
cp gpurun_out/r6g/quick.json gpurun_out/r6g/quick_1.json
bash tools/gpu_round.sh r6g quicke:k5_tail=0 quick "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded" || exit 2
