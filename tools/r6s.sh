set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6s
timeout -k 10 60 ./tools/probe/lane_xor > gpurun_out/r6s/probe.txt 2>&1 || { cat gpurun_out/r6s/probe.txt; exit 3; }
cat gpurun_out/r6s/probe.txt
bash tools/gpu_round.sh r6s quick quickv:base || exit 1
cp gpurun_out/r6s/quick.json gpurun_out/r6s/quick_1.json; cp gpurun_out/r6s/quick_base.json gpurun_out/r6s/quick_base_1.json
bash tools/gpu_round.sh r6s quick quickv:base quick4 quick4v:base "tests:all_candidates or full_size_kernels or big_top64 or every_user or sharded or wide_sets or heavy or scan or stream" || exit 2
