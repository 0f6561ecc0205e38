# round-6 tree, part B: cfg 3/4/5 lines, cfg-4 solo shards, K5 counter passes
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r7y
bash tools/gpu_round.sh r7y cfg3 cfg4 cfg5 || exit 1
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --solo-shards 8 > gpurun_out/r7y/cfg4_solo.json 2> gpurun_out/r7y/cfg4_solo.err || exit 2
TAG=r7y bash tools/gpu_round.sh r7y pmcpasses:fas_post_kernel || exit 3
