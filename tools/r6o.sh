# round-5 tree: GPU suite, the default bench line (CPU baseline + PMC), rocprof stats, cfg 3/4/5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6o
bash tools/gpu_round.sh r6o tests bench prof cfg3 cfg4 cfg5 || exit 1
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --solo-shards 8 > gpurun_out/r6o/cfg4_solo.json 2> gpurun_out/r6o/cfg4_solo.err || exit 2
