# final tree: full GPU suite, the default bench line (CPU baseline + PMC) and rocprof stats,
# cfg 4 / cfg 5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r8k
bash tools/gpu_round.sh r8k tests bench prof || exit 1
timeout -k 10 300 python3 bench.py --workload cfg4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/r8k/cfg4.json 2> gpurun_out/r8k/cfg4.err || exit 2
timeout -k 10 300 python3 bench.py --workload cfg5 --no-pmc --no-cpu-baseline > gpurun_out/r8k/cfg5.json 2> gpurun_out/r8k/cfg5.err || exit 3
