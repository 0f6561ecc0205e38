# round-3 final lines: the driver's default N=1 run, then cfg3 / cfg4 / cfg5 lines, each with its
# CPU baseline and PMC pass (bench.py does both by default)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3q && export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/r3q/bench.json 2> gpurun_out/r3q/bench.err || exit 1
timeout -k 10 600 python3 bench.py --workload cfg3 > gpurun_out/r3q/cfg3.json 2> gpurun_out/r3q/cfg3.err || exit 2
timeout -k 10 600 python3 bench.py --workload cfg4 > gpurun_out/r3q/cfg4.json 2> gpurun_out/r3q/cfg4.err || exit 3
timeout -k 10 900 python3 bench.py --workload cfg5 > gpurun_out/r3q/cfg5.json 2> gpurun_out/r3q/cfg5.err || exit 4
