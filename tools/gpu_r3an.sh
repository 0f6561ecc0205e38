# final-code cfg5 / cfg4 lines (CPU baseline + PMC pass each)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3an && export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py --workload cfg5 > gpurun_out/r3an/cfg5.json 2> gpurun_out/r3an/cfg5.err || exit 1
timeout -k 10 600 python3 bench.py --workload cfg4 > gpurun_out/r3an/cfg4.json 2> gpurun_out/r3an/cfg4.err || exit 2
