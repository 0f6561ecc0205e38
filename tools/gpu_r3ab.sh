# K3 gathers started early on the aux stream (beside the previous call's pair kernel): A/B vs the
# in-call fork (exp/v/late), correctness subset
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ab && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or set_adj or pipelined or async or contexts or digests or holdout or gathers" > gpurun_out/r3ab/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
L=$PWD/exp/v/late/libpokec_fas.so
timeout -k 10 300 $B > gpurun_out/r3ab/cfg3.json 2> gpurun_out/r3ab/cfg3.err || exit 2
PF_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/r3ab/cfg3_late.json 2> gpurun_out/r3ab/cfg3_late.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3ab/cfg3_b.json 2> gpurun_out/r3ab/cfg3_b.err || exit 4
PF_LIB_PATH=$L timeout -k 10 300 $B > gpurun_out/r3ab/cfg3_late_b.json 2> gpurun_out/r3ab/cfg3_late_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3ab/cfg5_c1.json 2> gpurun_out/r3ab/cfg5_c1.err || exit 6
PF_LIB_PATH=$L timeout -k 10 600 $C > gpurun_out/r3ab/cfg5_c1_late.json 2> gpurun_out/r3ab/cfg5_c1_late.err || exit 7
