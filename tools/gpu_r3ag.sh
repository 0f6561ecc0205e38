# pair epilogue in two queue rounds (no per-lane fallback for waves with 321..640 items) vs
# exp/v/oneround; GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ag && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3ag/gputest.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
O=$PWD/exp/v/oneround/libpokec_fas.so
timeout -k 10 300 $B > gpurun_out/r3ag/cfg3_two.json 2> gpurun_out/r3ag/cfg3_two.err || exit 2
PF_LIB_PATH=$O timeout -k 10 300 $B > gpurun_out/r3ag/cfg3_one.json 2> gpurun_out/r3ag/cfg3_one.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3ag/cfg3_two_b.json 2> gpurun_out/r3ag/cfg3_two_b.err || exit 4
PF_LIB_PATH=$O timeout -k 10 300 $B > gpurun_out/r3ag/cfg3_one_b.json 2> gpurun_out/r3ag/cfg3_one_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3ag/cfg5_c1_two.json 2> gpurun_out/r3ag/cfg5_c1_two.err || exit 6
PF_LIB_PATH=$O timeout -k 10 600 $C > gpurun_out/r3ag/cfg5_c1_one.json 2> gpurun_out/r3ag/cfg5_c1_one.err || exit 7
