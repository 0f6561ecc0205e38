# kHitCap 20 (exp/v/hc20: fewer overflowed pairs, a 384-item queue) vs the in-tree 16; alternating
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ai && export TMPDIR=/tmp
H=$PWD/exp/v/hc20/libpokec_fas.so
PF_LIB_PATH=$H timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or big_pairs or hub or async or digests" > gpurun_out/r3ai/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
PF_LIB_PATH=$H timeout -k 10 300 $B > gpurun_out/r3ai/cfg3_hc20.json 2> gpurun_out/r3ai/cfg3_hc20.err || exit 2
timeout -k 10 300 $B > gpurun_out/r3ai/cfg3_hc16.json 2> gpurun_out/r3ai/cfg3_hc16.err || exit 3
PF_LIB_PATH=$H timeout -k 10 300 $B > gpurun_out/r3ai/cfg3_hc20_b.json 2> gpurun_out/r3ai/cfg3_hc20_b.err || exit 4
timeout -k 10 300 $B > gpurun_out/r3ai/cfg3_hc16_b.json 2> gpurun_out/r3ai/cfg3_hc16_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3ai/cfg5_c1_hc16.json 2> gpurun_out/r3ai/cfg5_c1_hc16.err || exit 6
PF_LIB_PATH=$H timeout -k 10 600 $C > gpurun_out/r3ai/cfg5_c1_hc20.json 2> gpurun_out/r3ai/cfg5_c1_hc20.err || exit 7
timeout -k 10 600 $C > gpurun_out/r3ai/cfg5_c1_hc16_b.json 2> gpurun_out/r3ai/cfg5_c1_hc16_b.err || exit 8
PF_LIB_PATH=$H timeout -k 10 600 $C > gpurun_out/r3ai/cfg5_c1_hc20_b.json 2> gpurun_out/r3ai/cfg5_c1_hc20_b.err || exit 9
