# kHitCap 24 (exp/v/hc24) vs the in-tree 20; alternating
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ak && export TMPDIR=/tmp
H=$PWD/exp/v/hc24/libpokec_fas.so
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
PF_LIB_PATH=$H timeout -k 10 300 $B > gpurun_out/r3ak/cfg3_hc24.json 2> gpurun_out/r3ak/cfg3_hc24.err || exit 1
timeout -k 10 300 $B > gpurun_out/r3ak/cfg3_hc20.json 2> gpurun_out/r3ak/cfg3_hc20.err || exit 2
PF_LIB_PATH=$H timeout -k 10 300 $B > gpurun_out/r3ak/cfg3_hc24_b.json 2> gpurun_out/r3ak/cfg3_hc24_b.err || exit 3
timeout -k 10 300 $B > gpurun_out/r3ak/cfg3_hc20_b.json 2> gpurun_out/r3ak/cfg3_hc20_b.err || exit 4
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
timeout -k 10 600 $C > gpurun_out/r3ak/cfg5_c1_hc20.json 2> gpurun_out/r3ak/cfg5_c1_hc20.err || exit 5
PF_LIB_PATH=$H timeout -k 10 600 $C > gpurun_out/r3ak/cfg5_c1_hc24.json 2> gpurun_out/r3ak/cfg5_c1_hc24.err || exit 6
timeout -k 10 600 $C > gpurun_out/r3ak/cfg5_c1_hc20_b.json 2> gpurun_out/r3ak/cfg5_c1_hc20_b.err || exit 7
PF_LIB_PATH=$H timeout -k 10 600 $C > gpurun_out/r3ak/cfg5_c1_hc24_b.json 2> gpurun_out/r3ak/cfg5_c1_hc24_b.err || exit 8
