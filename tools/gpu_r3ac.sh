# a chunk's sums / top-k / copies on a tail stream (beside the next chunk's pair kernel), exp/v/tail,
# A/B against the in-tree library; its correctness subset through the variant
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3ac && export TMPDIR=/tmp
T=$PWD/exp/v/tail/libpokec_fas.so
PF_LIB_PATH=$T timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "collab or recommenders or set_adj or pipelined or async or contexts or digests or holdout or gathers or variants" > gpurun_out/r3ac/gputest_sub.log 2>&1 || exit 1
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
PF_LIB_PATH=$T timeout -k 10 300 $B > gpurun_out/r3ac/cfg3_tail.json 2> gpurun_out/r3ac/cfg3_tail.err || exit 2
timeout -k 10 300 $B > gpurun_out/r3ac/cfg3.json 2> gpurun_out/r3ac/cfg3.err || exit 3
PF_LIB_PATH=$T timeout -k 10 300 $B > gpurun_out/r3ac/cfg3_tail_b.json 2> gpurun_out/r3ac/cfg3_tail_b.err || exit 4
timeout -k 10 300 $B > gpurun_out/r3ac/cfg3_b.json 2> gpurun_out/r3ac/cfg3_b.err || exit 5
C="python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc"
PF_LIB_PATH=$T timeout -k 10 600 $C > gpurun_out/r3ac/cfg5_c1_tail.json 2> gpurun_out/r3ac/cfg5_c1_tail.err || exit 6
timeout -k 10 600 $C > gpurun_out/r3ac/cfg5_c1.json 2> gpurun_out/r3ac/cfg5_c1.err || exit 7
