# K1' epilogue: item-queue fallback counters (K5T build), a larger item queue (PF_QUEUE_EXTRA=8),
# the item loop's norm prefetch (pf); in-tree = neither
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3x && export TMPDIR=/tmp
B="python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc"
V=$PWD/exp/v
timeout -k 10 300 $B > gpurun_out/r3x/cfg3.json 2> gpurun_out/r3x/cfg3.err || exit 1
PF_LIB_PATH=$V/k5t/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_k5t.json 2> gpurun_out/r3x/cfg3_k5t.err || exit 2
PF_LIB_PATH=$V/q8/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_q8.json 2> gpurun_out/r3x/cfg3_q8.err || exit 3
PF_LIB_PATH=$V/pf/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_pf.json 2> gpurun_out/r3x/cfg3_pf.err || exit 4
PF_LIB_PATH=$V/pfq8/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_pfq8.json 2> gpurun_out/r3x/cfg3_pfq8.err || exit 5
PF_LIB_PATH=$V/q8k5t/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_q8k5t.json 2> gpurun_out/r3x/cfg3_q8k5t.err || exit 6
timeout -k 10 300 $B > gpurun_out/r3x/cfg3_b.json 2> gpurun_out/r3x/cfg3_b.err || exit 7
PF_LIB_PATH=$V/pfq8/libpokec_fas.so timeout -k 10 300 $B > gpurun_out/r3x/cfg3_pfq8_b.json 2> gpurun_out/r3x/cfg3_pfq8_b.err || exit 8
PF_LIB_PATH=$V/k5t/libpokec_fas.so PF_DEBUG=union=1 timeout -k 10 300 $B > gpurun_out/r3x/cfg3_union_k5t.json 2> gpurun_out/r3x/cfg3_union_k5t.err || exit 9
